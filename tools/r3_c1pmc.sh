set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
i=0
for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE SQ_INSTS_VALU" "SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d $PWD/gpurun_out/c1pmc/p$i -o run -- python tools/enc_trace.py > gpurun_out/c1pmc_p$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/c1pmc_p$i.log; exit 2; }
done
python - <<'PY'
import csv, glob, collections
for kern in ('conv2d_c1_kernel', 'gemm_kernel<64, 64, 32, 0, 6'):
    acc = collections.defaultdict(list)
    for f in glob.glob('gpurun_out/c1pmc/p*/run_counter_collection.csv'):
        for r in csv.DictReader(open(f)):
            if kern in r['Kernel_Name']:
                acc[r['Counter_Name']].append(float(r['Counter_Value']))
    print(kern)
    for k, v in sorted(acc.items()):
        print(f'  {k:26s} n={len(v):3d} avg={sum(v)/len(v):14.1f}')
PY
