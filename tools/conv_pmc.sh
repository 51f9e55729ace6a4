# SQ / TA / TCC counters of the decoder tap conv at B (tools/conv_one.py), one pass per group
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd); B=$1; CI=$2
OUT=gpurun_out/cpmc_$B; mkdir -p $OUT; export TMPDIR=/tmp
i=0
for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
            "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_MFMA" \
            "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TCP_TCC_READ_REQ_sum SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM" ; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d $REPO/$OUT/p$i -o run -- python tools/conv_one.py $B $CI 10 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 2; }
done
python - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(list)
for f in glob.glob(f'{out}/p*/run_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        if 'gemm_kernel' in r['Kernel_Name']:
            acc[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in sorted(acc.items()):
    print(f'{k:28s} n={len(v):3d} avg={sum(v)/len(v):14.1f}')
PY
