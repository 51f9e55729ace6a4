#!/bin/bash
# Per-variant GEMM kernel profile: for each "SHAPE|env" the average gemm_kernel duration
# (rocprofv3 --kernel-trace --stats) and one SQ counter pass (wave cycles split into
# active / issue-stall / wait, MFMA busy).   tools/gemm_variants.sh TAG "M,N,K|ENV=.." ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd); TAG=$1; shift
OUT=gpurun_out/gv_$TAG; mkdir -p $OUT; export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i+1))
  SHAPE=${v%%|*}; ENVS=${v#*|}; [ "$ENVS" = "$v" ] && ENVS=""
  env $ENVS NOGRAPH=1 timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/$OUT/t$i -o run -- python tools/gemm_bench.py $SHAPE > $OUT/t$i.log 2>&1 || { echo "trace $i failed"; tail -5 $OUT/t$i.log; exit 2; }
  env $ENVS NOGRAPH=1 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $REPO/$OUT/p$i -o run -- python tools/gemm_bench.py $SHAPE > $OUT/p$i.log 2>&1 || { echo "pmc $i failed"; tail -5 $OUT/p$i.log; exit 3; }
  python - "$OUT" "$i" "$v" <<'PY'
import csv, glob, sys, collections
out, i, v = sys.argv[1], sys.argv[2], sys.argv[3]
dur = [float(r['End_Timestamp']) - float(r['Start_Timestamp'])
       for f in glob.glob(f'{out}/t{i}/run_kernel_trace.csv') for r in csv.DictReader(open(f))
       if 'gemm_kernel' in r['Kernel_Name']]
acc = collections.defaultdict(list)
names = set()
for f in glob.glob(f'{out}/p{i}/run_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        if 'gemm_kernel' in r['Kernel_Name']:
            acc[r['Counter_Name']].append(float(r['Counter_Value']))
            names.add(r['Kernel_Name'][:60])
a = {k: sum(x) / len(x) for k, x in acc.items()}
us = sorted(dur)[len(dur) // 2] / 1e3 if dur else 0
W = a.get('SQ_WAVES', 1)
wc = a.get('SQ_WAVE_CYCLES', 0) * 4 / W
kern = a.get('GRBM_GUI_ACTIVE', 0) / 8
print(f'[{v}] {names}\n  median {us:.1f} us over {len(dur)}; kernel {kern:.0f} cyc; waves {W:.0f}; per wave {wc:.0f} cyc '
      f'(active {a.get("SQ_ACTIVE_INST_ANY",0)*4/W/max(wc,1):.2f}, issue-stall {a.get("SQ_WAIT_INST_ANY",0)*4/W/max(wc,1):.2f}, '
      f'wait {a.get("SQ_WAIT_ANY",0)*4/W/max(wc,1):.2f}); MFMA busy {a.get("SQ_VALU_MFMA_BUSY_CYCLES",0)/1024/max(kern,1):.2f} of kernel', flush=True)
PY
done
