#!/bin/bash
# SQ counters of the fused graph stack (tools/stack_bench.py hand), two PMC passes.
#   tools/stack_pmc.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=gpurun_out/stackpmc_$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python tools/stack_bench.py both 20 > $OUT/time.txt 2>&1 || exit 2
cat $OUT/time.txt
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $REPO/$OUT/p$i -o run -- python tools/stack_bench.py hand 3 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $OUT/p$i.log; exit 3; }
done
python - $OUT <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(sys.argv[1] + '/p*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'graph_stack' not in r['Kernel_Name']:
            continue
        agg[r['Counter_Name']] += float(r['Counter_Value']); n[r['Counter_Name']] += 1
for c in sorted(agg):
    print(f'{c:28s} {agg[c] / n[c]:.4g}')
PY
