#!/bin/bash
# SQ counters for selected ops (tools/op_bench.py filter), one PMC pass, no tracing domains.
#   tools/pmc_ops.sh TAG FILTER
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc ${PMC_SET:-SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES} \
  --output-format csv -d $REPO/gpurun_out/pmcops_$1 -o run -- python $REPO/tools/op_bench.py "$2" > gpurun_out/pmcops_$1.log 2>&1
rc=$?
python - "$REPO/gpurun_out/pmcops_$1" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name'].split('(')[0][:70]
    agg[k][r['Counter_Name']] += float(r['Counter_Value'])
    n[(k, r['Counter_Name'])] += 1
for k, d in agg.items():
    disp = max(n[(k, c)] for c in d)
    print(k, 'dispatches', disp)
    print('   ' + '  '.join(f'{c}={v / disp:.3g}' for c, v in sorted(d.items())))
PY
exit $rc
