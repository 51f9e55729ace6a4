#!/bin/bash
# Per-kernel SQ counters for any python command, one PMC pass per counter set (sets separated
# by ';' in PMC_SETS), no tracing domains.   tools/pmc_cmd.sh TAG FILTER python-args...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; FILTER=$2; shift 2
IFS=';' read -ra SETS <<< "${PMC_SETS:-SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE;SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_SALU}"
i=0
for set in "${SETS[@]}"; do
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $REPO/gpurun_out/pmc_${TAG}_$i -o run -- python "$@" > gpurun_out/pmc_${TAG}_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/pmc_${TAG}_$i.log; exit 3; }
  python - "$REPO/gpurun_out/pmc_${TAG}_$i" "$FILTER" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name'].split('(')[0][:70]
    if sys.argv[2] not in k:
        continue
    agg[k][r['Counter_Name']] += float(r['Counter_Value'])
    n[(k, r['Counter_Name'])] += 1
for k, d in agg.items():
    disp = max(n[(k, c)] for c in d)
    print(k, 'dispatches', disp)
    print('   ' + '  '.join(f'{c}={v / disp:.4g}' for c, v in sorted(d.items())))
PY
  find gpurun_out/pmc_${TAG}_$i -name "*counter_collection.csv" -size +20M -delete
  i=$((i+1))
done
exit 0
