#!/bin/bash
# GEMM block -> XCD grouping (A2M_GEMM_XCD) A/B: HBM fetch per GEMM launch over exactly the bench
# step (one FETCH_SIZE pass each) and the bench step time.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
for g in 0 2 4 8; do
  A2M_GEMM_XCD=$g timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $REPO/gpurun_out/xcd_f$g -o run -- python tools/step_pmc.py 3 > gpurun_out/xcd_f$g.log 2>&1 || { echo "pmc $g failed"; exit 2; }
  A2M_GEMM_XCD=$g timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $REPO/gpurun_out/xcd_w$g -o run -- python tools/step_pmc.py 3 > gpurun_out/xcd_w$g.log 2>&1 || { echo "pmc $g failed"; exit 2; }
  python tools/pmc_traffic.py gpurun_out/xcd_f$g gpurun_out/xcd_w$g --out gpurun_out/xcd_traffic$g.json --tag "xcd $g" > /dev/null || exit 3
  A2M_GEMM_XCD=$g timeout -k 10 200 python bench.py --no-cpu-baseline --steps 50 > gpurun_out/xcd_b$g.log 2>&1 || exit 4
  python - $g <<'PY'
import json, sys
g = sys.argv[1]
t = json.load(open(f'gpurun_out/xcd_traffic{g}.json'))
b = json.loads(open(f'gpurun_out/xcd_b{g}.log').read().strip().splitlines()[-1])
print(f"xcd {g}: step {b['ms_per_step']} ms, gemm {t['gemm_kernel']['bytes_per_launch'] / 1e6:.1f} MB/launch, "
      f"gemm frac {b['roofline']['frac']}")
PY
  find gpurun_out/xcd_f$g gpurun_out/xcd_w$g -name "*counter_collection.csv" -size +20M -delete
done
