#!/bin/bash
# A/B of an environment toggle on the default bench, alternating runs:  tools/ab_bench.sh VAR
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VAR=$1
for r in 1 2 3; do
  for v in 1 0; do
    env $VAR=$v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --warmup 10 > gpurun_out/ab.log 2>&1 || exit 4
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" "$VAR=$v"
  done
done
