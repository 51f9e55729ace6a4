#!/bin/bash
# im2col1d variants (channels per block x XCD-aware numbering) on the default bench, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for cfg in "16 0" "32 1" "32 0" "16 1"; do
    set -- $cfg
    A2M_I2C_C=$1 A2M_I2C_XCD=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --warmup 10 > gpurun_out/ab.log 2>&1 || exit 4
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'])" "C=$1 XCD=$2"
  done
done
