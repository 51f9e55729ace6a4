#!/bin/bash
# The decoders' 256x4096x768 tap convs (one 64x64 block per CU) at 2 splits (A2M_GEMM_PLAN_RULES)
# vs the planner's 1, fp32 and bf16 bench lines, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2 3; do
  for r in "" "256,4096,768:64:2"; do
    A2M_GEMM_PLAN_RULES="$r" timeout -k 10 300 python bench.py --no-cpu-baseline --no-trace --steps 300 > gpurun_out/ds_b.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/ds_b.log; exit 3; }
    A2M_GEMM_PLAN_RULES="$r" timeout -k 10 300 python bench.py --no-cpu-baseline --no-trace --steps 300 --dtype bf16 > gpurun_out/ds_b16.log 2>&1 || { echo "bench bf16 failed"; exit 3; }
    echo "rules='$r' fp32 $(python -c "import json; print(json.loads(open('gpurun_out/ds_b.log').read().strip().splitlines()[-1])['ms_per_step'])") bf16 $(python -c "import json; print(json.loads(open('gpurun_out/ds_b16.log').read().strip().splitlines()[-1])['ms_per_step'])")"
  done
done
exit 0
