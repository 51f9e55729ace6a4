#!/bin/bash
# The decoders' proj_in (M = nj * 64, N = B * T, K = 256, row-gathered B) on 128x128 tiles vs the
# planner's 64x64, in the replayed bench step (A2M_GEMM_PLAN_RULES), fp32 and bf16, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R128="2688,4096,256:128:1;640,4096,256:128:1"
for i in 1 2 3; do
  for rules in "" "$R128"; do
    A2M_GEMM_PLAN_RULES="$rules" timeout -k 10 300 python bench.py --no-cpu-baseline --no-trace --steps 300 > gpurun_out/pi_b.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/pi_b.log; exit 3; }
    A2M_GEMM_PLAN_RULES="$rules" timeout -k 10 300 python bench.py --no-cpu-baseline --no-trace --steps 300 --dtype bf16 > gpurun_out/pi_b16.log 2>&1 || { echo "bench bf16 failed"; exit 3; }
    echo "rules='${rules}' fp32 $(python -c "import json; print(json.loads(open('gpurun_out/pi_b.log').read().strip().splitlines()[-1])['ms_per_step'])") bf16 $(python -c "import json; print(json.loads(open('gpurun_out/pi_b16.log').read().strip().splitlines()[-1])['ms_per_step'])")"
  done
done
exit 0
