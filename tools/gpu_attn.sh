#!/bin/bash
# Attention iteration: attention parity tests, then op timings of the three attention shapes
# under the fused / packed / general paths.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-attn}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train.py -m gpu -q -x -k "attention or generator or headline" --timeout 120 --timeout-method thread > gpurun_out/attn_$TAG.log 2>&1 || { tail -30 gpurun_out/attn_$TAG.log; exit 2; }
tail -1 gpurun_out/attn_$TAG.log
for cfg in "A2M_X=1" "A2M_ATTN_EVAL_FUSED=0" "A2M_ATTN_EVAL_FUSED=0 A2M_ATTN_FUSED=0"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python tools/op_bench.py attn 2>&1 | grep attn || exit 3
done
exit 0
