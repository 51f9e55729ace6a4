#!/bin/bash
# Bench step time under the engine's experiment switches (two 100-step runs each), to re-check
# defaults after other changes.   tools/env_sweep.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in "" "A2M_GEMM_KS2=0" "A2M_GEMM_KS3=0" "A2M_GEMM_XCD=4" "A2M_GEMM_XCD=16" "A2M_GEMM_MCONTIG=0" "A2M_TAP_CONV=0" "A2M_ENC_NHWC=0" "A2M_ATTN_BTC=0" "A2M_HAND_FIRST=0" ""; do
  for rep in 1 2; do
    env $cfg timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/sweep.log 2>&1 || { echo "fail $cfg"; exit 3; }
    echo "[$cfg] $(python -c "import json,sys; print(json.loads(open('gpurun_out/sweep.log').read().strip().splitlines()[-1])['ms_per_step'])")"
  done
done
