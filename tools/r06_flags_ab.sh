#!/bin/bash
# Module-level route choices re-measured on the round-6 kernels: each flipped alone
# (tools/bench_flag.py) against the defaults, fp32 bench lines, two interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  timeout -k 10 300 python tools/bench_flag.py "$@" -- --no-cpu-baseline --no-trace --steps 300 > gpurun_out/fl_b.log 2>&1 || { echo "bench $* failed"; tail -5 gpurun_out/fl_b.log; exit 3; }
  echo "$* $(python -c "import json; print(json.loads(open('gpurun_out/fl_b.log').read().strip().splitlines()[-1])['ms_per_step'])")"
}
for i in 1 2; do
  run real_motion_model._FUSED_STACK=1
  run real_motion_model._BRANCH_STREAMS=0
  run model_layers._ENC_NHWC_ALL=0
  run model_layers._ENC_FUSED_INTERP=0
  run functional._TAP_CONV=0
  run functional._TAP_CONVT=0
  run functional._ATTN_EVAL_FUSED=0
done
exit 0
