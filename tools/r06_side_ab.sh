#!/bin/bash
# Decoder branch placement: hand on the side stream, issued first (default) vs body; fp32 and bf16.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "headline" > gpurun_out/sd_pytest.log 2>&1 || { tail -20 gpurun_out/sd_pytest.log; exit 1; }
for i in 1 2 3; do
  for v in 1 0; do
    timeout -k 10 300 python tools/bench_flag.py real_motion_model._HAND_ON_SIDE=$v -- --no-cpu-baseline --no-trace --steps 300 > gpurun_out/sd_b.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/sd_b.log; exit 3; }
    timeout -k 10 300 python tools/bench_flag.py real_motion_model._HAND_ON_SIDE=$v -- --no-cpu-baseline --no-trace --steps 300 --dtype bf16 > gpurun_out/sd_b16.log 2>&1 || { echo "bench bf16 failed"; exit 3; }
    echo "hand_on_side=$v fp32 $(python -c "import json; print(json.loads(open('gpurun_out/sd_b.log').read().strip().splitlines()[-1])['ms_per_step'])") bf16 $(python -c "import json; print(json.loads(open('gpurun_out/sd_b16.log').read().strip().splitlines()[-1])['ms_per_step'])")"
  done
done
exit 0
