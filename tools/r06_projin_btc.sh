#!/bin/bash
# bf16 mode: proj_in as a [B*T][C] copy + dense linear (real_motion_model._PROJ_IN_BTC, default on)
# vs the 1x1 conv over [B][C][T] (row-gathered B); bf16 parity tests, then bf16 bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread -k "bf16" > gpurun_out/pb_pytest.log 2>&1 || { tail -20 gpurun_out/pb_pytest.log; exit 1; }
tail -1 gpurun_out/pb_pytest.log
for i in 1 2 3; do
  for v in 1 0; do
    timeout -k 10 300 python tools/bench_flag.py real_motion_model._PROJ_IN_BTC=$v -- --no-cpu-baseline --no-trace --steps 300 --dtype bf16 > gpurun_out/pb_b64.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/pb_b64.log; exit 3; }
    timeout -k 10 300 python tools/bench_flag.py real_motion_model._PROJ_IN_BTC=$v -- --no-cpu-baseline --no-trace --steps 300 --dtype bf16 --batch 32 > gpurun_out/pb_b32.log 2>&1 || { echo "bench b32 failed"; exit 3; }
    echo "proj_in_btc=$v bf16 B=64 $(python -c "import json; print(json.loads(open('gpurun_out/pb_b64.log').read().strip().splitlines()[-1])['ms_per_step'])") B=32 $(python -c "import json; print(json.loads(open('gpurun_out/pb_b32.log').read().strip().splitlines()[-1])['ms_per_step'])")"
  done
done
exit 0
