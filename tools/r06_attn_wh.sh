#!/bin/bash
# bf16 fused eval attention staging the stacked weights' cached bf16 copy: parity tests, then bf16
# bench lines (B = 64, 32) with the flag on / off (tools/bench_flag.py), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bf16.py tests/test_gpu_configs.py tests/test_gpu_grouped.py -x -q --timeout 200 --timeout-method thread -k "attention or bf16 or headline or grouped" > gpurun_out/aw_pytest.log 2>&1 || { tail -30 gpurun_out/aw_pytest.log; exit 1; }
tail -1 gpurun_out/aw_pytest.log
for i in 1 2 3; do
  for v in 1 0; do
    timeout -k 10 300 python tools/bench_flag.py functional._ATTN_BF16_WEIGHTS=$v -- --no-cpu-baseline --no-trace --steps 300 --dtype bf16 > gpurun_out/aw_b64.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/aw_b64.log; exit 3; }
    timeout -k 10 300 python tools/bench_flag.py functional._ATTN_BF16_WEIGHTS=$v -- --no-cpu-baseline --no-trace --steps 300 --dtype bf16 --batch 32 > gpurun_out/aw_b32.log 2>&1 || { echo "bench b32 failed"; exit 3; }
    echo "attn_wh=$v bf16 B=64 $(python -c "import json; print(json.loads(open('gpurun_out/aw_b64.log').read().strip().splitlines()[-1])['ms_per_step'])") B=32 $(python -c "import json; print(json.loads(open('gpurun_out/aw_b32.log').read().strip().splitlines()[-1])['ms_per_step'])")"
  done
done
exit 0
