#!/bin/bash
# Weight gradients on a side stream, overlapping each layer's data gradient (autograd._WGRAD_SIDE,
# default on): the training GPU tests, then training lines with the flag on / off, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_train_graphs.py tests/test_gpu_rccl.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ws_pytest.log 2>&1 || { tail -30 gpurun_out/ws_pytest.log; exit 1; }
tail -1 gpurun_out/ws_pytest.log
for i in 1 2; do
  for v in 1 0; do
    timeout -k 10 300 python tools/bench_flag.py autograd._WGRAD_SIDE=$v -- --mode train --steps 10 --warmup 5 --no-trace > gpurun_out/ws_t64.log 2>&1 || { echo "train failed"; tail -5 gpurun_out/ws_t64.log; exit 3; }
    timeout -k 10 300 python tools/bench_flag.py autograd._WGRAD_SIDE=$v -- --mode train --steps 10 --warmup 5 --batch 8 --no-trace > gpurun_out/ws_t8.log 2>&1 || { echo "train b8 failed"; exit 3; }
    timeout -k 10 300 python tools/bench_flag.py autograd._WGRAD_SIDE=$v -- --mode train --steps 10 --warmup 5 --batch 32 --dtype bf16 --no-trace > gpurun_out/ws_t32.log 2>&1 || { echo "train bf16 failed"; exit 3; }
    echo "wgrad_side=$v fp32 B=64 $(python -c "import json; print(json.loads(open('gpurun_out/ws_t64.log').read().strip().splitlines()[-1])['ms_per_step'])") B=8 $(python -c "import json; print(json.loads(open('gpurun_out/ws_t8.log').read().strip().splitlines()[-1])['ms_per_step'])") bf16 B=32 $(python -c "import json; print(json.loads(open('gpurun_out/ws_t32.log').read().strip().splitlines()[-1])['ms_per_step'])")"
  done
done
exit 0
