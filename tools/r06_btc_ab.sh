#!/bin/bash
# The wide attentions' QKV projection: [B*T][C] copy + dense GEMM (in-tree) vs the 1x1 conv over the
# [B][C][T] layout (row-gathered B on the pipelined tile; _ab/nobtc.so), interleaved bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "self_attention or headline" > gpurun_out/btc_pytest.log 2>&1 || { tail -20 gpurun_out/btc_pytest.log; exit 1; }
L0=$PWD/audio-to-motion-generation_amd/a2m/liba2m_hip.so
for i in 1 2 3; do
  for lib in $L0 $PWD/_ab/nobtc.so; do
    A2M_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-trace --steps 300 > gpurun_out/btc_b.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/btc_b.log; exit 3; }
    A2M_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-trace --steps 300 --dtype bf16 > gpurun_out/btc_b16.log 2>&1 || { echo "bench bf16 failed"; exit 3; }
    echo "$(basename $lib) fp32 $(python -c "import json; print(json.loads(open('gpurun_out/btc_b.log').read().strip().splitlines()[-1])['ms_per_step'])") bf16 $(python -c "import json; print(json.loads(open('gpurun_out/btc_b16.log').read().strip().splitlines()[-1])['ms_per_step'])")"
  done
done
exit 0
