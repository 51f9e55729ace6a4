#!/bin/bash
# fp32 wide-attention QKV without the [B*T][C] copy (in-tree, A2M_WIDE_BTC=2) vs always copying
# (_ab/btc1.so): parity tests, inference and fp32 training lines, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread -k "self_attention or headline or train_step" > gpurun_out/btc2_pytest.log 2>&1 || { tail -20 gpurun_out/btc2_pytest.log; exit 1; }
tail -1 gpurun_out/btc2_pytest.log
L0=$PWD/audio-to-motion-generation_amd/a2m/liba2m_hip.so
for i in 1 2; do
  for lib in $L0 $PWD/_ab/btc1.so; do
    A2M_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-trace --steps 300 > gpurun_out/btc_b.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/btc_b.log; exit 3; }
    A2M_LIB=$lib timeout -k 10 300 python bench.py --mode train --steps 10 --warmup 5 > gpurun_out/btc_t.log 2>&1 || { echo "train failed"; tail -5 gpurun_out/btc_t.log; exit 3; }
    echo "$(basename $lib) fp32 $(python -c "import json; print(json.loads(open('gpurun_out/btc_b.log').read().strip().splitlines()[-1])['ms_per_step'])") train $(python -c "import json; print(json.loads(open('gpurun_out/btc_t.log').read().strip().splitlines()[-1])['ms_per_step'])")"
  done
done
exit 0
