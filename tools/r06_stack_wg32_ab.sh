#!/bin/bash
# fp32 graph stack at 2 workgroups per CU (_ab/f32wg2.so) vs 3 (in-tree); bf16 tests for the new
# bf16 default, stack_bench and fp32 bench lines, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bf16.py -x -q --timeout 200 --timeout-method thread -k "stack or bf16" > gpurun_out/wg3_pytest.log 2>&1 || { tail -20 gpurun_out/wg3_pytest.log; exit 1; }
tail -1 gpurun_out/wg3_pytest.log
L0=$PWD/audio-to-motion-generation_amd/a2m/liba2m_hip.so
for lib in $L0 $PWD/_ab/f32wg2.so; do
  echo "$(basename $lib) $(A2M_LIB=$lib timeout -k 10 120 python tools/stack_bench.py both 50 | tr '\n' ' ')"
done
for i in 1 2 3 4; do
  for lib in $L0 $PWD/_ab/f32wg2.so; do
    A2M_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-trace --steps 300 > gpurun_out/wg3_b.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/wg3_b.log; exit 3; }
    echo "$(basename $lib) fp32 $(python -c "import json; print(json.loads(open('gpurun_out/wg3_b.log').read().strip().splitlines()[-1])['ms_per_step'])")"
  done
done
exit 0
