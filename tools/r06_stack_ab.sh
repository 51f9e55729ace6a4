#!/bin/bash
# Graph-stack epilogue A/B: parity tests of the stack, then tools/stack_bench.py (each stack alone)
# for the in-tree library and _ab/tepi0.so (the round-5 epilogue), interleaved, then in-step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bf16.py -m gpu -x -q --timeout 200 -k "stack or headline or g_eval" > gpurun_out/stk_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/stk_pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/stk_pytest.log | head; exit $rc; }
for i in 1 2 3; do
  for lib in audio-to-motion-generation_amd/a2m/liba2m_hip.so _ab/tepi0.so; do
    A2M_LIB=$PWD/$lib timeout -k 10 120 python tools/stack_bench.py both 50 2>&1 | grep stack | sed "s|^|$(basename $lib .so) |" || exit 3
  done
done
for i in 1 2; do
  for lib in audio-to-motion-generation_amd/a2m/liba2m_hip.so _ab/tepi0.so; do
    A2M_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-trace --steps 200 > gpurun_out/stk_bench.log 2>&1 || exit 4
    python -c "import json,sys; d=json.loads(open('gpurun_out/stk_bench.log').read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['roofline']['frac'])" $(basename $lib .so)
  done
done
