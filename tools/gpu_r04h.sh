#!/bin/bash
# mode-5 halo layout: parity (tap-conv + generator tests), conv sweep and step A/B against A2M_GEMM_HALO=0
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_tapconv.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04h_tests.log 2>&1 || { tail -30 gpurun_out/r04h_tests.log; exit 1; }
tail -3 gpurun_out/r04h_tests.log
for h in 0 1 0 1; do
  echo "== A2M_GEMM_HALO=$h"
  A2M_GEMM_HALO=$h timeout -k 10 120 python tools/conv_scaling.py 2>&1 | grep -v amdgpu.ids || exit 2
done > gpurun_out/r04h_conv.txt 2>&1 || { cat gpurun_out/r04h_conv.txt; exit 2; }
cat gpurun_out/r04h_conv.txt
bash tools/ab_env.sh "A2M_GEMM_HALO=0" 3 > gpurun_out/r04h_ab.txt 2>&1; rc=$?
cat gpurun_out/r04h_ab.txt
exit $rc
