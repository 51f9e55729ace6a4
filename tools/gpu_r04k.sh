#!/bin/bash
# in-launch split-K combine: full GPU tests, then step A/B against A2M_GEMM_FIXUP=0
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tapconv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04k_pytest.log 2>&1 || { tail -30 gpurun_out/r04k_pytest.log; exit 1; }
tail -2 gpurun_out/r04k_pytest.log
bash tools/ab_env.sh "A2M_GEMM_FIXUP=0" 3 > gpurun_out/r04k_ab.txt 2>&1; rc=$?
cat gpurun_out/r04k_ab.txt
exit $rc
