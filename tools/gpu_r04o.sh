#!/bin/bash
# LDS-DMA GEMM staging (KS = 4): parity under A2M_GEMM_GLDS=2, then A/B 0 / 1 / 2
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A2M_GEMM_GLDS=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tapconv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04o_tests.log 2>&1 || { tail -30 gpurun_out/r04o_tests.log; exit 1; }
tail -2 gpurun_out/r04o_tests.log
bash tools/ab_envs.sh A2M_GEMM_GLDS "0 1 2" 3
