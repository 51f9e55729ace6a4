#!/bin/bash
# engine k-loop changes: GPU tests, lib A/B vs HEAD build, then the r04b probes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04c_pytest_gpu.log 2>&1 || { tail -5 gpurun_out/r04c_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r04c_pytest_gpu.log
bash tools/ab_lib.sh 3 _ab/liba2m_base.so > gpurun_out/r04c_ablib.txt 2>&1 || exit 2
cat gpurun_out/r04c_ablib.txt
bash tools/gpu_r04b.sh; echo "r04b rc=$?"
