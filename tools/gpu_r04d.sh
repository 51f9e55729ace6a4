#!/bin/bash
# branch-free mode 0/6 loads (+ DB / PRIO switches): parity subset, then lib / env A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04d_pytest_gpu.log 2>&1 || { tail -5 gpurun_out/r04d_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r04d_pytest_gpu.log
A2M_GEMM_DB=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tapconv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04d_db_parity.log 2>&1 || { tail -5 gpurun_out/r04d_db_parity.log; exit 2; }
tail -1 gpurun_out/r04d_db_parity.log
bash tools/ab_lib.sh 3 _ab/liba2m_base.so > gpurun_out/r04d_ablib.txt 2>&1 || exit 3
cat gpurun_out/r04d_ablib.txt
bash tools/ab_env.sh "A2M_GEMM_DB=1" 2 > gpurun_out/r04d_ab_db.txt 2>&1; cat gpurun_out/r04d_ab_db.txt
bash tools/ab_env.sh "A2M_GEMM_PRIO=1" 2 > gpurun_out/r04d_ab_prio.txt 2>&1; cat gpurun_out/r04d_ab_prio.txt
