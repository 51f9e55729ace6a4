#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tapconv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04e_parity.log 2>&1 || { tail -5 gpurun_out/r04e_parity.log; exit 1; }
tail -1 gpurun_out/r04e_parity.log
bash tools/ab_lib.sh 4 _ab/liba2m_base.so > gpurun_out/r04e_ablib.txt 2>&1 || exit 3
cat gpurun_out/r04e_ablib.txt
bash tools/ab_env.sh "A2M_GEMM_PRIO=1" 3 > gpurun_out/r04e_ab_prio.txt 2>&1; cat gpurun_out/r04e_ab_prio.txt
timeout -k 10 120 python tools/instep_spans.py 10 > gpurun_out/r04_instep_spans.txt 2>&1; tail -40 gpurun_out/r04_instep_spans.txt
