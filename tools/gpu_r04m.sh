#!/bin/bash
# bf16x6 graph stack: parity, isolated timing (x6 vs fp32 kernel), step A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04m_tests.log 2>&1 || { tail -30 gpurun_out/r04m_tests.log; exit 1; }
tail -2 gpurun_out/r04m_tests.log
for v in 0 1 0 1; do echo "A2M_STACK_X6=$v"; A2M_STACK_X6=$v timeout -k 10 120 python tools/stack_bench.py both 50 2>&1 | grep stack || exit 2; done
bash tools/ab_env.sh "A2M_STACK_X6=0" 3 > gpurun_out/r04m_ab.txt 2>&1; rc=$?
cat gpurun_out/r04m_ab.txt
exit $rc
