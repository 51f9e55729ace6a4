#!/bin/bash
# interleaved decoder-branch capture: parity + step A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A2M_INTERLEAVE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "headline or generator" > gpurun_out/r04n_tests.log 2>&1 || { tail -30 gpurun_out/r04n_tests.log; exit 1; }
tail -2 gpurun_out/r04n_tests.log
bash tools/ab_env.sh "A2M_INTERLEAVE=1" 3 > gpurun_out/r04n_ab.txt 2>&1; rc=$?
cat gpurun_out/r04n_ab.txt
exit $rc
