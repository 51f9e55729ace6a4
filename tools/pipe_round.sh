#!/bin/bash
# GPU round for the pipelined tile: GPU tests, per-launch probe (pipe on / off), bench A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pipe.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_pipe.log; fatal $rc pytest
for v in 1 0; do
  A2M_GEMM_PIPE=$v timeout -k 10 150 python tools/pipe_probe.py > gpurun_out/probe$v.log 2>&1
  rc=$?; cat gpurun_out/probe$v.log; fatal $rc probe
done
bash tools/ab_envs.sh A2M_GEMM_PIPE "1 0" ${ROUNDS:-2}
