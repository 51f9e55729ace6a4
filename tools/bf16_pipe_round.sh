#!/bin/bash
# bf16 pipelined tile: its GPU tests, the per-launch probe (pipe / gemm_tile) and the bf16 bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2"; exit $1;; esac; }
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 300 python -u -m pytest tests/test_gpu_pipe.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pipe.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ -n "${SKIP_TESTS:-}" ] || tail -5 gpurun_out/pytest_pipe.log; fatal $rc pytest; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  A2M_GEMM_PIPE=$v timeout -k 10 150 python tools/pipe_probe.py bf16 > gpurun_out/probe_bf16_$v.log 2>&1
  rc=$?; cat gpurun_out/probe_bf16_$v.log | grep -v amdgpu.ids; fatal $rc probe
done
[ -n "${SKIP_BENCH:-}" ] || BENCH_ARGS="--dtype bf16" bash tools/ab_envs.sh A2M_GEMM_PIPE "1 0" 2
