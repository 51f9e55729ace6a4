#!/bin/bash
# GPU tests + per-launch probe + one default bench line with its kernel trace kept
#   tools/gpu_check.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-chk}
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_$TAG.log; fatal $rc pytest
if [ -n "${PROBE:-}" ]; then
  for v in 1 0; do
    A2M_GEMM_PIPE=$v timeout -k 10 150 python tools/pipe_probe.py > gpurun_out/probe${v}_$TAG.log 2>&1
    rc=$?; grep -E "gemm-kr|gemm 2688|conv1d B=64 Ci=256 Co=256" gpurun_out/probe${v}_$TAG.log; fatal $rc probe
  done
fi
A2M_BENCH_TRACE_DIR=gpurun_out/trace_$TAG timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; tail -c 3000 gpurun_out/bench_$TAG.json; fatal $rc bench
head -12 gpurun_out/trace_$TAG/step_breakdown.txt
