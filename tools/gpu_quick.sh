#!/bin/bash
# Quick GPU iteration: parity tests, bench (no CPU baseline), per-launch GEMM shape profile.
#   tools/gpu_quick.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
mkdir -p gpurun_out
TAG=${1:-q}
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/pytest_$TAG.log | head -20; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.log; exit 3; }
tail -1 gpurun_out/bench_$TAG.log
export TMPDIR=/tmp
A2M_GEMM_LOG=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $REPO/gpurun_out/shapes_$TAG -o run -- \
  python $REPO/bench.py --no-graph --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/shapes_$TAG.out 2> gpurun_out/shapes_$TAG.err || { echo "shape profile failed"; tail -5 gpurun_out/shapes_$TAG.err; exit 4; }
python tools/gemm_shapes.py gpurun_out/shapes_$TAG.err gpurun_out/shapes_$TAG/run_kernel_trace.csv 49 > gpurun_out/shapes_$TAG.txt
python tools/prof_summary.py gpurun_out/shapes_$TAG/run_kernel_trace.csv 3 > gpurun_out/breakdown_$TAG.txt
exit 0
