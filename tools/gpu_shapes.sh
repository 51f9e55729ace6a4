#!/bin/bash
# Per-launch GEMM shape table + kernel breakdown of one eager bench step (no tests).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
mkdir -p gpurun_out
TAG=${1:-s}
export TMPDIR=/tmp
A2M_GEMM_LOG=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $REPO/gpurun_out/shapes_$TAG -o run -- \
  python $REPO/bench.py --no-graph --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/shapes_$TAG.out 2> gpurun_out/shapes_$TAG.err || { echo "shape profile failed"; tail -5 gpurun_out/shapes_$TAG.err; exit 4; }
python tools/gemm_shapes.py gpurun_out/shapes_$TAG.err gpurun_out/shapes_$TAG/run_kernel_trace.csv 49 > gpurun_out/shapes_$TAG.txt
python tools/prof_summary.py gpurun_out/shapes_$TAG/run_kernel_trace.csv 3 > gpurun_out/breakdown_$TAG.txt
exit 0
