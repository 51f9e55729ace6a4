#!/bin/bash
# Round evidence in one GPU call, every GPU step under its own time limit, stopping at the first
# failure: the GPU parity tests, smoke(), the bench line, a rocprof kernel trace + stats of that
# same bench command (its engine-family average launch must agree with the line's
# roofline: tools/bench_stats.py), and the replayed-step rocprof / PMC passes
# (tools/step_pmc.sh: per-step breakdown, HBM traffic, MFMA busy).
#   tools/gpu_round.sh TAG [--skip-tests]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
TAG=$1
mkdir -p gpurun_out
if [ "${2:-}" != "--skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread --durations=15 > gpurun_out/${TAG}_pytest_gpu.log 2>&1
  rc=$?
  tail -2 gpurun_out/${TAG}_pytest_gpu.log
  [ $rc -eq 0 ] || { echo "pytest rc=$rc: stopping"; exit 1; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -5 gpurun_out/${TAG}_smoke.log; exit 2; }
  tail -1 gpurun_out/${TAG}_smoke.log
fi
A2M_BENCH_TRACE_DIR=gpurun_out/${TAG}_trace timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 3; }
cat gpurun_out/${TAG}_bench.json
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/gpurun_out/${TAG}_benchprof -o run -- \
  python bench.py --no-cpu-baseline --no-trace > gpurun_out/${TAG}_benchprof.json 2> gpurun_out/${TAG}_benchprof.err || { echo "rocprof bench failed"; tail -20 gpurun_out/${TAG}_benchprof.err; exit 4; }
python tools/bench_stats.py gpurun_out/${TAG}_benchprof gpurun_out/${TAG}_bench.json --out gpurun_out/${TAG}_bench_kernel_stats.txt || exit 5
find gpurun_out/${TAG}_benchprof -name "*kernel_trace.csv" -delete
bash tools/step_pmc.sh $TAG || exit 6
exit 0
