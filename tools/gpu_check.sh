#!/bin/bash
# One GPU session: parity tests, bench, rocprof kernel trace, two PMC passes (HBM traffic).
# Every GPU step has its own time limit; a step that faults / aborts / times out ends the
# script before any further GPU work.
#   tools/gpu_check.sh TAG [--skip-tests]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
mkdir -p gpurun_out
TAG=${1:-r1}
SKIP_TESTS=${2:-}
if [ "$SKIP_TESTS" != "--skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread --durations=15 > gpurun_out/pytest_gpu_$TAG.log 2>&1
  rc=$?
  tail -5 gpurun_out/pytest_gpu_$TAG.log
  if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.log; exit 3; }
tail -1 gpurun_out/bench_$TAG.log
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/gpurun_out/prof_$TAG -o run -- \
  python $REPO/bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_$TAG.log; exit 4; }
tail -1 gpurun_out/prof_$TAG.log
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $REPO/gpurun_out/pmc_fetch_$TAG -o run -- \
  python $REPO/bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline > gpurun_out/pmc_fetch_$TAG.log 2>&1 || { echo "pmc fetch failed"; tail -20 gpurun_out/pmc_fetch_$TAG.log; exit 5; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $REPO/gpurun_out/pmc_write_$TAG -o run -- \
  python $REPO/bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline > gpurun_out/pmc_write_$TAG.log 2>&1 || { echo "pmc write failed"; tail -20 gpurun_out/pmc_write_$TAG.log; exit 6; }
python tools/pmc_traffic.py gpurun_out/pmc_fetch_$TAG gpurun_out/pmc_write_$TAG --out gpurun_out/traffic_$TAG.json --tag $TAG > /dev/null || echo "pmc parse failed"
find gpurun_out/prof_$TAG -name "*stats*"
# drop the bulky per-dispatch PMC csvs once summarised (keeps gpurun_out small)
find gpurun_out/pmc_fetch_$TAG gpurun_out/pmc_write_$TAG -name "*counter_collection.csv" -size +20M -delete
exit 0
