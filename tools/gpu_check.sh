#!/bin/bash
# One GPU session: parity tests, bench, rocprof kernel trace.  Every GPU step has its own time
# limit; a step that faults / aborts / times out (exit >= 2 for pytest, != 0 otherwise) ends
# the script before any further GPU work.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r1}
timeout -k 10 900 python -m pytest tests -m gpu -q -x --durations=15 > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu_$TAG.log
if [ $rc -ge 2 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.log; exit 3; }
tail -2 gpurun_out/bench_$TAG.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
  python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_$TAG.log; exit 4; }
find gpurun_out/prof_$TAG -name "*stats*" | head
exit $rc
