#!/bin/bash
# Log-mel iteration: mel parity tests, then the bench's graph-timed mel kernel and its rocprof row.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-mel}
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "logmel or end_to_end or invariance" --timeout 120 --timeout-method thread > gpurun_out/mel_$TAG.log 2>&1 || { tail -30 gpurun_out/mel_$TAG.log; exit 2; }
tail -1 gpurun_out/mel_$TAG.log
timeout -k 10 300 python tools/mel_bench.py > gpurun_out/melbench_$TAG.log 2>&1 || { tail -20 gpurun_out/melbench_$TAG.log; exit 3; }
cat gpurun_out/melbench_$TAG.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/melprof_$TAG -o run -- python tools/mel_bench.py > /dev/null 2>&1 || { echo "rocprof failed"; exit 4; }
grep -i logmel gpurun_out/melprof_$TAG/run_kernel_stats.csv
exit 0
