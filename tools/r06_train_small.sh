#!/bin/bash
# Training-path tests, then B=8 fp32 / B=32 bf16 / B=64 fp32 lines and a B=8 trace.   tools/r06_train_small.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-ts}
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_train_graphs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "train or loss or motion or graph or pose" > gpurun_out/pytest_$TAG.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_$TAG.log | head -20; exit 1; }
for a in "b8 --batch 8" "b32bf16 --batch 32 --dtype bf16" "b64"; do
  set -- $a; name=$1; shift
  timeout -k 10 300 python bench.py --mode train --steps 20 --warmup 5 "$@" > gpurun_out/tr_${TAG}_$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/tr_${TAG}_$name.log; exit 3; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], 'ms')" gpurun_out/tr_${TAG}_$name.log $name
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $PWD/gpurun_out/trc_${TAG} -o run -- python bench.py --mode train --steps 5 --warmup 5 --batch 8 > gpurun_out/trc_${TAG}.log 2>&1 || { echo "trace failed"; tail -3 gpurun_out/trc_${TAG}.log; exit 4; }
python tools/train_graph_trace.py $(find gpurun_out/trc_${TAG} -name "*kernel_trace.csv" | head -1) 5 > gpurun_out/trc_${TAG}.txt
find gpurun_out/trc_${TAG} -name "*.csv" -delete
head -6 gpurun_out/trc_${TAG}.txt; grep -E "pose_loss|motion_terms" gpurun_out/trc_${TAG}.txt
