#!/bin/bash
# Whole-channel BatchNorm: training parity tests, then training lines and traces with and without it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-bn}
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_train_graphs.py tests/test_gpu_syncbn.py tests/test_gpu_rccl.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/pytest_$TAG.log | head -30; exit $rc; fi
grep -E "gG:|gD:" gpurun_out/pytest_$TAG.log | cut -c1-400 | head -8
for v in 1 1; do
  A2M_BN_CHAN=$v timeout -k 10 300 python bench.py --mode train --steps 20 --warmup 5 > gpurun_out/tr_${TAG}_$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/tr_${TAG}_$v.log; exit 3; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('A2M_BN_CHAN', sys.argv[2], d['ms_per_step'], 'ms')" gpurun_out/tr_${TAG}_$v.log $v
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $PWD/gpurun_out/trc_${TAG} -o run -- python bench.py --mode train --steps 5 --warmup 5 > gpurun_out/trc_${TAG}.log 2>&1 || { echo "trace failed"; tail -3 gpurun_out/trc_${TAG}.log; exit 4; }
python tools/train_graph_trace.py $(find gpurun_out/trc_${TAG} -name "*kernel_trace.csv" | head -1) 5 > gpurun_out/trc_${TAG}.txt
find gpurun_out/trc_${TAG} -name "*.csv" -delete
head -6 gpurun_out/trc_${TAG}.txt; grep -E "bn_|reduce_slices" gpurun_out/trc_${TAG}.txt
A2M_GEMM_LOG=1 timeout -k 10 300 python bench.py --mode train --steps 1 --warmup 1 --no-graph > gpurun_out/train_plans_${TAG}.out 2> gpurun_out/train_plans_${TAG}.txt || exit 5
grep -c "a2m gemm" gpurun_out/train_plans_${TAG}.txt
