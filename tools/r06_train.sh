#!/bin/bash
# Round 6: graph-replayed training -- its tests, then one-GPU training lines with and without
# the graphs (configs[2]'s per-rank shard B=8 fp32, configs[4]'s B=32 bf16, B=64 fp32).
#   tools/r06_train.sh TAG [pytest selection]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-t}
SEL=${2:-tests/test_gpu_train_graphs.py tests/test_gpu_rccl.py tests/test_gpu_train.py}
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/pytest_$TAG.log | head -30; exit $rc; fi
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python bench.py --mode train --steps 20 --warmup 5 "$@" > gpurun_out/tr_${TAG}_$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/tr_${TAG}_$name.log; exit 3; }
  tail -1 gpurun_out/tr_${TAG}_$name.log > gpurun_out/tr_${TAG}_$name.json
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['unit'], d['ms_per_step'], 'ms', d['dtype'], d['config'].get('hip_graph'))" gpurun_out/tr_${TAG}_$name.json $name
}
run b8_fp32_graph --batch 8
run b8_fp32_eager --batch 8 --no-graph
run b32_bf16_graph --batch 32 --dtype bf16
run b32_bf16_eager --batch 32 --dtype bf16 --no-graph
run b64_fp32_graph
run b64_fp32_eager --no-graph
run b32_bf16_graph2 --batch 32 --dtype bf16
run b32_bf16_graph3 --batch 32 --dtype bf16
exit 0
