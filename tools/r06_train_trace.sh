#!/bin/bash
# Kernel traces of the graph-replayed training iteration: per-iteration kernel time vs span.
#   tools/r06_train_trace.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-tt}
export TMPDIR=/tmp
one() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $PWD/gpurun_out/trc_${TAG}_$name -o run -- \
    python bench.py --mode train --steps 5 --warmup 5 "$@" > gpurun_out/trc_${TAG}_$name.log 2>&1 || { echo "$name failed"; tail -3 gpurun_out/trc_${TAG}_$name.log; exit 4; }
  python tools/train_graph_trace.py $(find gpurun_out/trc_${TAG}_$name -name "*kernel_trace.csv" | head -1) 5 > gpurun_out/trc_${TAG}_$name.txt
  find gpurun_out/trc_${TAG}_$name -name "*.csv" -delete
  echo "== $name: $(tail -1 gpurun_out/trc_${TAG}_$name.log | python -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], "ms wall under the tracer")')"
  head -3 gpurun_out/trc_${TAG}_$name.txt
}
one b8_fp32 --batch 8
one b32_bf16 --batch 32 --dtype bf16
one b64_fp32
exit 0
