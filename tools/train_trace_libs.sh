#!/bin/bash
# Kernel-trace per-kernel summaries of the training iteration for several libraries
#   tools/train_trace_libs.sh lib1.so lib2.so ... ("" = working tree)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in "$@"; do
  tag=$(basename "${lib:-new}" .so)
  env ${lib:+A2M_LIB=$PWD/$lib} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $PWD/gpurun_out/tt_$tag -o run -- python bench.py --mode train --steps 3 --warmup 1 > gpurun_out/tt_$tag.log 2>&1 || { echo "trace fail $tag"; tail -3 gpurun_out/tt_$tag.log; exit 4; }
  python tools/prof_summary.py $(find gpurun_out/tt_$tag -name "*kernel_trace.csv" | head -1) 4 > gpurun_out/train_breakdown_$tag.txt
  find gpurun_out/tt_$tag -name "*.csv" -size +5M -delete
  echo "== $tag"; head -3 gpurun_out/train_breakdown_$tag.txt
done
