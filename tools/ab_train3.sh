#!/bin/bash
# Training iteration (bench.py --mode train) with several libraries interleaved, N rounds, plus a
# kernel-trace summary of the working tree's iteration.   tools/ab_train3.sh N lib1.so lib2.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
N=$1; shift
for i in $(seq $N); do
  for lib in "$@" ""; do
    tag=${lib:-new}
    env ${lib:+A2M_LIB=$PWD/$lib} timeout -k 10 300 python bench.py --mode train --steps 5 --warmup 2 ${TRAIN_ARGS:-} > gpurun_out/abt.log 2>&1 || { echo "fail $tag"; tail -3 gpurun_out/abt.log; exit 3; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/abt.log').read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'])" $tag
  done
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $PWD/gpurun_out/trtrain -o run -- python bench.py --mode train --steps 3 --warmup 1 ${TRAIN_ARGS:-} > gpurun_out/trtrain.log 2>&1 || { echo "trace fail"; tail -3 gpurun_out/trtrain.log; exit 4; }
python tools/prof_summary.py $(find gpurun_out/trtrain -name "*kernel_trace.csv" | head -1) 4 > gpurun_out/train_breakdown.txt
head -30 gpurun_out/train_breakdown.txt
find gpurun_out/trtrain -name "*.csv" -size +5M -delete
