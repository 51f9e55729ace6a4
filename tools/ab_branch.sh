#!/bin/bash
# A/B of the decoder branch order / side-stream priority (bench line per setting).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in "1 0" "0 0" "1 0" "0 0" "0 1"; do
  set -- $v
  A2M_HAND_FIRST=$1 A2M_SIDE_PRIO=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 50 > gpurun_out/bench_ab.log 2>&1 || exit 3
  echo "hand_first=$1 prio=$2 $(tail -1 gpurun_out/bench_ab.log | cut -c100-200)"
done
