#!/bin/bash
# bf16 inference step (B = 64 and B = 32): replayed-step breakdown and per-queue lanes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for B in 64 32; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/bl_tr_$B -o run -- python tools/step_pmc.py 10 --sync --engine-json gpurun_out/bl_eng_$B.json --dtype bf16 --batch $B > gpurun_out/bl_tr_$B.log 2>&1 || { echo "trace $B failed"; tail -5 gpurun_out/bl_tr_$B.log; exit 4; }
  GF=$(python -c "import json; print(json.load(open('gpurun_out/bl_eng_$B.json'))['gflop'])")
  python tools/replay_breakdown.py gpurun_out/bl_tr_$B 10 --gflop $GF --out gpurun_out/bl_breakdown_$B.txt > /dev/null || exit 5
  python tools/step_lanes.py gpurun_out/bl_tr_$B 3 > gpurun_out/bl_lanes_$B.txt || exit 6
  head -3 gpurun_out/bl_breakdown_$B.txt
  find gpurun_out/bl_tr_$B -name "*kernel_trace.csv" -delete
done
exit 0
