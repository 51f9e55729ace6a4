#!/bin/bash
# Engine span stamps vs the rocprof kernel trace of the same replayed bench steps, launch by
# launch (tools/stamp_vs_trace.py).   tools/stamp_trace.sh TAG [--ready]
# --ready: also the ready marks (A2M_GEMM_TIMING_READY=1: one extra kernel per engine launch)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=gpurun_out/svt_$1
mkdir -p $OUT
export TMPDIR=/tmp
[ "${2:-}" = "--ready" ] && export A2M_GEMM_TIMING_READY=1
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $REPO/$OUT/trace -o run -- python tools/step_pmc.py 10 --sync --stamps $OUT/stamps.json > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
python tools/stamp_vs_trace.py $OUT/trace $OUT/stamps.json --out $OUT/stamp_vs_trace.txt
