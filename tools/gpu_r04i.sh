#!/bin/bash
# stamps vs rocprof kernel trace on the same replayed steps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=gpurun_out/r04i_svt
mkdir -p $OUT
export TMPDIR=/tmp
A2M_GEMM_TIMING_READY=1 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $REPO/$OUT/trace -o run -- python tools/step_pmc.py 10 --sync --stamps $OUT/stamps.json > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
python tools/stamp_vs_trace.py $OUT/trace $OUT/stamps.json --out $OUT/stamp_vs_trace.txt
find $OUT -name "*kernel_trace.csv" -size +20M -delete
exit 0
