#!/bin/bash
# Kernel trace of the bench step with the decoder branches serialised (A2M_BRANCH_STREAMS=0),
# so every launch's duration is its own (no concurrent kernel shares the CUs).
#   tools/serial_prof.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
TAG=${1:-serial}
OUT=gpurun_out/serial_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
A2M_BRANCH_STREAMS=0 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $REPO/$OUT/trace -o run -- python tools/step_pmc.py 3 > $OUT/trace.log 2>&1 || { echo trace failed; tail -5 $OUT/trace.log; exit 2; }
python tools/step_ops.py $OUT/trace/run_kernel_trace.csv > $OUT/ops.txt && cat $OUT/ops.txt | tail -100
