#!/bin/bash
# rocprof passes over exactly the bench step (tools/step_pmc.py), counting only the graph-replayed
# steps after its marker kernel (tools/replay_filter.py): a kernel-trace/stats pass over replays
# each followed by a device sync (step_pmc.py --sync: free-running replays slow down under the
# trace) for the per-step breakdown and the GEMM engine's in-step roofline
# (tools/replay_breakdown.py), FETCH_SIZE,
# WRITE_SIZE, MFMA busy + GRBM cycles; then per-launch HBM traffic and MFMA utilisation per
# kernel family (tools/pmc_traffic.py, tools/pmc_mfma.py).   tools/step_pmc.sh TAG [--dtype bf16]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
TAG=$1; shift
R=${STEP_PMC_REPS:-10}
OUT=gpurun_out/steppmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/$OUT/trace -o run -- python tools/step_pmc.py $R --sync --engine-json $OUT/engine.json "$@" > $OUT/trace.log 2>&1 || { echo trace failed; tail -5 $OUT/trace.log; exit 2; }
GF=$(python -c "import json; print(json.load(open('$OUT/engine.json'))['gflop'])")
python tools/replay_breakdown.py $OUT/trace $R --gflop $GF --out $OUT/breakdown.txt > /dev/null || exit 8
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $REPO/$OUT/fetch -o run -- python tools/step_pmc.py 3 "$@" > $OUT/fetch.log 2>&1 || { echo fetch failed; tail -5 $OUT/fetch.log; exit 3; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $REPO/$OUT/write -o run -- python tools/step_pmc.py 3 "$@" > $OUT/write.log 2>&1 || { echo write failed; tail -5 $OUT/write.log; exit 4; }
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $REPO/$OUT/mfma -o run -- python tools/step_pmc.py 3 "$@" > $OUT/mfma.log 2>&1 || { echo mfma failed; tail -5 $OUT/mfma.log; exit 5; }
A2M_GEMM_LOG=1 timeout -k 10 120 python tools/plan_log.py "$@" > /dev/null 2> $OUT/plans.txt || { echo plan log failed; exit 9; }
python tools/pmc_traffic.py $OUT/fetch $OUT/write --steps 3 --plans $OUT/plans.txt --out $OUT/traffic.json --tag "$TAG (tools/step_pmc.sh)" > /dev/null || exit 6
python tools/pmc_mfma.py $OUT/mfma $OUT/trace --out $OUT/mfma.json > /dev/null || exit 7
find $OUT -name "*counter_collection.csv" -size +20M -delete
exit 0
