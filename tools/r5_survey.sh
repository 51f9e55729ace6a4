#!/bin/bash
# One-call survey of the current build: engine plans of one eager step (fp32 and bf16) and the
# bf16 bench step's replayed kernel trace with its per-step breakdown.   tools/r5_survey.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
TAG=${1:-survey}
OUT=gpurun_out/survey_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
A2M_GEMM_LOG=1 timeout -k 10 120 python tools/plan_log.py > /dev/null 2> $OUT/plans_fp32.txt || { echo plan fp32 failed; tail -5 $OUT/plans_fp32.txt; exit 2; }
A2M_GEMM_LOG=1 timeout -k 10 120 python tools/plan_log.py bf16 > /dev/null 2> $OUT/plans_bf16.txt || { echo plan bf16 failed; tail -5 $OUT/plans_bf16.txt; exit 3; }
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/$OUT/trace_bf16 -o run -- python tools/step_pmc.py 10 --sync --engine-json $OUT/engine_bf16.json --dtype bf16 > $OUT/trace_bf16.log 2>&1 || { echo trace failed; tail -5 $OUT/trace_bf16.log; exit 4; }
python tools/replay_breakdown.py $OUT/trace_bf16 10 --out $OUT/breakdown_bf16.txt > /dev/null || exit 5
head -30 $OUT/breakdown_bf16.txt
exit 0
