#!/bin/bash
# Training iteration of one library under several env settings, interleaved, N rounds
#   tools/ab_train_env.sh N LIB "VAR=val VAR2=val" ...   (LIB "" = the working tree's; setting "-" = none)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
N=$1; LIB=$2; shift 2
for i in $(seq $N); do
  for setting in "$@"; do
    envs=""; [ "$setting" != "-" ] && envs="$setting"
    env ${LIB:+A2M_LIB=$PWD/$LIB} $envs timeout -k 10 300 python bench.py --mode train --steps ${TRAIN_STEPS:-5} --warmup ${TRAIN_WARMUP:-2} ${TRAIN_ARGS:-} > gpurun_out/abte.log 2>&1 || { echo "fail $setting"; tail -3 gpurun_out/abte.log; exit 3; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/abte.log').read().strip().splitlines()[-1]); print(sys.argv[1], sys.argv[2], d['ms_per_step'])" "${LIB:-new}" "$setting"
  done
done
