#!/bin/bash
# Interleaved A/B of one experiment switch against the defaults (N pairs of 100-step bench runs).
#   tools/ab_env.sh "A2M_X=0" [pairs]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFG=$1; N=${2:-4}
for i in $(seq $N); do
  for cfg in "" "$CFG"; do
    env $cfg timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 > gpurun_out/abenv.log 2>&1 || { echo "fail $cfg"; exit 3; }
    echo "[$cfg] $(python -c "import json; print(json.loads(open('gpurun_out/abenv.log').read().strip().splitlines()[-1])['ms_per_step'])")"
  done
done
