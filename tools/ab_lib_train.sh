#!/bin/bash
# Interleaved A/B of the working tree's library against a baseline build on the training
# iteration (bench.py --mode train): N pairs.   tools/ab_lib_train.sh [pairs] [baseline.so]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
N=${1:-3}; BASE=${2:-_ab/liba2m_base.so}
for i in $(seq $N); do
  for lib in "$BASE" ""; do
    if [ -n "$lib" ]; then export A2M_LIB=$PWD/$lib; tag=base; else unset A2M_LIB; tag=new; fi
    timeout -k 10 300 python bench.py --mode train --steps 5 --warmup 2 > gpurun_out/ablibt.log 2>&1 || { echo "fail $tag"; tail -3 gpurun_out/ablibt.log; exit 3; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/ablibt.log').read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'])" $tag
  done
done
unset A2M_LIB
