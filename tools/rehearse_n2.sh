#!/bin/bash
# Rehearsal of the driver's N = 2 bench on a 1-GPU box: two gloo ranks spawned by bench.py --gpus 2
# (inference replicas and the DP training iteration with bucketed gradient all-reduces).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export A2M_BENCH_BACKEND=gloo
timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/reh_inf.log 2>&1 || { tail -5 gpurun_out/reh_inf.log; exit 2; }
tail -1 gpurun_out/reh_inf.log
timeout -k 10 300 python bench.py --gpus 2 --mode train --steps 3 --warmup 1 > gpurun_out/reh_train.log 2>&1 || { tail -5 gpurun_out/reh_train.log; exit 3; }
tail -1 gpurun_out/reh_train.log
