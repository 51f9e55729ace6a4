#!/bin/bash
# A/B of the planner's split-K reduce fixed cost (3 us in-tree vs _ab/red6.so, _ab/red10.so):
# training B=8 / B=64 and the inference bench, interleaved.   tools/r06_red_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -m gpu -x -q --timeout 300 --timeout-method thread -k "loss or motion or pose or train_step" > gpurun_out/pytest_red.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_red.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_red.log | head -20; exit 1; }
L0=$PWD/audio-to-motion-generation_amd/a2m/liba2m_hip.so
for i in 1 2; do
  for lib in $L0 $PWD/_ab/red6.so $PWD/_ab/red10.so; do
    n=$(basename $lib .so)
    A2M_LIB=$lib timeout -k 10 300 python bench.py --mode train --steps 20 --warmup 5 --batch 8 > gpurun_out/red_b8.log 2>&1 || { echo "b8 $n failed"; tail -3 gpurun_out/red_b8.log; exit 3; }
    A2M_LIB=$lib timeout -k 10 300 python bench.py --mode train --steps 10 --warmup 5 > gpurun_out/red_b64.log 2>&1 || { echo "b64 $n failed"; exit 3; }
    A2M_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-trace --steps 200 > gpurun_out/red_inf.log 2>&1 || { echo "inf $n failed"; exit 3; }
    python - $n <<'PY'
import json, sys
g = lambda f: json.loads(open(f).read().strip().splitlines()[-1])['ms_per_step']
print(sys.argv[1], 'train B=8', g('gpurun_out/red_b8.log'), 'B=64', g('gpurun_out/red_b64.log'), 'infer B=64', g('gpurun_out/red_inf.log'))
PY
  done
done
