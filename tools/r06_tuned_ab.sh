#!/bin/bash
# The fp32 hand-tuned plan table (kTunedPlans, fitted in rounds 4-5) vs the planner alone
# (_ab/notuned.so), fp32 inference and training, interleaved; plus each one's plan log.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L0=$PWD/audio-to-motion-generation_amd/a2m/liba2m_hip.so
A2M_LIB=$PWD/_ab/notuned.so A2M_GEMM_LOG=1 timeout -k 10 120 python tools/plan_log.py > /dev/null 2> gpurun_out/tu_plans_notuned.txt || exit 1
for i in 1 2 3; do
  for lib in $L0 $PWD/_ab/notuned.so; do
    A2M_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-trace --steps 300 > gpurun_out/tu_b.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/tu_b.log; exit 3; }
    echo "$(basename $lib) fp32 $(python -c "import json; print(json.loads(open('gpurun_out/tu_b.log').read().strip().splitlines()[-1])['ms_per_step'])")"
  done
done
for lib in $L0 $PWD/_ab/notuned.so; do
  A2M_LIB=$lib timeout -k 10 300 python bench.py --mode train --steps 10 --warmup 5 > gpurun_out/tu_t.log 2>&1 || { echo "train failed"; exit 3; }
  echo "$(basename $lib) train $(python -c "import json; print(json.loads(open('gpurun_out/tu_t.log').read().strip().splitlines()[-1])['ms_per_step'])")"
done
exit 0
