#!/bin/bash
# bf16 graph stack at 2 workgroups per CU (256 VGPRs, no spills; _ab/wg2.so) vs 3 (in-tree: 168
# VGPRs + 114 spilled), now that its weights come as cached bf16 copies; stack_bench and bf16 lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L0=$PWD/audio-to-motion-generation_amd/a2m/liba2m_hip.so
for i in 1 2; do
  for lib in $L0 $PWD/_ab/wg2.so; do
    echo "$(basename $lib) $(A2M_LIB=$lib timeout -k 10 120 python tools/stack_bench.py both 50 bf16 | tr '\n' ' ')"
  done
done
for i in 1 2 3; do
  for lib in $L0 $PWD/_ab/wg2.so; do
    A2M_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-trace --steps 300 --dtype bf16 > gpurun_out/wg_b64.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/wg_b64.log; exit 3; }
    A2M_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-trace --steps 300 --dtype bf16 --batch 32 > gpurun_out/wg_b32.log 2>&1 || { echo "bench b32 failed"; exit 3; }
    echo "$(basename $lib) bf16 B=64 $(python -c "import json; print(json.loads(open('gpurun_out/wg_b64.log').read().strip().splitlines()[-1])['ms_per_step'])") B=32 $(python -c "import json; print(json.loads(open('gpurun_out/wg_b32.log').read().strip().splitlines()[-1])['ms_per_step'])")"
  done
done
exit 0
