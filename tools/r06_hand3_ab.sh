#!/bin/bash
# bf16 stack occupancy per graph: hand (J = 42) at 3 workgroups per CU, body at 2 (_ab/hand3.so) vs
# both at 2 (in-tree); bf16 bench lines, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L0=$PWD/audio-to-motion-generation_amd/a2m/liba2m_hip.so
for i in 1 2 3; do
  for lib in $L0 $PWD/_ab/hand3.so; do
    A2M_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-trace --steps 300 --dtype bf16 > gpurun_out/h3_b64.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/h3_b64.log; exit 3; }
    A2M_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-trace --steps 300 --dtype bf16 --batch 32 > gpurun_out/h3_b32.log 2>&1 || { echo "bench b32 failed"; exit 3; }
    echo "$(basename $lib) bf16 B=64 $(python -c "import json; print(json.loads(open('gpurun_out/h3_b64.log').read().strip().splitlines()[-1])['ms_per_step'])") B=32 $(python -c "import json; print(json.loads(open('gpurun_out/h3_b32.log').read().strip().splitlines()[-1])['ms_per_step'])")"
  done
done
exit 0
