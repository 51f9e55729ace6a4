#!/bin/bash
# The training graph layer (graph_layer_kernel) at 2 workgroups per CU (no spills; _ab/gl2.so) vs 3
# (in-tree, 9 VGPRs spilled): training lines fp32 B = 64 / B = 8 and bf16 B = 32, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L0=$PWD/audio-to-motion-generation_amd/a2m/liba2m_hip.so
for i in 1 2; do
  for lib in $L0 $PWD/_ab/gl2.so; do
    A2M_LIB=$lib timeout -k 10 300 python bench.py --mode train --steps 10 --warmup 5 > gpurun_out/gl_t64.log 2>&1 || { echo "train failed"; tail -5 gpurun_out/gl_t64.log; exit 3; }
    A2M_LIB=$lib timeout -k 10 300 python bench.py --mode train --steps 10 --warmup 5 --batch 8 > gpurun_out/gl_t8.log 2>&1 || { echo "train b8 failed"; exit 3; }
    A2M_LIB=$lib timeout -k 10 300 python bench.py --mode train --steps 10 --warmup 5 --batch 32 --dtype bf16 > gpurun_out/gl_t32.log 2>&1 || { echo "train bf16 failed"; exit 3; }
    echo "$(basename $lib) fp32 B=64 $(python -c "import json; print(json.loads(open('gpurun_out/gl_t64.log').read().strip().splitlines()[-1])['ms_per_step'])") B=8 $(python -c "import json; print(json.loads(open('gpurun_out/gl_t8.log').read().strip().splitlines()[-1])['ms_per_step'])") bf16 B=32 $(python -c "import json; print(json.loads(open('gpurun_out/gl_t32.log').read().strip().splitlines()[-1])['ms_per_step'])")"
  done
done
exit 0
