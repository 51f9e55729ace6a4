#!/bin/bash
# bf16 graph stack: weights as ready bf16 fragments (diagnostic _ab/abl5.so, wrong values, same
# traffic as a pre-packed bf16 weight copy) vs the in-tree fp32 loads + packing: the upper bound
# of a bf16 weight cache.  tools/stack_bench.py, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2 3; do
  for lib in $PWD/audio-to-motion-generation_amd/a2m/liba2m_hip.so $PWD/_ab/abl5.so; do
    echo "$(basename $lib) $(A2M_LIB=$lib timeout -k 10 120 python tools/stack_bench.py both 50 bf16 | tr '\n' ' ')"
  done
done
