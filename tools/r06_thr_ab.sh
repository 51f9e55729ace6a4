#!/bin/bash
# fp32 planner constants re-fit probe: the 64x64 tile's throughput x1.15 / x0.90 and no gathered
# penalty, against the in-tree fit; fp32 bench lines (and each variant's plan count), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L0=$PWD/audio-to-motion-generation_amd/a2m/liba2m_hip.so
for i in 1 2 3; do
  for lib in $L0 $PWD/_ab/thr115.so $PWD/_ab/thr090.so $PWD/_ab/gf100.so; do
    A2M_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-trace --steps 300 > gpurun_out/th_b.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/th_b.log; exit 3; }
    echo "$(basename $lib) fp32 $(python -c "import json; d=json.loads(open('gpurun_out/th_b.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['reduces_per_step'], d['roofline']['launches_per_step'])")"
  done
done
exit 0
