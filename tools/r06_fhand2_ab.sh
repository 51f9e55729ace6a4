#!/bin/bash
# fp32 stack occupancy per graph: hand (J = 42) at 2 workgroups per CU, body at 3 (_ab/fhand2.so) vs
# both at 3 (in-tree); fp32 bench lines, four interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L0=$PWD/audio-to-motion-generation_amd/a2m/liba2m_hip.so
for i in 1 2 3 4; do
  for lib in $L0 $PWD/_ab/fhand2.so; do
    A2M_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-trace --steps 300 > gpurun_out/fh_b.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/fh_b.log; exit 3; }
    echo "$(basename $lib) fp32 $(python -c "import json; print(json.loads(open('gpurun_out/fh_b.log').read().strip().splitlines()[-1])['ms_per_step'])")"
  done
done
exit 0
