#!/bin/bash
# A/B of the bf16 planner's split-K reduce fixed cost (3 us in-tree vs _ab/rb6.so, _ab/rb12.so):
# bf16 inference at B = 32 / 64 and bf16 B = 32 training, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L0=$PWD/audio-to-motion-generation_amd/a2m/liba2m_hip.so
for i in 1 2; do
  for lib in $L0 $PWD/_ab/rb6.so $PWD/_ab/rb12.so; do
    n=$(basename $lib .so)
    A2M_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-trace --steps 200 --dtype bf16 --batch 32 > gpurun_out/rb_32.log 2>&1 || { echo "b32 $n failed"; tail -3 gpurun_out/rb_32.log; exit 3; }
    A2M_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-trace --steps 200 --dtype bf16 > gpurun_out/rb_64.log 2>&1 || { echo "b64 $n failed"; exit 3; }
    A2M_LIB=$lib timeout -k 10 300 python bench.py --mode train --steps 10 --warmup 5 --dtype bf16 --batch 32 > gpurun_out/rb_tr.log 2>&1 || { echo "tr $n failed"; exit 3; }
    python - $n <<'PY'
import json, sys
g = lambda f: json.loads(open(f).read().strip().splitlines()[-1])
a, b, c = g('gpurun_out/rb_32.log'), g('gpurun_out/rb_64.log'), g('gpurun_out/rb_tr.log')
print(sys.argv[1], 'bf16 infer B=32', a['ms_per_step'], 'reduces', a['roofline'].get('reduces_per_step'), 'B=64', b['ms_per_step'], 'train B=32', c['ms_per_step'])
PY
  done
done
