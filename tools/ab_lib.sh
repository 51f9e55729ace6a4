#!/bin/bash
# Interleaved A/B of the working tree's library against a baseline build (tools/build_ab_lib.sh):
# N pairs of 100-step bench runs in one call (box clocks differ between calls).
#   tools/ab_lib.sh [pairs] [baseline.so] [extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
N=${1:-3}; BASE=${2:-_ab/liba2m_base.so}; shift 2 2>/dev/null || shift $#
for i in $(seq $N); do
  for lib in "$BASE" ""; do
    if [ -n "$lib" ]; then export A2M_LIB=$PWD/$lib; tag=base; else unset A2M_LIB; tag=new; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-trace --steps 100 "$@" > gpurun_out/ablib.log 2>&1 || { echo "fail $tag"; tail -3 gpurun_out/ablib.log; exit 3; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/ablib.log').read().strip().splitlines()[-1]); r=d['roofline']; m=d['mel_encoder_roofline']; print(sys.argv[1], d['ms_per_step'], 'gemm', r['frac'], 'enc_ms', m['encoder_ms'], 'path', m['path_frac'], 'instep', m.get('path_frac_instep'))" $tag
  done
done
unset A2M_LIB
