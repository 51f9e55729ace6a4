#!/bin/bash
# Two round-3/4 constants re-measured on the round-6 kernels: the encoder's split-K reduce price
# (A2M_RED_SCALE_ROWS 2.0 in-tree vs 1.0, _ab/rsr1.so) and the fp32 graph stack's MFMA / VALU
# interleave hint (STACK_IGLP 2 in-tree vs none, _ab/iglpn.so); fp32 bench lines, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L0=$PWD/audio-to-motion-generation_amd/a2m/liba2m_hip.so
for i in 1 2 3; do
  for lib in $L0 $PWD/_ab/rsr1.so $PWD/_ab/iglpn.so; do
    A2M_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-trace --steps 300 > gpurun_out/cs_b.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/cs_b.log; exit 3; }
    echo "$(basename $lib) fp32 $(python -c "import json; d=json.loads(open('gpurun_out/cs_b.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['mel_encoder_roofline']['path_frac_instep'])")"
  done
done
exit 0
