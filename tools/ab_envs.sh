#!/bin/bash
# Interleaved bench runs over several settings of one switch (N rounds):
#   tools/ab_envs.sh VAR "v1 v2 ..." [rounds]
# prints ms/step, GEMM frac, encoder ms, path_frac (isolated / in-step) per run
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VAR=$1; VALS=$2; N=${3:-3}
for i in $(seq $N); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-trace --steps 100 ${BENCH_ARGS:-} > gpurun_out/abenvs.log 2>&1 || { echo "fail $VAR=$v"; tail -5 gpurun_out/abenvs.log; exit 3; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/abenvs.log').read().strip().splitlines()[-1]); r=d['roofline']; m=d['mel_encoder_roofline']; print(sys.argv[1], d['ms_per_step'], 'gemm', r['frac'], 'enc_ms', m['encoder_ms'], 'path', m['path_frac'], 'instep', m.get('path_frac_instep'))" "$VAR=$v"
  done
done
