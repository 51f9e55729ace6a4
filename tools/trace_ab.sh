#!/bin/bash
# Kernel-trace breakdowns of the replayed bench step for a baseline library and the working tree
#   tools/trace_ab.sh BASE.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in "$1" ""; do
  tag=${lib:+base}; tag=${tag:-new}
  env ${lib:+A2M_LIB=$PWD/$lib} A2M_BENCH_TRACE_DIR=gpurun_out/tr_$tag timeout -k 10 300 python bench.py --no-cpu-baseline --steps 50 > gpurun_out/tr_$tag.json 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "rc $rc $tag"; tail -3 gpurun_out/tr_$tag.json; exit $rc; }
  echo "== $tag $(tail -1 gpurun_out/tr_$tag.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['frac'], d['mel_encoder_roofline'].get('path_frac_instep_trace'))")"
  head -22 gpurun_out/tr_$tag/step_breakdown.txt | cut -c1-100
done
