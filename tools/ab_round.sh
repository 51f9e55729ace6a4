#!/bin/bash
# GPU tests + per-launch probe (baseline lib vs working tree) + interleaved bench pairs
#   tools/ab_round.sh BASE.so [pairs]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
BASE=$1; N=${2:-3}
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2"; exit $1;; esac; }
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ab.log; fatal $rc pytest
  [ $rc -ne 0 ] && exit $rc
fi
for lib in "$BASE" ""; do
  tag=${lib:+base}; tag=${tag:-new}
  env ${lib:+A2M_LIB=$PWD/$lib} timeout -k 10 150 python tools/pipe_probe.py > gpurun_out/probe_$tag.log 2>&1
  rc=$?; fatal $rc probe
  echo "== $tag"; grep -vE "amdgpu.ids" gpurun_out/probe_$tag.log | cut -c1-64
done
bash tools/ab_lib.sh $N $BASE
