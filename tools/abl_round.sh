#!/bin/bash
# pipe-kernel ablations: the per-launch probe with each diagnostic library (tools/build_variant.sh)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in "" $@; do
  if [ -z "$lib" ]; then name=base; else name=$lib; fi
  env ${lib:+A2M_LIB=_ab/$lib.so} timeout -k 10 150 python tools/pipe_probe.py > gpurun_out/abl_$name.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "rc $rc $name"; tail -3 gpurun_out/abl_$name.log; exit $rc; }
  echo "== $name"; grep -E "gemm 256x4096|conv1d B=64 Ci=(256|512) Co=256|gemm-kr 2688|nhwc" gpurun_out/abl_$name.log | cut -c1-70
done
