#!/bin/bash
# GEMM k-loop ablation (diagnostic): the same shapes timed on the shipped library and on
# builds with -DA2M_ABLATE=1 (no MFMAs) / 2 (no global loads after the prologue) / 3 (no
# barriers).  Build the variants first:
#   for k in 1 2 3; do make -C audio-to-motion-generation_amd BUILD=build_ab$k OUT=a2m/liba2m_ab$k.so EXTRA=-DA2M_ABLATE=$k; done
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LIB=audio-to-motion-generation_amd/a2m
for v in hip ab1 ab2 ab3; do
  echo "== $v"
  A2M_LIB=$PWD/$LIB/liba2m_$v.so timeout -k 10 120 python tools/gemm_bench.py "$@" 2>&1 | grep gemm || exit 2
done
