#!/bin/bash
# tools/stack_bench.py under several library builds, interleaved: tools/stack_libs.sh "a.so b.so" [rounds]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LIBS=$1; N=${2:-2}
for i in $(seq $N); do
  for lib in $LIBS; do
    A2M_LIB=$PWD/$lib timeout -k 10 120 python tools/stack_bench.py both 50 2>&1 | grep stack | sed "s|^|$(basename $lib .so) |" || exit 3
  done
done
