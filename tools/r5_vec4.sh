#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A2M_LIB=$PWD/_ab/stamps.so timeout -k 10 120 python tools/pipe_stamps.py 2>&1 | grep -E "gemm|conv"
NOTEST= bash tools/ab_round.sh _ab/base.so 3 2>&1 | grep -vE "^pipe (gemm|conv)"
