#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_ks3.log 2>&1 || { tail -30 gpurun_out/pt_ks3.log; exit 3; }
tail -2 gpurun_out/pt_ks3.log
bash tools/ab_env.sh A2M_GEMM_KS3=1 4
