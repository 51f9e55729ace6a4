#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_ks3.log 2>&1 || { tail -30 gpurun_out/pt_ks3.log; exit 3; }
tail -2 gpurun_out/pt_ks3.log
for v in 0 1; do A2M_GEMM_KS3=$v timeout -k 10 120 python tools/conv_plan_probe.py > gpurun_out/probe_ks3_$v.log 2>&1 || exit 4; echo "KS3=$v"; head -8 gpurun_out/probe_ks3_$v.log; done
bash tools/ab_env.sh A2M_GEMM_KS3=0 3
