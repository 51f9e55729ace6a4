#!/bin/bash
# Per-shape engine times of one fp32 B=64 training iteration (tools/train_gemm_times.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A2M_GEMM_LOG=2 timeout -k 10 300 python tools/train_gemm_times.py > gpurun_out/tg.out 2> gpurun_out/tg.log || { tail -5 gpurun_out/tg.log; exit 1; }
cat gpurun_out/tg.out
python tools/train_gemm_times.py --summarise gpurun_out/tg.log > gpurun_out/tg_summary.txt
rm -f gpurun_out/tg.log
head -45 gpurun_out/tg_summary.txt
