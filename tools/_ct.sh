#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k convt -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_ct.log 2>&1 || { tail -30 gpurun_out/pt_ct.log; exit 3; }
tail -1 gpurun_out/pt_ct.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_ct_all.log 2>&1 || { tail -30 gpurun_out/pt_ct_all.log; exit 4; }
tail -1 gpurun_out/pt_ct_all.log
timeout -k 10 200 python tools/shape_probe.py > gpurun_out/shape_probe2.txt 2>&1 || exit 5
grep convT gpurun_out/shape_probe2.txt
A2M_GEMM_LOG=2 timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/gl4.out 2> gpurun_out/gemmtime4.txt || exit 6
bash tools/ab_env.sh A2M_CONVT_TAP=0 4
