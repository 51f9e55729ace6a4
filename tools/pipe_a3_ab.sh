# A in mode 3 on the pipelined tile: pipe-vs-tile tests, training tests, plans, iteration A/B
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pipe.py > gpurun_out/pipe_tests.txt 2>&1 || { tail -30 gpurun_out/pipe_tests.txt; exit 3; }
tail -1 gpurun_out/pipe_tests.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_train.py > gpurun_out/train_tests.txt 2>&1 || { tail -30 gpurun_out/train_tests.txt; exit 3; }
tail -1 gpurun_out/train_tests.txt
A2M_GEMM_LOG=1 timeout -k 10 300 python bench.py --mode train --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/train_plans.out 2> gpurun_out/train_plans.txt || { tail -5 gpurun_out/train_plans.txt; exit 3; }
grep -c "(pipe) modes=3" gpurun_out/train_plans.txt
TRAIN_STEPS=20 TRAIN_WARMUP=3 bash tools/ab_train_env.sh 3 "" A2M_GEMM_PIPE_A3=0 A2M_GEMM_PIPE_A3=1 "A2M_GEMM_PIPE_A3=1 A2M_GEMM_TILE=64"
