# bf16 pipelined tile on the training modes (mode-4 runs, plain mode-3 A): tests, then the bf16
# B=32 training iteration with / without (both switches), interleaved
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pipe.py tests/test_gpu_train.py tests/test_gpu_bf16.py > gpurun_out/bf16p_tests.txt 2>&1 || { tail -30 gpurun_out/bf16p_tests.txt; exit 3; }
tail -1 gpurun_out/bf16p_tests.txt
TRAIN_STEPS=30 TRAIN_WARMUP=5 TRAIN_ARGS="--dtype bf16 --batch 32" bash tools/ab_train_env.sh 3 "" "A2M_GEMM_PIPE4=0 A2M_GEMM_PIPE_A3=0" -
