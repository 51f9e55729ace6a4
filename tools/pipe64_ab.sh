# fp32 planner kept to the 64x64 tile where the pipelined tile takes the operands: tests, then the
# training iteration A/B (and the headline step, whose fp32 B=64 plans are all 64x64 already)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pipe.py tests/test_gpu_train.py > gpurun_out/p64_tests.txt 2>&1 || { tail -30 gpurun_out/p64_tests.txt; exit 3; }
tail -1 gpurun_out/p64_tests.txt
TRAIN_STEPS=20 TRAIN_WARMUP=3 bash tools/ab_train_env.sh 3 "" A2M_GEMM_PIPE64=0 A2M_GEMM_PIPE64=1 || exit 3
bash tools/ab_envs.sh A2M_GEMM_PIPE64 "0 1" 1
