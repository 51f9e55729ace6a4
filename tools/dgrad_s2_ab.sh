# strided conv1d dgrad as ConvTranspose tap phases: tests, traces, training A/B
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_pipe.py > gpurun_out/ds2_tests.txt 2>&1 || { tail -30 gpurun_out/ds2_tests.txt; exit 3; }
tail -1 gpurun_out/ds2_tests.txt
bash tools/train_trace.sh > gpurun_out/train_trace_run.txt 2>&1 || { tail -5 gpurun_out/train_trace_run.txt; exit 3; }
grep -E "total" gpurun_out/train_breakdown_fp32_b64.txt gpurun_out/train_breakdown_bf16_b32.txt
TRAIN_STEPS=20 TRAIN_WARMUP=3 bash tools/ab_train_env.sh 2 "" A2M_DGRAD_TAP=0 -
