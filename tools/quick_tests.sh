set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pipe.py tests/test_gpu_train.py tests/test_gpu_bf16.py > gpurun_out/quick_tests.txt 2>&1; rc=$?
tail -2 gpurun_out/quick_tests.txt; exit $rc
