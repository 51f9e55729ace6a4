set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
A2M_GEMM_KS3_SKEW=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tapconv.py tests/test_gpu_parity.py tests/test_gpu_eval.py > gpurun_out/skew_tests.log 2>&1 || { tail -30 gpurun_out/skew_tests.log; exit 2; }
tail -1 gpurun_out/skew_tests.log
for v in 0 1 0 1; do echo "skew=$v"; A2M_GEMM_KS3_SKEW=$v timeout -k 10 200 python tools/epi_probe.py | tail -1; done
bash tools/r3_ab_long.sh A2M_GEMM_KS3_SKEW "0 1" 3
