set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_tapconv.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c1_pytest.log 2>&1; rc=$?; tail -1 gpurun_out/c1_pytest.log; [ $rc -ne 0 ] && exit $rc
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/enc_tr3 -o run -- python tools/enc_trace.py > gpurun_out/enc_tr3.log 2>&1 || exit 5
grep -E "conv2d_c1|interp|splitk|gemm" gpurun_out/enc_tr3/run_kernel_stats.csv | cut -d, -f1-5
