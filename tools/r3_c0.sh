set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tapconv.py tests/test_gpu_eval.py -k "nhwc or eval or generator or c1 or conv2d" > gpurun_out/c0_tests.log 2>&1 || { tail -30 gpurun_out/c0_tests.log; exit 2; }
tail -1 gpurun_out/c0_tests.log
for v in new prev; do
if [ $v = prev ]; then export A2M_LIB=$PWD/audio-to-motion-generation_amd/a2m/liba2m_prev.so; else unset A2M_LIB; fi
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $PWD/gpurun_out/c0_$v -o run -- python tools/enc_trace.py > gpurun_out/c0_$v.log 2>&1 || { tail -5 gpurun_out/c0_$v.log; exit 3; }
echo "$v: $(grep 'encoder graph' gpurun_out/c0_$v.log)"; python tools/prof_summary.py gpurun_out/c0_$v/run_kernel_trace.csv 31 | grep conv2d_c1
done
unset A2M_LIB
bash tools/r3_lib_ab.sh 3
