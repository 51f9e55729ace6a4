set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tapconv.py tests/test_gpu_parity.py tests/test_gpu_eval.py tests/test_gpu_grouped.py > gpurun_out/m5_tests.log 2>&1 || { tail -30 gpurun_out/m5_tests.log; exit 2; }
tail -1 gpurun_out/m5_tests.log
echo new; timeout -k 10 200 python tools/conv_scaling.py
echo prev; A2M_LIB=$PWD/audio-to-motion-generation_amd/a2m/liba2m_prev.so timeout -k 10 200 python tools/conv_scaling.py
bash tools/r3_lib_ab.sh 3
