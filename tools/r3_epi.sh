set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_grouped.py tests/test_gpu_train.py tests/test_gpu_configs.py tests/test_gpu_bf16.py tests/test_gpu_syncbn.py > gpurun_out/epi_tests.log 2>&1 || { tail -30 gpurun_out/epi_tests.log; exit 2; }
tail -1 gpurun_out/epi_tests.log
echo new; timeout -k 10 200 python tools/epi_probe.py
echo prev; A2M_LIB=$PWD/audio-to-motion-generation_amd/a2m/liba2m_prev.so timeout -k 10 200 python tools/epi_probe.py
bash tools/r3_lib_ab.sh 3
