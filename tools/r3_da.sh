set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in 1 2; do
A2M_GEMM_DA=$v timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tapconv.py tests/test_gpu_parity.py tests/test_gpu_eval.py > gpurun_out/da_tests$v.log 2>&1 || { tail -30 gpurun_out/da_tests$v.log; exit 2; }
echo "DA=$v $(tail -1 gpurun_out/da_tests$v.log)"
done
for v in 0 1; do echo "== DA=$v"; A2M_GEMM_DA=$v timeout -k 10 200 python tools/conv_scaling.py; done
for v in 0 2; do echo "== DA=$v"; A2M_GEMM_DA=$v timeout -k 10 200 python tools/epi_probe.py; done
bash tools/r3_ab_long.sh A2M_GEMM_DA "0 1 2" 2
