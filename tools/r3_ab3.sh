set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_eval.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab3_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/ab3_pytest.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/ab3_pytest.log | head -20; exit $rc; fi
for i in 1 2; do for v in 1 2 4; do
  A2M_ENC_SPLIT=$v timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ab_bench.json 2>/dev/null || exit 4
  echo "split$v $(python -c "import json;d=json.load(open('gpurun_out/ab_bench.json'));print('step',d['ms_per_step'],'gemm',d['roofline']['achieved'],'enc_ms',d['mel_encoder_roofline']['encoder_ms'],'path_frac',d['mel_encoder_roofline']['path_frac'])")"
done; done
