set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab2_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/ab2_pytest.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/ab2_pytest.log | head -20; exit $rc; fi
R02=$PWD/audio-to-motion-generation_amd/a2m/liba2m_r02.so
for i in 1 2 3; do for v in r02 cur all0; do
  unset A2M_LIB A2M_ENC_NHWC_ALL
  [ $v = r02 ] && export A2M_LIB=$R02 A2M_ENC_NHWC_ALL=0
  [ $v = all0 ] && export A2M_ENC_NHWC_ALL=0
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ab_bench.json 2>/dev/null || exit 4
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/ab_bench.json'));print('step',d['ms_per_step'],'gemm',d['roofline']['achieved'],'enc_ms',d['mel_encoder_roofline']['encoder_ms'],'path_frac',d['mel_encoder_roofline']['path_frac'])")"
done; done
