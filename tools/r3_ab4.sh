set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab4_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/ab4_pytest.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/ab4_pytest.log | head -20; exit $rc; fi
for i in 1 2; do for v in 0 1; do
  A2M_C1_MFMA=$v timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ab_bench.json 2>/dev/null || exit 4
  echo "c1mfma$v $(python -c "import json;d=json.load(open('gpurun_out/ab_bench.json'));print('step',d['ms_per_step'],'gemm',d['roofline']['achieved'],'enc_ms',d['mel_encoder_roofline']['encoder_ms'],'path_frac',d['mel_encoder_roofline']['path_frac'])")"
done; done
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/enc_tr2 -o run -- python tools/enc_trace.py > gpurun_out/enc_tr2.log 2>&1 || exit 5
grep -E "conv2d_c1|interp|splitk|gemm" gpurun_out/enc_tr2/run_kernel_stats.csv | cut -d, -f1-5
