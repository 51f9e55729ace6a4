set -o pipefail
cd $GRAFT_REPO_ROOT
SH="128,22528,1024 256,5120,2048 512,4096,2304 256,512,12288 256,4096,768 2560,2048,2048 4096,4096,4096"
A2M_GEMM_GLDS=1 timeout -k 10 120 python tools/gemm_bench.py 300,1000,500 128,22528,1024 > gpurun_out/g_corr.txt 2>&1; cat gpurun_out/g_corr.txt | grep gemm || exit 2
A2M_GEMM_GLDS=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/g_parity.log 2>&1; rc=$?; tail -3 gpurun_out/g_parity.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/g_parity.log | head; exit $rc; }
for v in "A2M_GEMM_GLDS=0" "A2M_GEMM_GLDS=1" "A2M_GEMM_GLDS=1 A2M_GLDS_STAGES=4" "A2M_GEMM_GLDS=1 A2M_GLDS_STAGES=2"; do
  echo "== $v"; env $v timeout -k 10 300 python tools/gemm_bench.py $SH 2>&1 | grep gemm || exit 3
done | tee gpurun_out/g_perf.txt
for v in "A2M_GEMM_GLDS=0" "A2M_GEMM_GLDS=1"; do
  env $v timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/g_bench.json 2>/dev/null || exit 4
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/g_bench.json'));print('step',d['ms_per_step'],'gemm',d['roofline']['achieved'],'enc_ms',d['mel_encoder_roofline']['encoder_ms'],'path_frac',d['mel_encoder_roofline']['path_frac'])")"
done
