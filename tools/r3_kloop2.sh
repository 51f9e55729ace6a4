set -o pipefail
cd $GRAFT_REPO_ROOT
A2M_GEMM_GLDS=1 timeout -k 10 120 python tools/gemm_bench.py 300,1000,500 128,22528,1024 2>&1 | grep gemm || exit 2
A2M_GEMM_GLDS=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/g_parity.log 2>&1; rc=$?; tail -1 gpurun_out/g_parity.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/g_parity.log | head; exit $rc; }
for spec in "128:128,32768,4096 128,65536,4096" "12864:128,16384,4096 128,32768,4096" "64:64,16384,4096 64,32768,4096"; do
  t=${spec%%:*}; sh=${spec#*:}
  echo "== GLDS=1 tile $t"
  A2M_GEMM_GLDS=1 A2M_GEMM_TILE=$t A2M_GEMM_SPLIT=1 A2M_GEMM_KS2=0 timeout -k 10 200 python tools/gemm_bench.py $sh 2>&1 | grep gemm || exit 3
done
SH="128,22528,1024 256,5120,2048 512,4096,2304 256,512,12288 256,4096,768 2560,2048,2048 4096,4096,4096"
A2M_GEMM_GLDS=1 timeout -k 10 300 python tools/gemm_bench.py $SH 2>&1 | grep gemm || exit 4
A2M_GEMM_GLDS=1 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/g_bench.json 2>/dev/null || exit 5
python -c "import json;d=json.load(open('gpurun_out/g_bench.json'));print('step',d['ms_per_step'],'gemm',d['roofline']['achieved'],'enc_ms',d['mel_encoder_roofline']['encoder_ms'],'path_frac',d['mel_encoder_roofline']['path_frac'])"
