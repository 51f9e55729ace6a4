# in-call A/B of engine variants (box-to-box clock spread is 10-20 %: compare only within a call)
set -o pipefail
cd $GRAFT_REPO_ROOT
SH="128,32768,4096 64,16384,4096 128,22528,1024 256,5120,2048 512,4096,2304 256,512,12288 256,4096,768 2560,2048,2048"
for v in "A2M_GEMM_GLDS=0" "A2M_GEMM_GLDS=1" "A2M_GEMM_GLDS=1 A2M_GLDS_INTER=1" "A2M_GEMM_GLDS=0" "A2M_GEMM_GLDS=1 A2M_GLDS_INTER=1" "A2M_GEMM_GLDS=1"; do
  echo "== $v"; env $v timeout -k 10 300 python tools/gemm_bench.py $SH 2>&1 | grep gemm || exit 3
done | tee gpurun_out/r3_ab.txt
