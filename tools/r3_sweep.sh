set -o pipefail
cd $GRAFT_REPO_ROOT
SH="128,22528,1024 256,5120,2048 512,4096,2304 256,512,12288 256,4096,768 2560,2048,2048"
for k in 0 2 3; do
  echo "== KS128=$k"
  A2M_GEMM_KS128=$k SWEEP=1 timeout -k 10 300 python tools/gemm_bench.py $SH 2>&1 | grep gemm || exit 2
done | tee gpurun_out/r3_sweep.txt
