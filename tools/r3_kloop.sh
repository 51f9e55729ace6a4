set -o pipefail
cd $GRAFT_REPO_ROOT
# k-loop efficiency at exactly 1 and 2 blocks per CU (256 / 512 tiles, K = 4096, split 1)
for g in 0 1; do
for spec in "128:128,32768,4096 128,65536,4096" "12864:128,16384,4096 128,32768,4096" "64:64,16384,4096 64,32768,4096"; do
  t=${spec%%:*}; sh=${spec#*:}
  echo "== GLDS=$g tile $t"
  A2M_GEMM_GLDS=$g A2M_GEMM_TILE=$t A2M_GEMM_SPLIT=1 A2M_GEMM_KS2=0 timeout -k 10 200 python tools/gemm_bench.py $sh 2>&1 | grep gemm || exit 2
done
done | tee gpurun_out/r3_kloop.txt
