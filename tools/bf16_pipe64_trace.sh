# bf16 training with the training-mode launches kept on the 64x64 pipelined tile (A2M_GEMM_PIPE64=2)
# against the default: kernel time per step from traces (the wall time varies run to run with fixed work)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for mode in 1 2; do
  A2M_GEMM_PIPE64=$mode timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $PWD/gpurun_out/tp_$mode -o run -- python bench.py --mode train --steps 3 --warmup 1 --batch 32 --dtype bf16 --no-cpu-baseline > gpurun_out/tp_$mode.log 2>&1 || { echo fail; tail -3 gpurun_out/tp_$mode.log; exit 4; }
  python tools/prof_summary.py $(find gpurun_out/tp_$mode -name "*kernel_trace.csv" | head -1) 4 > gpurun_out/tp_$mode.txt
  find gpurun_out/tp_$mode -name "*.csv" -size +5M -delete
  echo "== A2M_GEMM_PIPE64=$mode"; head -1 gpurun_out/tp_$mode.txt; grep -E "4, 4|4, 1|7, 0, 4|3, 0, 3|3, 3" gpurun_out/tp_$mode.txt || true
done
