# bf16 B=32 training kernel traces with the training-mode pipelined tiles off / on: per-family
# kernel time per step and launch counts (the iteration's wall time varies run to run with fixed
# work -- the gaps between its short kernels -- the kernel sums do not)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for mode in off on; do
  if [ $mode = off ]; then E="A2M_GEMM_PIPE4=0 A2M_GEMM_PIPE_A3=0"; else E=""; fi
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $PWD/gpurun_out/tb_$mode -o run -- python bench.py --mode train --steps 3 --warmup 1 --batch 32 --dtype bf16 --no-cpu-baseline > gpurun_out/tb_$mode.log 2>&1 || { echo fail; tail -3 gpurun_out/tb_$mode.log; exit 4; }
  python tools/prof_summary.py $(find gpurun_out/tb_$mode -name "*kernel_trace.csv" | head -1) 4 > gpurun_out/tb_$mode.txt
  find gpurun_out/tb_$mode -name "*.csv" -size +5M -delete
  echo "== $mode"; head -12 gpurun_out/tb_$mode.txt
done
