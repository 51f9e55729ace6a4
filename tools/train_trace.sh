# kernel trace of the training iteration (fp32 B=64 and bf16 B=32): per-kernel time per step
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $PWD/gpurun_out/tt32 -o run -- python bench.py --mode train --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/tt32.log 2>&1 || { echo fail; tail -3 gpurun_out/tt32.log; exit 4; }
python tools/prof_summary.py $(find gpurun_out/tt32 -name "*kernel_trace.csv" | head -1) 4 > gpurun_out/train_breakdown_fp32_b64.txt
find gpurun_out/tt32 -name "*.csv" -size +5M -delete
tail -1 gpurun_out/tt32.log
head -16 gpurun_out/train_breakdown_fp32_b64.txt
bash tools/train_trace_bf16.sh
