set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $PWD/gpurun_out/tt16 -o run -- python bench.py --mode train --steps 3 --warmup 1 --batch 32 --dtype bf16 --no-cpu-baseline > gpurun_out/tt16.log 2>&1 || { echo fail; tail -3 gpurun_out/tt16.log; exit 4; }
python tools/prof_summary.py $(find gpurun_out/tt16 -name "*kernel_trace.csv" | head -1) 4 > gpurun_out/train_breakdown_bf16_b32.txt
find gpurun_out/tt16 -name "*.csv" -size +5M -delete
head -28 gpurun_out/train_breakdown_bf16_b32.txt
