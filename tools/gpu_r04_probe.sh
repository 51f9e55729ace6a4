set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/b1.json 2> gpurun_out/b1.err && \
STEP_PMC_REPS=10 timeout -k 10 600 bash tools/step_pmc.sh r04_v1 > gpurun_out/spmc.log 2>&1
echo rc=$?
