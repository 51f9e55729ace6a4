# every engine launch of the training iteration with its plan (A2M_GEMM_LOG=1), one warmup + one step
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
A2M_GEMM_LOG=1 timeout -k 10 300 python bench.py --mode train --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/train_plans.out 2> gpurun_out/train_plans.txt
rc=$?; grep -c "a2m gemm" gpurun_out/train_plans.txt; exit $rc
