set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_eval.py -k "graph or eval or generator" > gpurun_out/fold_tests.log 2>&1 || { tail -30 gpurun_out/fold_tests.log; exit 2; }
tail -1 gpurun_out/fold_tests.log
for v in 0 1 0 1; do echo "fold=$v"; A2M_STACK_FOLD=$v timeout -k 10 120 python tools/stack_bench.py both 50; done
bash tools/r3_ab_long.sh A2M_STACK_FOLD "0 1" 3
