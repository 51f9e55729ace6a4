#!/bin/bash
# Tuning session: parity tests (must pass) then op timings under several GEMM settings.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-perf}
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log
if [ $rc -ge 2 ]; then exit $rc; fi
for cfg in "" "A2M_GEMM_TILE=64" "A2M_GEMM_TILE=128" ; do
  env $cfg timeout -k 10 300 python tools/op_bench.py >> gpurun_out/opbench_$TAG.log 2>&1 || { echo "op_bench failed ($cfg)"; tail -5 gpurun_out/opbench_$TAG.log; exit 3; }
done
cat gpurun_out/opbench_$TAG.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1 || { tail -5 gpurun_out/bench_$TAG.log; exit 4; }
tail -1 gpurun_out/bench_$TAG.log
exit $rc
