#!/bin/bash
# GEMM engine configuration sweep: parity under the experimental settings first (must pass),
# then op timings and the end-to-end bench per setting.
#   tools/gemm_sweep.sh TAG "ENV1" "ENV2" ...     (each ENV is e.g. "A2M_GEMM_BK=32 A2M_GEMM_XCD=2")
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=$1; shift
for cfg in "$@"; do
  echo "== parity under [$cfg]"
  env $cfg timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/sweep_${TAG}_pytest.log 2>&1
  rc=$?; tail -1 gpurun_out/sweep_${TAG}_pytest.log
  if [ $rc -ne 0 ]; then tail -30 gpurun_out/sweep_${TAG}_pytest.log; exit $rc; fi
done
for cfg in "" "$@"; do
  env $cfg timeout -k 10 300 python tools/op_bench.py ${OPFILTER:-} >> gpurun_out/sweep_${TAG}_ops.log 2>&1 || { echo "op_bench failed [$cfg]"; tail -5 gpurun_out/sweep_${TAG}_ops.log; exit 3; }
  env $cfg timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/sweep_${TAG}_bench.log 2>&1 || { echo "bench failed [$cfg]"; tail -5 gpurun_out/sweep_${TAG}_bench.log; exit 4; }
  echo "[$cfg] $(python -c "import json,sys; d=json.loads(open('gpurun_out/sweep_${TAG}_bench.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['achieved'])")"
done
grep -v amdgpu.ids gpurun_out/sweep_${TAG}_ops.log
exit 0
