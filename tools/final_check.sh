#!/bin/bash
# Round-end evidence in one GPU call: parity tests + bench + rocprof kernel stats + HBM PMC
# passes (tools/gpu_check.sh), smoke(), the step-only PMC / MFMA-busy passes
# (tools/step_pmc.sh) and the step timeline.   tools/final_check.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1
bash tools/gpu_check.sh $TAG || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.txt 2>&1 || { tail -5 gpurun_out/smoke_$TAG.txt; exit 7; }
tail -1 gpurun_out/smoke_$TAG.txt
bash tools/step_pmc.sh $TAG || exit $?
python tools/step_ops.py gpurun_out/steppmc_$TAG/trace/run_kernel_trace.csv > gpurun_out/timeline_$TAG.txt 2>/dev/null || \
  python tools/step_ops.py $(find gpurun_out/steppmc_$TAG/trace -name '*kernel_trace.csv' | head -1) > gpurun_out/timeline_$TAG.txt
tail -1 gpurun_out/timeline_$TAG.txt
exit 0
