#!/bin/bash
# queued-basis in-step roofline: timing tests, bench line, stamps (with ready marks) vs the trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r04j_bench.json 2> gpurun_out/r04j_bench.err || { tail -20 gpurun_out/r04j_bench.err; exit 2; }
python -c "import json; d=json.loads(open('gpurun_out/r04j_bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], json.dumps(d['roofline']))"
bash tools/gpu_r04i.sh || exit 3
head -4 gpurun_out/r04i_svt/stamp_vs_trace.txt
timeout -k 10 200 bash tools/step_pmc.sh r04j > /dev/null 2>&1; head -3 gpurun_out/steppmc_r04j/breakdown.txt
