#!/bin/bash
# round-4 probes: in-step spans, branch overlap, projection plans, A2M_PROJ_DENSE / A2M_TWO_SIDES
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --steps 100 --no-cpu-baseline > gpurun_out/r04f_bench.json 2> gpurun_out/r04f_bench.err || exit 1
timeout -k 10 120 python tools/branch_probe.py 100 > gpurun_out/r04_branch_probe.txt 2>&1 || exit 2
A2M_TWO_SIDES=1 timeout -k 10 120 python tools/branch_probe.py 100 >> gpurun_out/r04_branch_probe.txt 2>&1 || exit 3
timeout -k 10 120 python tools/proj_probe.py > gpurun_out/r04_proj_probe.txt 2>&1 || exit 4
A2M_PROJ_DENSE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "generator or headline or graph_stack" > gpurun_out/r04_projdense_parity.log 2>&1 || { tail -5 gpurun_out/r04_projdense_parity.log; exit 5; }
A2M_TWO_SIDES=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "headline" > gpurun_out/r04_twosides_parity.log 2>&1 || { tail -5 gpurun_out/r04_twosides_parity.log; exit 5; }
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $PWD/gpurun_out/r04_bp_trace -o run -- python tools/branch_probe.py 30 >> gpurun_out/r04_branch_probe.txt 2>&1 || exit 7
A2M_TWO_SIDES=1 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $PWD/gpurun_out/r04_bp2_trace -o run -- python tools/branch_probe.py 30 >> gpurun_out/r04_branch_probe.txt 2>&1 || exit 8
bash tools/ab_env.sh "A2M_PROJ_DENSE=1" 3 > gpurun_out/r04_ab_projdense.txt 2>&1 || exit 6
bash tools/ab_env.sh "A2M_TWO_SIDES=1" 3 > gpurun_out/r04_ab_twosides.txt 2>&1 || exit 9
exit 0
