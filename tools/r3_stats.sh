set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r03}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "interp or conv2d or eval" > gpurun_out/st_tests.log 2>&1 || { tail -20 gpurun_out/st_tests.log; exit 2; }
tail -1 gpurun_out/st_tests.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/stats_$TAG -o run -- python tools/step_pmc.py 20 > gpurun_out/stats_$TAG.log 2>&1 || { tail -5 gpurun_out/stats_$TAG.log; exit 3; }
python tools/prof_summary.py gpurun_out/stats_$TAG/run_kernel_trace.csv 22 > gpurun_out/${TAG}_step_breakdown.txt
python tools/step_lanes.py gpurun_out/stats_$TAG/run_kernel_trace.csv 15 > gpurun_out/${TAG}_step_lanes.txt
head -30 gpurun_out/${TAG}_step_breakdown.txt
tail -2 gpurun_out/${TAG}_step_lanes.txt
