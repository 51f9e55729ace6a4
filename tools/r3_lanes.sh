set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $PWD/gpurun_out/lanes -o run -- python tools/step_pmc.py 5 > gpurun_out/lanes.log 2>&1 || { tail -5 gpurun_out/lanes.log; exit 2; }
python tools/step_lanes.py gpurun_out/lanes/run_kernel_trace.csv 4 > gpurun_out/r3_lanes${LANES_TAG}.txt
cat gpurun_out/r3_lanes${LANES_TAG}.txt
