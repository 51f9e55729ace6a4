set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in 0 1 2 0 1 2; do
A2M_GROUPED_DEC=$v timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $PWD/gpurun_out/lanes$v -o run -- python tools/step_pmc.py 12 > gpurun_out/lanes$v.log 2>&1 || { tail -5 gpurun_out/lanes$v.log; exit 2; }
python tools/step_lanes.py gpurun_out/lanes$v/run_kernel_trace.csv 6 > gpurun_out/r3_lanes_m$v.txt
echo "mode $v"; tail -1 gpurun_out/r3_lanes_m$v.txt
done
