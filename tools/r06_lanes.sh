set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $PWD/gpurun_out/lanes_tr -o run -- python tools/step_pmc.py 10 --sync > gpurun_out/lanes_tr.log 2>&1 || { tail -5 gpurun_out/lanes_tr.log; exit 2; }
python tools/step_lanes.py gpurun_out/lanes_tr 3 > gpurun_out/lanes_step3.txt && python tools/step_lanes.py gpurun_out/lanes_tr 6 > gpurun_out/lanes_step6.txt
find gpurun_out/lanes_tr -name "*kernel_trace.csv" -delete
