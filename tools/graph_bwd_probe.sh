# graph-layer backward at the training shapes: both paths timed (tools/graph_bwd_bench.py), then
# the per-phase stamps of the recompute and saved paths (diagnostic build _ab/gbst.so)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 120 python tools/graph_bwd_bench.py > gpurun_out/gbwd_bench.txt 2>&1 && \
A2M_LIB=_ab/gbst.so timeout -k 10 120 python tools/graph_bwd_phases.py > gpurun_out/gbwd_phases.txt 2>&1 && \
SAVED=1 A2M_LIB=_ab/gbst.so timeout -k 10 120 python tools/graph_bwd_phases.py > gpurun_out/gbwd_phases_saved.txt 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_train.py -k "graph_layer" > gpurun_out/gbwd_tests.txt 2>&1
rc=$?; cat gpurun_out/gbwd_bench.txt; grep -v "^  h[123]" gpurun_out/gbwd_phases_saved.txt; tail -3 gpurun_out/gbwd_tests.txt; exit $rc
