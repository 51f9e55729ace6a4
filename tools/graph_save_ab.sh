# graph-layer backward probe (tools/graph_bwd_probe.sh), the GPU training tests, then the
# training iteration with / without the saved pre-LayerNorm output, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/graph_bwd_probe.sh > gpurun_out/gbwd_probe_all.txt 2>&1 || { tail -30 gpurun_out/gbwd_probe_all.txt; exit 3; }
head -12 gpurun_out/gbwd_bench.txt; grep -v "^  h[123]" gpurun_out/gbwd_phases_saved.txt | head -14
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_train.py > gpurun_out/train_tests.txt 2>&1 || { tail -20 gpurun_out/train_tests.txt; exit 3; }
tail -2 gpurun_out/train_tests.txt
TRAIN_STEPS=20 TRAIN_WARMUP=3 bash tools/ab_train_env.sh 2 "" A2M_GRAPH_SAVE_PRE=0 A2M_GRAPH_SAVE_PRE=1
