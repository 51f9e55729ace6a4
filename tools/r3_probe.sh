set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 250 --timeout-method thread tests/test_gpu_configs.py -k "bf16_train" > gpurun_out/r3_bf16.log 2>&1
grep -E "cosine|PASS|FAIL|Error" gpurun_out/r3_bf16.log | head
timeout -k 10 300 python -u tools/tile_probe.py > gpurun_out/r3_tile_probe_m1.txt 2>&1 || { tail -20 gpurun_out/r3_tile_probe_m1.txt; exit 3; }
A2M_GEMM_KS2_MODES=3 timeout -k 10 300 python -u tools/tile_probe.py > gpurun_out/r3_tile_probe_m3.txt 2>&1 || { tail -20 gpurun_out/r3_tile_probe_m3.txt; exit 4; }
grep -E "best|default|dense" gpurun_out/r3_tile_probe_m*.txt
