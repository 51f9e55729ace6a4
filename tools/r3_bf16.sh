set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 250 --timeout-method thread tests/test_gpu_configs.py -k "bf16_train" > gpurun_out/r3_bf16.log 2>&1
rc=$?
grep -E "cosine|PASS|FAIL|Error" gpurun_out/r3_bf16.log | head
exit $rc
