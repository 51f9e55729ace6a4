set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread tests/test_gpu_configs.py > gpurun_out/r3_cfg.log 2>&1
rc=$?
tail -40 gpurun_out/r3_cfg.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/enc_layers.py > gpurun_out/r3_enc_layers.txt 2>&1; cat gpurun_out/r3_enc_layers.txt
