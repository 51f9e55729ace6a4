set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for i in 1 2 3; do timeout -k 10 300 python -u -m pytest tests/test_gpu_rccl.py -m gpu -x -q --timeout 250 -k graph > gpurun_out/rccl_g$i.log 2>&1 || { tail -5 gpurun_out/rccl_g$i.log; exit 3; }; tail -1 gpurun_out/rccl_g$i.log; done
bash tools/r06_bn_chan.sh bn5
