set -o pipefail
cd $GRAFT_REPO_ROOT
A2M_GEMM_LOG=2 timeout -k 10 300 python tools/train_gemm_times.py > gpurun_out/tg.out 2> gpurun_out/tg.log || { tail -5 gpurun_out/tg.log; exit 2; }
cat gpurun_out/tg.out
python tools/train_gemm_times.py --summarise gpurun_out/tg.log | tee gpurun_out/r03_train_gemms.txt | head -45
