set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/enc_r3 -o run -- python tools/enc_trace.py > gpurun_out/enc_r3.log 2>&1 || { tail -5 gpurun_out/enc_r3.log; exit 2; }
grep "encoder graph" gpurun_out/enc_r3.log
python tools/prof_summary.py gpurun_out/enc_r3/run_kernel_trace.csv 31 > gpurun_out/r3_encoder_mode6.txt
head -20 gpurun_out/r3_encoder_mode6.txt
bash tools/r3_c1pmc.sh > gpurun_out/r3_conv0_pmc.txt 2>&1 || { tail -5 gpurun_out/r3_conv0_pmc.txt; exit 3; }
cat gpurun_out/r3_conv0_pmc.txt
