set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_syncbn.py tests/test_gpu_configs.py tests/test_gpu_bf16.py > gpurun_out/gbwd_tests.log 2>&1 || { tail -30 gpurun_out/gbwd_tests.log; exit 2; }
tail -1 gpurun_out/gbwd_tests.log
PREV=$PWD/audio-to-motion-generation_amd/a2m/liba2m_prev.so
for r in 1 2; do
for v in new prev; do
if [ $v = prev ]; then export A2M_LIB=$PREV; else unset A2M_LIB; fi
timeout -k 10 300 python bench.py --mode train --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/tr_$v.json 2>gpurun_out/tr_$v.err || { tail -5 gpurun_out/tr_$v.err; exit 3; }
python -c "import json;d=json.load(open('gpurun_out/tr_$v.json'));print('$v train ms',d['ms_per_step'])"
done
done
unset A2M_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/trainprof4 -o run -- python bench.py --mode train --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/trainprof4.log 2>&1 || { tail -5 gpurun_out/trainprof4.log; exit 4; }
python tools/prof_summary.py gpurun_out/trainprof4/run_kernel_trace.csv 6 > gpurun_out/r03_train_breakdown_v5.txt
head -8 gpurun_out/r03_train_breakdown_v5.txt
