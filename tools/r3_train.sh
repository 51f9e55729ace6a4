set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --mode train --steps 10 --warmup 3 > gpurun_out/train_bench.json 2>gpurun_out/train_bench.err || { tail -5 gpurun_out/train_bench.err; exit 2; }
python -c "import json;d=json.load(open('gpurun_out/train_bench.json'));print('train ms',d['ms_per_step'],'value',d['value'],'frac',d['path_roofline']['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $PWD/gpurun_out/trainprof -o run -- python bench.py --mode train --steps 5 --warmup 1 > gpurun_out/trainprof.log 2>&1 || { tail -5 gpurun_out/trainprof.log; exit 3; }
python tools/prof_summary.py gpurun_out/trainprof/run_kernel_trace.csv 6 > gpurun_out/r3_train_breakdown.txt
head -40 gpurun_out/r3_train_breakdown.txt
