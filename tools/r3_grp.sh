set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_grouped.py tests/test_gpu_eval.py tests/test_gpu_tapconv.py tests/test_gpu_train.py > gpurun_out/grp_tests.log 2>&1 || { tail -30 gpurun_out/grp_tests.log; exit 2; }
tail -3 gpurun_out/grp_tests.log
for r in 1 2; do
for v in 0 1; do
A2M_GROUPED_DEC=$v timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/grp_b$v.json 2>gpurun_out/grp_b$v.err || { tail -5 gpurun_out/grp_b$v.err; exit 3; }
python -c "import json;d=json.load(open('gpurun_out/grp_b$v.json'));print('grouped=$v ms',d['ms_per_step'],'value',d['value'])"
done
done
timeout -k 10 300 python bench.py --mode train --steps 10 --warmup 3 > gpurun_out/train_bench.json 2>gpurun_out/train_bench.err || { tail -5 gpurun_out/train_bench.err; exit 4; }
python -c "import json;d=json.load(open('gpurun_out/train_bench.json'));print('train ms',d['ms_per_step'],'value',d['value'])"
bash tools/r3_enc.sh
