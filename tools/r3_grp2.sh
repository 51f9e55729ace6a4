set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_grouped.py > gpurun_out/grp_tests.log 2>&1 || { tail -30 gpurun_out/grp_tests.log; exit 2; }
tail -1 gpurun_out/grp_tests.log
for r in 1 2; do
for v in 0 1 2; do
A2M_GROUPED_DEC=$v timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/grp_b$v.json 2>gpurun_out/grp_b$v.err || { tail -5 gpurun_out/grp_b$v.err; exit 3; }
python -c "import json;d=json.load(open('gpurun_out/grp_b$v.json'));print('grouped=$v ms',d['ms_per_step'])"
done
done
A2M_GROUPED_DEC=1 LANES_TAG=_grp1 bash tools/r3_lanes.sh > /dev/null && tail -40 gpurun_out/r3_lanes_grp1.txt
