# round-3 checkpoint on one box: full GPU suite, smoke, default bench line, step PMC passes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r03_v1}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 2; }
tail -1 gpurun_out/${TAG}_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -10 gpurun_out/${TAG}_smoke.log; exit 3; }
tail -2 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -10 gpurun_out/${TAG}_bench.err; exit 4; }
cat gpurun_out/${TAG}_bench.json
bash tools/step_pmc.sh $TAG || exit 5
python tools/prof_summary.py gpurun_out/steppmc_$TAG/trace/run_kernel_trace.csv 5 > gpurun_out/${TAG}_step_breakdown.txt
head -12 gpurun_out/${TAG}_step_breakdown.txt
