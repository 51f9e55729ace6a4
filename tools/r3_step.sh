# GPU check of an engine change: the GPU test suite, the bench line, the encoder plan probe.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-x}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/${TAG}_pytest.log | head -20; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -5 gpurun_out/${TAG}_bench.err; exit 3; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print('step',d['ms_per_step'],'gemm',d['roofline']['achieved'],'mel+enc',d['mel_encoder_roofline'])"
timeout -k 10 400 python -u tools/tile_probe.py > gpurun_out/${TAG}_probe.txt 2>&1 || { tail -5 gpurun_out/${TAG}_probe.txt; exit 4; }
grep -E "best|default" gpurun_out/${TAG}_probe.txt
