set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=$PWD/audio-to-motion-generation_amd/a2m
A2M_LIB=$L/liba2m_ig.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tapconv.py tests/test_gpu_parity.py > gpurun_out/ig_tests.log 2>&1 || { tail -20 gpurun_out/ig_tests.log; exit 2; }
tail -1 gpurun_out/ig_tests.log
for v in ig prev; do echo "== $v"; A2M_LIB=$L/liba2m_$v.so timeout -k 10 200 python tools/conv_scaling.py | head -5; done
for r in 1 2 3; do for v in ig prev; do
A2M_LIB=$L/liba2m_$v.so timeout -k 10 240 python bench.py --steps 200 --warmup 30 --no-cpu-baseline > gpurun_out/ig_$v.json 2>/dev/null || exit 3
python -c "import json;d=json.load(open('gpurun_out/ig_$v.json'));print('$v ms',d['ms_per_step'],d['mel_encoder_roofline']['path_frac'])"
done; done
