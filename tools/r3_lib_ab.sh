# interleaved bench A/B of the in-tree library against a2m/liba2m_prev.so: bash tools/r3_lib_ab.sh [pairs] [extra bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
PAIRS=${1:-3}; shift
PREV=$PWD/audio-to-motion-generation_amd/a2m/liba2m_prev.so
for r in $(seq $PAIRS); do
for v in new prev; do
if [ $v = prev ]; then export A2M_LIB=$PREV; else unset A2M_LIB; fi
timeout -k 10 240 python bench.py --steps 200 --warmup 30 --no-cpu-baseline "$@" > gpurun_out/lab_$v.json 2>gpurun_out/lab_$v.err || { tail -5 gpurun_out/lab_$v.err; exit 3; }
python -c "import json;d=json.load(open('gpurun_out/lab_$v.json'));print('$v ms',d['ms_per_step'],'path_frac',d.get('mel_encoder_roofline',{}).get('path_frac'))"
done
done
