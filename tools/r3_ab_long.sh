# interleaved long A/B of an env switch: bash tools/r3_ab_long.sh VAR "v1 v2 ..." [pairs]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
VAR=$1; VALS=$2; PAIRS=${3:-3}
for r in $(seq $PAIRS); do
for v in $VALS; do
env $VAR=$v timeout -k 10 240 python bench.py --steps 200 --warmup 30 --no-cpu-baseline > gpurun_out/ab_$v.json 2>gpurun_out/ab_$v.err || { tail -5 gpurun_out/ab_$v.err; exit 3; }
python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('$VAR=$v ms',d['ms_per_step'])"
done
done
