# interleaved training-iteration A/B of an env switch: bash tools/r3_train_env.sh VAR "v1 v2" [pairs]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
VAR=$1; VALS=$2; PAIRS=${3:-2}
for r in $(seq $PAIRS); do
for v in $VALS; do
env $VAR=$v timeout -k 10 300 python bench.py --mode train --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/te_$v.json 2>gpurun_out/te_$v.err || { tail -5 gpurun_out/te_$v.err; exit 3; }
python -c "import json;d=json.load(open('gpurun_out/te_$v.json'));print('$VAR=$v train ms',d['ms_per_step'])"
done
done
