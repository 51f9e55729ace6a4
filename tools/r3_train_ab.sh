set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for r in 1 2; do
for t in . _r02; do
(cd $t && timeout -k 10 300 python bench.py --mode train --steps 10 --warmup 3 --no-cpu-baseline > /tmp/tb.json 2>/tmp/tb.err) || { tail -5 /tmp/tb.err; exit 3; }
python -c "import json;d=json.load(open('/tmp/tb.json'));print('$t train ms',d['ms_per_step'])"
done
done
