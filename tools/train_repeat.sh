# repeated training-iteration lines on one box (the bf16 B=32 wall time varies run to run with fixed work)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --mode train --steps 30 --warmup 5 --batch 32 --dtype bf16 --no-cpu-baseline > gpurun_out/trr.log 2>&1 || { tail -3 gpurun_out/trr.log; exit 3; }
  python -c "import json; d=json.loads(open('gpurun_out/trr.log').read().strip().splitlines()[-1]); print('bf16 b32', d['ms_per_step'], d['value'])"
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --mode train --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/trr.log 2>&1 || { tail -3 gpurun_out/trr.log; exit 3; }
  python -c "import json; d=json.loads(open('gpurun_out/trr.log').read().strip().splitlines()[-1]); print('fp32 b64', d['ms_per_step'], d['value'])"
done
