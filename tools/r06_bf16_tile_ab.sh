#!/bin/bash
# bf16 mode: the plan log, then the UNet's 128x128-tile launches forced onto the 64x64 pipelined
# bf16 tile (A2M_GEMM_PLAN_RULES built from the log) vs the planner, bf16 bench lines interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A2M_GEMM_LOG=1 timeout -k 10 120 python tools/plan_log.py bf16 > /dev/null 2> gpurun_out/bt_plans.txt || { tail -5 gpurun_out/bt_plans.txt; exit 1; }
RULES=$(python - <<'PY'
import re
rules = []
for l in open('gpurun_out/bt_plans.txt'):
    if l.startswith('--- second'):
        break
    m = re.match(r'a2m gemm M=(\d+) N=(\d+) K=(\d+) batch=\d+ tile=(\d+) bk=\d+ splits=(\d+)', l)
    if m and m.group(4) == '128':
        M, N, K = m.group(1), m.group(2), m.group(3)
        S = int(m.group(5))
        rules.append(f'{M},{N},{K}:64:{max(1, min(S * 2, 8))}')
print(';'.join(dict.fromkeys(rules)))
PY
)
echo "rules: $RULES"
grep -c "tile=128" gpurun_out/bt_plans.txt
for i in 1 2 3; do
  for r in "" "$RULES"; do
    A2M_GEMM_PLAN_RULES="$r" timeout -k 10 300 python bench.py --no-cpu-baseline --no-trace --steps 300 --dtype bf16 > gpurun_out/bt_b64.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bt_b64.log; exit 3; }
    A2M_GEMM_PLAN_RULES="$r" timeout -k 10 300 python bench.py --no-cpu-baseline --no-trace --steps 300 --dtype bf16 --batch 32 > gpurun_out/bt_b32.log 2>&1 || { echo "bench b32 failed"; exit 3; }
    echo "rules=$([ -z "$r" ] && echo planner || echo pipe64) bf16 B=64 $(python -c "import json; print(json.loads(open('gpurun_out/bt_b64.log').read().strip().splitlines()[-1])['ms_per_step'])") B=32 $(python -c "import json; print(json.loads(open('gpurun_out/bt_b32.log').read().strip().splitlines()[-1])['ms_per_step'])")"
  done
done
exit 0
