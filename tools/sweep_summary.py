"""Best plan per (shape, precision) from tools/gemm_bench.py SWEEP output.  usage: sweep_summary.py LOG"""
import re
import sys
best = {}
plan = {}
for line in open(sys.argv[1]):
    m = re.match(r'gemm (\d+x\d+x\d+) (\S+)\s+(planner|tile (\d+) split (\d+))\s*:\s+([\d.]+) us', line)
    if not m:
        continue
    shape, prec, us = m.group(1), m.group(2), float(m.group(6))
    tag = 'planner' if m.group(3) == 'planner' else f't{m.group(4)}s{m.group(5)}'
    if tag == 'planner':
        plan[(shape, prec)] = us
    elif us < best.get((shape, prec), (1e9, ''))[0]:
        best[(shape, prec)] = (us, tag)
shapes = sorted({k[0] for k in best}, key=lambda s: [int(v) for v in s.split('x')])
precs = sorted({k[1] for k in best})
tot = {p: [0.0, 0.0] for p in precs}
for s in shapes:
    row = f'{s:18s}'
    for p in precs:
        b = best.get((s, p), (0, ''))
        pl = plan.get((s, p), 0)
        tot[p][0] += pl
        tot[p][1] += b[0]
        row += f' | {p:6s} planner {pl:7.1f} best {b[0]:7.1f} {b[1]:7s}'
    print(row)
for p in precs:
    print(f'total {p}: planner {tot[p][0]:.1f} us, best {tot[p][1]:.1f} us')
