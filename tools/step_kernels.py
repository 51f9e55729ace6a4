"""Kernel time by kind over replayed bench steps of a rocprofv3 kernel trace (steps start at the
log-mel launch).  usage: python tools/step_kernels.py run_kernel_trace.csv [first_step last_step]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
starts = [i for i, r in enumerate(rows) if 'logmel' in r['Kernel_Name']]
s0 = int(sys.argv[2]) if len(sys.argv) > 2 else 3
s1 = int(sys.argv[3]) if len(sys.argv) > 3 else min(len(starts) - 2, 7)
agg = collections.defaultdict(lambda: [0, 0.0])
wins = []
for s in range(s0, s1 + 1):
    a, b = starts[s], starts[s + 1]
    t0 = int(rows[a]['Start_Timestamp'])
    wins.append((max(int(r['End_Timestamp']) for r in rows[a:b]) - t0) / 1e3)
    for r in rows[a:b]:
        k = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('a2m::', '')[-48:]
        agg[k][0] += 1
        agg[k][1] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
n = s1 - s0 + 1
tot = sum(v[1] for v in agg.values()) / n
print(f'{n} steps, window {sum(wins) / n:.1f} us, kernel sum {tot:.1f} us/step')
for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f'{t / n:9.1f} us {c / n:5.1f} x {t / c:7.1f} us  {100 * t / n / tot:5.1f}%  {k}')
