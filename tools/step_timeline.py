"""Critical-path view of one graph-replayed bench step from a rocprofv3 kernel trace: window
length, union of busy time (kernels on any stream), summed kernel time, idle gaps.
usage: python tools/step_timeline.py run_kernel_trace.csv [step_index]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
idx = int(sys.argv[2]) if len(sys.argv) > 2 else 6
starts = [i for i, r in enumerate(rows) if 'logmel' in r['Kernel_Name']]
# forward steps: a logmel launch followed by a non-logmel one (the mel-only timing loop is last)
steps = [i for i in starts if i + 1 < len(rows) and 'logmel' not in rows[i + 1]['Kernel_Name']]
a, b = steps[idx], steps[idx + 1]
win = rows[a:b]
t0 = int(win[0]['Start_Timestamp'])
t1 = int(rows[b]['Start_Timestamp'])
iv = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'].split('(')[0][-60:]) for r in win)
busy, cur_s, cur_e, gaps = 0, iv[0][0], iv[0][1], []
prev_name = iv[0][2]
for s, e, n in iv[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        gaps.append((s - cur_e, prev_name, n))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
    prev_name = n
busy += cur_e - cur_s
ksum = sum(e - s for s, e, _ in iv)
print(f'step window {(t1 - t0) / 1e3:.1f} us, kernels {len(win)}, busy union {busy / 1e3:.1f} us, '
      f'kernel sum {ksum / 1e3:.1f} us, idle {(t1 - t0 - busy) / 1e3:.1f} us in {len(gaps)} gaps')
for g, p, n in sorted(gaps, reverse=True)[:12]:
    print(f'  gap {g / 1e3:6.2f} us  after {p}  before {n}')
agg = {}
for s, e, n in iv:
    c, t = agg.get(n, (0, 0))
    agg[n] = (c + 1, t + e - s)
print('per-kernel time in this step:')
for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f'  {t / 1e3:8.1f} us {c:4d} x  {n}')
per_q = {}
for r in win:
    q = r.get('Queue_Id', '?')
    per_q[q] = per_q.get(q, 0) + int(r['End_Timestamp']) - int(r['Start_Timestamp'])
print('kernel time per hardware queue:', {k: round(v / 1e3, 1) for k, v in per_q.items()})
