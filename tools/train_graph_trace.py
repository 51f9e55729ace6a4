"""Per-iteration kernel time vs the iteration's span in a rocprofv3 kernel trace of
`bench.py --mode train` (round 6: graph-replayed training).  Iterations are delimited by the
Adam launches (3 G-steps + 1 D-step = 4 per iteration); the last N iterations are the timed ones.
usage: python tools/train_graph_trace.py run_kernel_trace.csv N [steps_per_iter=4]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
n_it = int(sys.argv[2])
per = int(sys.argv[3]) if len(sys.argv) > 3 else 4
adam = [i for i, r in enumerate(rows) if 'adam' in r['Kernel_Name'] and 'tick' not in r['Kernel_Name']]
ends = adam[-per * n_it - 1::per]          # the Adam that closes each iteration (and the one before)
assert len(ends) == n_it + 1, (len(adam), len(ends))
busy, span, launches = [], [], []
agg = collections.defaultdict(lambda: [0, 0.0])
for a, b in zip(ends[:-1], ends[1:]):
    seg = rows[a + 1:b + 1]
    t0 = int(rows[a]['End_Timestamp'])
    t1 = int(rows[b]['End_Timestamp'])
    busy.append(sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in seg) / 1e6)
    span.append((t1 - t0) / 1e6)
    launches.append(len(seg))
    for r in seg:
        k = r['Kernel_Name'].split('(')[0][:90]
        agg[k][0] += 1
        agg[k][1] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
print(f'{n_it} iterations: kernel time {sum(busy) / n_it:.3f} ms, span {sum(span) / n_it:.3f} ms an iteration '
      f'(kernels / span {sum(busy) / sum(span):.3f}), {sum(launches) / n_it:.0f} launches an iteration')
print('per iteration kernel ms:', ' '.join(f'{b:.2f}' for b in busy))
print('per iteration span ms:  ', ' '.join(f'{s:.2f}' for s in span))
tot = sum(v[1] for v in agg.values())
fam = {'batchnorm (bn_*, reduce_slices)': ('bn_', 'reduce_slices'), 'split-K reduce': ('splitk_reduce',),
       'engine tiles (gemm_kernel, gemm_pipe*)': ('gemm_kernel', 'gemm_pipe')}
for name, keys in fam.items():
    us = sum(v[1] for k, v in agg.items() if any(q in k for q in keys))
    n = sum(v[0] for k, v in agg.items() if any(q in k for q in keys))
    print(f'family {name}: {us / n_it / 1e3:.3f} ms / iter, {n / n_it:.0f} launches / iter')
for k, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f'{us / n_it:10.1f} us/iter {n / n_it:7.1f} calls/iter {100 * us / tot:5.1f}%  {k}')
