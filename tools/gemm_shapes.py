"""Per-launch GEMM engine efficiency: match the engine's launch log (A2M_GEMM_LOG=1, stderr)
with a rocprofv3 kernel trace of the same eager (--no-graph) run, in dispatch order.
usage: python tools/gemm_shapes.py bench_stderr.log prof_dir/..._kernel_trace.csv [last_n]"""
import collections
import csv
import re
import sys

log = [l for l in open(sys.argv[1]) if l.startswith('a2m gemm ')]
rows = sorted(csv.DictReader(open(sys.argv[2])), key=lambda r: int(r['Start_Timestamp']))
launches = []   # (tile kernel row, reduce row or None)
i = 0
while i < len(rows):
    n = rows[i]['Kernel_Name']
    if 'gemm_kernel' in n:
        red = rows[i + 1] if i + 1 < len(rows) and 'splitk_reduce' in rows[i + 1]['Kernel_Name'] else None
        launches.append((rows[i], red))
        i += 2 if red else 1
    else:
        i += 1
if len(launches) != len(log):
    print(f'warning: {len(launches)} gemm dispatches vs {len(log)} log lines; aligning at the end')
k = min(len(launches), len(log))
last = int(sys.argv[3]) if len(sys.argv) > 3 else k
pairs = list(zip(log[-k:], launches[-k:]))[-last:]
agg = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])
dur = lambda r: (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
for l, (kr, rr) in pairs:
    m = re.search(r'M=(\d+) N=(\d+) K=(\d+) batch=(\d+) tile=(\d+) bk=\d+ splits=(\d+) modes=(\d),(\d)', l)
    M, N, K, b, tile, s, ma, mb = map(int, m.groups())
    som = re.search(r'som=(\d+)', l)
    key = (M, N, K, b, tile, s, ma, mb, int(som.group(1)) if som else -1)
    a = agg[key]
    a[0] += 1
    a[1] += dur(kr)
    a[2] += dur(rr) if rr else 0.0
    a[3] += 2.0 * M * N * K * b
tot = sum(a[1] + a[2] for a in agg.values())
print(f'{len(pairs)} launches, {tot:.1f} us total')
print(f'{"M":>5} {"N":>6} {"K":>6} {"b":>3} {"tile":>4} {"spl":>3} {"md":>3} {"som":>5} {"n":>3} {"tile_us":>8} {"red_us":>7} {"TF":>6} {"%":>5}')
for key, (n, tk, tr, fl) in sorted(agg.items(), key=lambda kv: -(kv[1][1] + kv[1][2])):
    M, N, K, b, tile, s, ma, mb, som = key
    t = (tk + tr) / n
    print(f'{M:5d} {N:6d} {K:6d} {b:3d} {tile:4d} {s:3d} {ma}{mb:>2} {som:5d} {n:3d} {tk / n:8.1f} {tr / n:7.1f} '
          f'{fl / n / t / 1e6:6.1f} {100 * (tk + tr) / tot:5.1f}')
