"""Per-step kernel-time breakdown from a rocprofv3 kernel-trace CSV.
usage: python tools/prof_summary.py gpurun_out/prof_r1/run_kernel_trace.csv [steps]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    name = r['Kernel_Name']
    key = name.split('(')[0][:90]
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    agg[key][0] += 1
    agg[key][1] += d
tot = sum(v[1] for v in agg.values())
print(f'total kernel time {tot / 1e3:.2f} ms over all dispatches; per step (/{steps}) {tot / steps / 1e3:.3f} ms')
for k, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
    print(f'{us / steps:10.1f} us/step {n / steps:7.1f} calls/step {100 * us / tot:5.1f}%  {k}')
