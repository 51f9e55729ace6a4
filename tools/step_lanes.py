"""One graph-replayed bench step from a rocprofv3 kernel trace, kernel by kernel: hardware
queue, start / end offset, duration, grid, name -- the two decoder branches show up as the
two queues after the UNet.  usage: python tools/step_lanes.py run_kernel_trace.csv [step]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
idx = int(sys.argv[2]) if len(sys.argv) > 2 else 3
starts = [i for i, r in enumerate(rows) if 'logmel' in r['Kernel_Name']]
steps = [i for i in starts if i + 1 < len(rows) and 'logmel' not in rows[i + 1]['Kernel_Name']]
a, b = steps[idx], steps[idx + 1]
t0 = int(rows[a]['Start_Timestamp'])
qmap = {}
end = {}
for r in rows[a:b]:
    q = qmap.setdefault(r.get('Queue_Id', '?'), f'q{len(qmap)}')
    s, e = (int(r['Start_Timestamp']) - t0) / 1e3, (int(r['End_Timestamp']) - t0) / 1e3
    end[q] = max(end.get(q, 0), e)
    grid = f"{r.get('Grid_Size_X', r.get('Grid_Size', '?'))}"
    print(f'{q:3s} {s:8.1f} {e:8.1f} {e - s:7.1f}  {r["Kernel_Name"].split("(")[0][-56:]:56s} grid={grid}')
print('queue end times:', {q: round(v, 1) for q, v in end.items()})
durs = [(int(rows[steps[i + 1]]['Start_Timestamp']) - int(rows[steps[i]]['Start_Timestamp'])) / 1e3
        for i in range(len(steps) - 1)]
print('step start-to-start (us):', [round(d, 1) for d in durs])
