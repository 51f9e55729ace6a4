"""One replayed bench step from a tools/step_pmc.py kernel trace, kernel by kernel per hardware
queue (the graph's two branch streams land on different queues): start / end relative to the
step's first dispatch, so the critical path of the two decoder branches can be read off.

    python tools/step_lanes.py TRACE_DIR [step_index]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from replay_filter import load, replayed  # noqa: E402


def main():
    rows = replayed(load(sys.argv[1], '*kernel_trace.csv'))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    starts = [i for i, r in enumerate(rows) if 'logmel' in r['Kernel_Name']]
    lo, hi = starts[k], starts[k + 1] if k + 1 < len(starts) else len(rows)
    t0 = int(rows[lo]['Start_Timestamp'])
    queues = sorted({r['Queue_Id'] for r in rows[lo:hi]})
    print(f'step {k}: {hi - lo} kernels, queues {queues}')
    for r in rows[lo:hi]:
        a = (int(r['Start_Timestamp']) - t0) / 1e3
        b = (int(r['End_Timestamp']) - t0) / 1e3
        name = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('a2m::', '')[:48]
        grid = f"{r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}/{r['Workgroup_Size_X']}"
        print(f"q{queues.index(r['Queue_Id'])} {a:8.1f} {b:8.1f} {b - a:7.1f}  {name:48s} {grid}")


if __name__ == '__main__':
    main()
