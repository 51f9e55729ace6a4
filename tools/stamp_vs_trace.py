"""Per-launch comparison of the GEMM engine's span stamps (bench.py's in-step roofline basis)
with the rocprofv3 kernel trace of the same replayed dispatches (tools/step_pmc.py --stamps
under --kernel-trace).  Within each replayed step the engine launches are matched in start
order; the two clocks are aligned on the median end-time difference (a kernel's completion and
its last block's end are nearly simultaneous), so for every launch

    start_wait = stamp first-block start - trace start   (dispatch, and waiting for free CUs)
    end_tail   = trace end - stamp last-block end         (completion signalling)

and trace duration = stamp span + start_wait + end_tail.  `queued` = last block end - the
launch's ready mark (bench.py's in-step basis: the engine enqueues a one-thread mark kernel right
before each tile kernel while timing), compared with the trace duration per launch.

    python tools/stamp_vs_trace.py TRACE_DIR STAMPS.json [--out f.txt]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from replay_filter import load, replayed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('trace')
    ap.add_argument('stamps')
    ap.add_argument('--out', default=None)
    a = ap.parse_args()
    reps = json.load(open(a.stamps))['replays']
    rows = [r for r in replayed(load(a.trace, '*kernel_trace.csv')) if 'gemm_kernel' in r['Kernel_Name']]
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    per = len(reps[0])
    assert len(rows) == per * len(reps), (len(rows), per, len(reps))
    dur, span, wait, tail, qd = [[0.0] * per for _ in range(5)]
    for k, st in enumerate(reps):
        tr = rows[k * per:(k + 1) * per]
        st = sorted([tuple(x) if len(x) == 3 else (None,) + tuple(x) for x in st], key=lambda x: x[1])
        ts = [(int(r['Start_Timestamp']) / 1e3, int(r['End_Timestamp']) / 1e3) for r in tr]
        off = statistics.median(t[1] - s[2] for t, s in zip(ts, st))
        for i, (t, s) in enumerate(zip(ts, st)):
            dur[i] += (t[1] - t[0]) / len(reps)
            span[i] += (s[2] - s[1]) / len(reps)
            wait[i] += (s[1] + off - t[0]) / len(reps)
            tail[i] += (t[1] - (s[2] + off)) / len(reps)
            qd[i] += (s[2] - s[0]) / len(reps) if s[0] is not None else 0.0
    lines = [f'{len(reps)} replayed steps, {per} engine launches each (matched in start order)',
             f'per step: trace {sum(dur):.1f} us, stamp spans {sum(span):.1f} us, start waits '
             f'{sum(wait):.1f} us, end tails {sum(tail):.1f} us',
             f'per launch: trace - span mean {(sum(dur) - sum(span)) / per:.2f} us, median '
             f'{statistics.median(d - s for d, s in zip(dur, span)):.2f} us',
             f'per step: queued (ready mark .. last end) {sum(qd):.1f} us = {sum(qd) / sum(dur):.4f} of the trace',
             ' idx  trace_us  span_us  start_wait  end_tail  queued_us']
    for i in range(per):
        lines.append(f'{i:4d} {dur[i]:9.1f} {span[i]:8.1f} {wait[i]:10.1f} {tail[i]:9.1f} {qd[i]:10.1f}')
    txt = '\n'.join(lines)
    print(txt)
    if a.out:
        with open(a.out, 'w') as f:
            f.write(txt + '\n')


if __name__ == '__main__':
    main()
