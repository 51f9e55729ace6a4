"""Per-step kernel breakdown of the graph-replayed bench steps in a rocprofv3 kernel trace of
tools/step_pmc.py (dispatches after the marker only, tools/replay_filter.py), and the GEMM
engine's in-step roofline figure from it: algorithmic FLOPs per step (bench.py
g_forward GEMM count, passed in) / summed GEMM-engine durations per step (both tile kernels and the
split-K reduces, as bench.py's roofline).

    python tools/replay_breakdown.py TRACE_DIR_or_kernel_trace.csv STEPS [--gflop 184.4] [--out f.txt]
"""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from replay_filter import load, replayed  # noqa: E402

FP32_PEAK = 157.3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('trace')
    ap.add_argument('steps', type=int)
    ap.add_argument('--gflop', type=float, default=None, help='engine GFLOP per step (bench line)')
    ap.add_argument('--peak', type=float, default=FP32_PEAK)
    ap.add_argument('--out', default=None)
    a = ap.parse_args()
    rows = replayed(load(a.trace, '*kernel_trace.csv'))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in rows:
        k = r['Kernel_Name'].split('(')[0].replace('void ', '')[:80]
        agg[k][0] += 1
        agg[k][1] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    n = a.steps
    tot = sum(v[1] for v in agg.values())
    span = (int(rows[-1]['End_Timestamp']) - int(rows[0]['Start_Timestamp'])) / 1e3
    lines = [f'{len(rows)} dispatches after the marker = {n} replayed steps; first-to-last span '
             f'{span / n:.1f} us/step; kernel-time sum {tot / n:.1f} us/step']
    def engine(k):
        return 'gemm_kernel' in k or 'gemm_pipe' in k or 'splitk_reduce' in k
    gemm = sum(v[1] for k, v in agg.items() if engine(k)) / n
    gcalls = sum(v[0] for k, v in agg.items() if engine(k)) / n
    lines.append(f'GEMM engine (gemm_kernel + gemm_pipe_kernel + splitk_reduce): {gcalls:.1f} launches/step, {gemm:.1f} us/step')
    if a.gflop:
        tf = a.gflop * 1e9 / (gemm * 1e-6) / 1e12
        lines.append(f'gemm roofline: {a.gflop:.1f} GFLOP / {gemm:.1f} us = {tf:.1f} TF = {tf / a.peak:.4f} of {a.peak}')
    for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        lines.append(f'{t / n:9.1f} us/step {c / n:6.1f} calls/step {t / c:8.1f} us/call {100 * t / tot:5.1f}%  {k}')
    txt = '\n'.join(lines)
    print(txt)
    if a.out:
        with open(a.out, 'w') as f:
            f.write(txt + '\n')


if __name__ == '__main__':
    main()
