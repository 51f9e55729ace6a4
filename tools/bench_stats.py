"""Cross-check of the bench line's roofline against a rocprofv3 --kernel-trace --stats run of the
same bench command (tools/gpu_round.sh): the engine family's average launch duration (tile kernels
and split-K reduces) over every launch of the run (the timed replays dominate: 200 steps x 47
launches) against the line's roofline (its replayed-step kernel trace), and the top kernels.

    python tools/bench_stats.py PROF_DIR BENCH_JSON_LINE_FILE [--out file.txt]
"""
import argparse
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('prof_dir')
    ap.add_argument('bench_json')
    ap.add_argument('--out', default=None)
    a = ap.parse_args()
    fn = glob.glob(os.path.join(a.prof_dir, '**', '*kernel_stats.csv'), recursive=True)[0]
    rows = list(csv.DictReader(open(fn, newline='')))
    line = json.loads([x for x in open(a.bench_json) if x.startswith('{')][-1])
    def engine(n):
        return 'gemm_kernel' in n or 'gemm_pipe' in n or 'splitk_reduce' in n
    calls = sum(int(r['Calls']) for r in rows if engine(r['Name']))
    ns = sum(float(r['TotalDurationNs']) for r in rows if engine(r['Name']))
    rp = line['roofline']
    avg_ms = ns / calls / 1e6
    n_launch = rp.get('trace_launches_per_step') or (rp['launches_per_step'] + rp.get('reduces_per_step', 0))
    line_avg = rp['family_ms_per_step'] / n_launch
    gfl = rp['gflop_per_step'] / n_launch
    out = [f'rocprofv3 --kernel-trace --stats of `python bench.py --no-cpu-baseline --no-trace` ({os.path.basename(fn)})',
           f'bench line: {line["ms_per_step"]} ms/step, roofline {rp["achieved"]} TF = {rp["frac"]} '
           f'({rp["family_ms_per_step"]} ms of engine per step over {n_launch} launches = {line_avg:.4f} ms per '
           f'launch, {gfl:.3f} GFLOP per launch on average)',
           f'rocprof engine family (gemm_kernel / gemm_pipe_kernel / splitk_reduce*) over the whole command: '
           f'{calls} launches, average {avg_ms:.4f} ms -> {gfl / avg_ms:.2f} TF = {gfl / avg_ms / rp["peak"]:.4f} of '
           f'{rp["peak"]}; line / rocprof average = {line_avg / avg_ms:.4f}',
           '', 'Calls  TotalDurationNs  AverageNs  Percentage  Name']
    for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:30]:
        out.append(f'{r["Calls"]:>6} {float(r["TotalDurationNs"]):>15.0f} {float(r["AverageNs"]):>10.0f} '
                   f'{float(r["Percentage"]):>10.2f}  {r["Name"][:110]}')
    txt = '\n'.join(out)
    print('\n'.join(out[:3]))
    if a.out:
        with open(a.out, 'w') as f:
            f.write(txt + '\n')


if __name__ == '__main__':
    main()
