"""MFMA utilisation per kernel family from a rocprofv3 PMC pass of
SQ_VALU_MFMA_BUSY_CYCLES + SQ_BUSY_CYCLES + GRBM_GUI_ACTIVE and a kernel-trace pass of the
same command (tools/step_pmc.sh), replayed steps only (tools/replay_filter.py).

  busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x cycles), cycles = GRBM_GUI_ACTIVE / 8
  (rocprofv3 sums GRBM_GUI_ACTIVE over the 8 XCDs: MI355X_MICROARCH.md, DVFS give-back).
The counter's scale is calibrated in DESIGN.md against the engine's known MFMA count
(mfma_cycles_per_mfma below: busy cycles per v_mfma_f32_32x32x2_f32).

    python tools/pmc_mfma.py MFMA_DIR TRACE_DIR [--out file.json]
"""
import argparse
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from replay_filter import load, replayed  # noqa: E402

FAMILIES = ('gemm_pipe_bf16_kernel', 'gemm_pipe_kernel', 'gemm_kernel', 'splitk_reduce_kernel', 'graph_stack_kernel', 'logmel2048_kernel', 'graph_layer_kernel',
            'attn_fused_eval_kernel', 'attn_core', 'im2col', 'channel_att', 'layernorm_kernel')


def fam_of(name):
    return next((f for f in FAMILIES if f in name), 'other')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('mfma_dir')
    ap.add_argument('trace_dir')
    ap.add_argument('--out', default=None)
    a = ap.parse_args()
    per = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in replayed(load(a.mfma_dir, '*counter_collection.csv')):
        f = fam_of(r['Kernel_Name'])
        per[f][r['Counter_Name']] += float(r['Counter_Value'])
        disp[f].add(r.get('Dispatch_Id') or r.get('Correlation_Id'))
    dur = defaultdict(lambda: [0, 0.0])
    for r in replayed(load(a.trace_dir, '*kernel_trace.csv')):
        f = fam_of(r['Kernel_Name'])
        dur[f][0] += 1
        dur[f][1] += float(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
    out = {}
    for f, d in sorted(per.items()):
        n = len(disp[f])
        cyc = d.get('GRBM_GUI_ACTIVE', 0.0) / 8.0
        busy = d.get('SQ_VALU_MFMA_BUSY_CYCLES', 0.0)
        out[f] = {'dispatches': n, 'mfma_busy_cycles_per_launch': busy / max(n, 1),
                  'gpu_cycles_per_launch': cyc / max(n, 1),
                  'busy_frac': busy / (1024.0 * cyc) if cyc else None,
                  'trace_avg_us': dur[f][1] / max(dur[f][0], 1) / 1e3 if f in dur else None}
    # the GEMM engine as one family (bench.py's roofline): both tile kernels and the split-K reduces
    eng = [f for f in ('gemm_pipe_bf16_kernel', 'gemm_pipe_kernel', 'gemm_kernel', 'splitk_reduce_kernel') if f in per]
    if eng:
        cyc = sum(per[f].get('GRBM_GUI_ACTIVE', 0.0) for f in eng) / 8.0
        busy = sum(per[f].get('SQ_VALU_MFMA_BUSY_CYCLES', 0.0) for f in eng)
        out['gemm_engine'] = {'families': eng, 'dispatches': sum(len(disp[f]) for f in eng),
                              'busy_frac': busy / (1024.0 * cyc) if cyc else None}
    txt = json.dumps(out, indent=1)
    print(txt)
    if a.out:
        with open(a.out, 'w') as fh:
            fh.write(txt)


if __name__ == '__main__':
    main()
