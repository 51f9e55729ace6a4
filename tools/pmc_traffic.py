"""HBM traffic per launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE are too big
for one pass on gfx950), with the MI355X_MICROARCH.md corrections:

  * counter unit: kilobytes (rocprofv3's derived FETCH_SIZE/WRITE_SIZE divide by 1024);
  * gfx950 FETCH_SIZE counts exactly half the bytes of wide (16 B/lane) coalesced reads,
    so it is doubled; WRITE_SIZE is exact for 16 B/lane and dword stores.

    python tools/pmc_traffic.py FETCH_DIR WRITE_DIR [--out profiles/traffic_latest.json]

Each DIR is a rocprofv3 `-d` output directory holding a *counter_collection.csv of a
tools/step_pmc.py run; only the replayed steps' dispatches (after the marker kernel,
tools/replay_filter.py) are counted.  Kernel families are matched by substring (gemm_kernel,
logmel_kernel, graph_layer_kernel, ...).
"""
import argparse
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from replay_filter import load, replayed  # noqa: E402

FAMILIES = ('gemm_pipe_bf16_kernel', 'gemm_pipe_kernel', 'gemm_kernel', 'splitk_reduce_kernel', 'logmel2048_kernel', 'logmel_kernel',
            'graph_stack_kernel', 'graph_layer_kernel', 'graph_att_proj_kernel', 'attn_fused_eval_kernel',
            'attn_core_wide_kernel', 'conv2d_c1_kernel', 'im2col2d_kernel', 'im2col1d_kernel',
            'channel_attention_kernel', 'softmax_rows_kernel', 'layernorm_kernel')


def read_counter(d, name):
    per = defaultdict(lambda: [0, 0.0])       # family -> [dispatches, KB]
    seen = set()
    for row in replayed(load(d, '*counter_collection.csv')):
        if row.get('Counter_Name') != name:
            continue
        kn = row.get('Kernel_Name', '')
        fam = next((x for x in FAMILIES if x in kn), None)
        if fam is None:
            continue
        key = row.get('Dispatch_Id') or row.get('Correlation_Id')
        if key not in seen:
            seen.add(key)
            per[fam][0] += 1
        per[fam][1] += float(row['Counter_Value'])
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('fetch_dir')
    ap.add_argument('write_dir')
    ap.add_argument('--out', default='profiles/traffic_latest.json')
    ap.add_argument('--tag', default='')
    ap.add_argument('--steps', type=int, default=3, help='replayed steps in the PMC runs (tools/step_pmc.py R)')
    ap.add_argument('--plans', default=None, help='A2M_GEMM_LOG=1 tools/plan_log.py output of the same build: '
                    'the step\'s dense operand + output bytes, 4 (M K + K N + M N) per launch')
    a = ap.parse_args()
    fetch, write = read_counter(a.fetch_dir, 'FETCH_SIZE'), read_counter(a.write_dir, 'WRITE_SIZE')
    out = {}
    for fam in FAMILIES:
        if fam not in fetch or fam not in write:
            continue
        nf, kf = fetch[fam]
        nw, kw = write[fam]
        rd = 2.0 * kf * 1024 / nf
        wr = kw * 1024 / nw
        out[fam] = {'bytes_per_launch': round(rd + wr), 'read_bytes_per_launch': round(rd),
                    'write_bytes_per_launch': round(wr), 'dispatches': [nf, nw],
                    'source': f'rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes {a.tag}, replayed steps only; FETCH x2 (gfx950), KB x1024'}
    # the implicit-GEMM engine as one family (bench.py's roofline): tile kernels of both kinds and
    # every split-K reduce; bytes per step over the replayed steps, and per tile launch
    eng = [f for f in ('gemm_pipe_bf16_kernel', 'gemm_pipe_kernel', 'gemm_kernel', 'splitk_reduce_kernel') if f in out]
    if eng:
        steps = a.steps
        rd = sum(out[f]['read_bytes_per_launch'] * out[f]['dispatches'][0] for f in eng)
        wr = sum(out[f]['write_bytes_per_launch'] * out[f]['dispatches'][1] for f in eng)
        tiles = sum(out[f]['dispatches'][0] for f in eng if f != 'splitk_reduce_kernel')
        out['gemm_engine'] = {'bytes_per_step': round((rd + wr) / steps), 'read_bytes_per_step': round(rd / steps),
                              'write_bytes_per_step': round(wr / steps),
                              'bytes_per_launch': round((rd + wr) / max(tiles, 1)),
                              'tile_launches_per_step': tiles / steps, 'families': eng,
                              'source': out[eng[0]]['source'] + f'; {steps} replayed steps'}
    if a.plans and 'gemm_engine' in out:
        import re
        txt = open(a.plans).read().split('--- second step')[-1]
        dense = 0
        for m in re.finditer(r'M=(\d+) N=(\d+) K=(\d+) batch=(\d+)', txt):
            M, N, K, b = map(int, m.groups())
            dense += 4 * b * (M * K + K * N + M * N)
        e = out['gemm_engine']
        e['dense_operand_bytes_per_step'] = dense
        e['traffic_over_dense'] = round(e['bytes_per_step'] / dense, 3) if dense else None
        e['dense_basis'] = ('4 (M K + K N + M N) bytes per engine launch of one eager step (plan log): the '
                            'implicit B operand of a conv counted as its K x N im2col matrix')
    os.makedirs(os.path.dirname(a.out) or '.', exist_ok=True)
    with open(a.out, 'w') as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
