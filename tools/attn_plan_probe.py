"""Times the UNet's SelfAttention(2048) (T = 16 / 32, B = 64) eval call under forced GEMM plans
for its QKV projection (a2m_gemm_plan_override).   python tools/attn_plan_probe.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'audio-to-motion-generation_amd'))
import torch  # noqa: E402

from a2m import functional as F  # noqa: E402
from a2m import _native as NN  # noqa: E402

dev = torch.device('cuda')


def t(fn, it=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / it


C = 2048
for T in (16, 32):
    x = torch.randn(64, C, T, device=dev)
    wq, wk = torch.randn(C // 8, C, 1, device=dev) * 0.02, torch.randn(C // 8, C, 1, device=dev) * 0.02
    wv = torch.randn(C, C, 1, device=dev) * 0.02
    bq, bk, bv = torch.randn(C // 8, device=dev), torch.randn(C // 8, device=dev), torch.randn(C, device=dev)
    g = torch.full((1,), 0.3, device=dev)
    ref = None
    for tile, split in [(0, 0), (64, 1), (64, 2), (128, 1), (128, 2), (128, 3), (128, 4)]:
        NN.lib.a2m_gemm_plan_override(tile, split)
        cache = {}
        y = F.self_attention(x, wq, bq, wk, bk, wv, bv, g, cache=cache)
        if ref is None:
            ref = y.clone()
        err = ((y - ref).abs().max() / ref.abs().max()).item()
        us = t(lambda: F.self_attention(x, wq, bq, wk, bk, wv, bv, g, cache=cache))
        print(f'attn C={C} T={T} tile {tile} split {split}: {us:6.1f} us (vs planner {err:.1e})', flush=True)
    NN.lib.a2m_gemm_plan_override(0, 0)
