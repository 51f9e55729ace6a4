"""Times the decoders' conv1d (B=64, 256 -> 256, k3, T=64: the tap-chunked path) under forced
GEMM plans (a2m_gemm_plan_override), eager, events around 20 launches.
    python tools/conv_plan_probe.py"""
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


for (B, Ci, Co, T) in [(64, 256, 256, 64), (64, 512, 256, 64)]:
    x = torch.randn(B, Ci, T, device=dev)
    w = torch.randn(Co, Ci, 3, device=dev) * 0.05
    b = torch.randn(Co, device=dev)
    ref = None
    for tile, split in [(0, 0), (64, 1), (64, 2), (64, 3), (64, 4), (128, 1), (128, 2), (128, 4)]:
        NN.lib.a2m_gemm_plan_override(tile, split)
        cache = {}
        y = F.conv1d(x, w, b, 1, 1, act=F.ACT_LRELU, cache=cache)
        if ref is None:
            ref = y.clone()
        err = ((y - ref).abs().max() / ref.abs().max()).item()
        us = t(lambda: F.conv1d(x, w, b, 1, 1, act=F.ACT_LRELU, cache=cache))
        print(f'conv B={B} {Ci}->{Co} T={T} tile {tile} split {split}: {us:6.1f} us '
              f'{2 * Co * Ci * 3 * B * T / us / 1e6:5.1f} TF  (vs planner {err:.1e})', flush=True)
    NN.lib.a2m_gemm_plan_override(0, 0)
