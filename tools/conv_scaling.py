"""Decoder-conv cost model probe (diagnostic): the tap-chunked k3 conv1d at M = Co = 256,
N = B*T = 4096 with Ci (K = 3 Ci) swept, and at Ci = 256 with B swept, graph-replayed.
A linear fit t = a + b*K separates per-launch fixed cost from the per-k-step cost.
    python tools/conv_scaling.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'audio-to-motion-generation_amd'))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from a2m import functional as F  # noqa: E402
from tools.conv_ab import graph_time  # noqa: E402

dev = torch.device('cuda')
g = torch.Generator(device=dev).manual_seed(0)
res = []
for B, Ci in [(64, 64), (64, 128), (64, 256), (64, 512), (64, 1024), (16, 256), (32, 256), (128, 256), (256, 256)]:
    x = torch.randn(B, Ci, 64, device=dev, generator=g)
    w = torch.randn(256, Ci, 3, device=dev, generator=g) * 0.05
    b = torch.randn(256, device=dev, generator=g)
    cache = {}
    fn = lambda: F.conv1d(x, w, b, 1, 1, cache=cache)
    t = graph_time(fn, iters=20, reps=5)
    fl = 2.0 * 256 * 3 * Ci * B * 64
    print(f'B={B:4d} Ci={Ci:5d} K={3 * Ci:5d}: {t:7.1f} us  {fl / t / 1e6:6.1f} TF', flush=True)
