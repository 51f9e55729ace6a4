"""Fused eval SelfAttention (a2m_self_attention_eval_f32) at the decoders' shape, graph-replayed
(diagnostic).   python tools/attn_probe.py"""
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
C, T, B = 256, 64, 64
x = torch.randn(B, C, T, device=dev, generator=g)
res = torch.randn(B, C, T, device=dev, generator=g)
W = [torch.randn(C // 8, C, device=dev, generator=g) * 0.05, torch.randn(C // 8, device=dev, generator=g),
     torch.randn(C // 8, C, device=dev, generator=g) * 0.05, torch.randn(C // 8, device=dev, generator=g),
     torch.randn(C, C, device=dev, generator=g) * 0.05, torch.randn(C, device=dev, generator=g),
     torch.tensor([0.4], device=dev)]
cache = {}
out = torch.empty_like(x)
fn = lambda: F.self_attention(x, *W, res=res, out=out, cache=cache)
print(f'fused eval attention B={B} C={C} T={T}: {graph_time(fn, iters=20, reps=5):.1f} us', flush=True)
