"""AudioEncoder eval (B=64 x T=64, graph-replayed) under per-layer forced GEMM plans, the
variants interleaved over several rounds after a warm-up (so clock ramp-up does not favour
the later ones).  Diagnostic (tools/)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'audio-to-motion-generation_amd'))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from a2m import functional as F  # noqa: E402
from a2m import _native as N  # noqa: E402
from a2m.real_motion_model import SelfAttention_G  # noqa: E402
from tools.conv_ab import graph_time  # noqa: E402

torch.manual_seed(0)
enc = SelfAttention_G(p=0.2).cuda().eval().audio_encoder
x = torch.randn(64, 64, 128, device='cuda')
cols = enc.live_columns(128)


def chain(plans=None, fused=True):
    h = x.unsqueeze(-1)
    for i, (layer, c) in enumerate(zip(enc.conv, cols)):
        k, s, p = layer.geometry()
        if plans is not None:
            N.check(N.lib.a2m_gemm_plan_override(*plans[i]))
        if i + 1 == len(enc.conv) and fused:
            h = F.conv2d_nhwc_interp(h, layer.conv.weight, layer.conv.bias, s, tuple(p), 64, c[0],
                                     bn=layer.bn_eval(), act=layer.act, cache=layer._nhwc)
        else:
            h = F.conv2d_nhwc(h, layer.conv.weight, layer.conv.bias, s, tuple(p), bn=layer.bn_eval(),
                              act=layer.act, cols=c, out_nhwc=i + 1 < len(enc.conv), cache=layer._nhwc)
    N.check(N.lib.a2m_gemm_plan_override(0, 0))
    return h if fused else F.interp_time(h, 64)


Z = (0, 0)
VARIANTS = {
    'enc(x) default': lambda: enc(x),
    'unfused interp, default plans': lambda: chain(fused=False),
    'l2 64/4 l3 64/1 l4 64/16': lambda: chain([Z, Z, (64, 4), (64, 1), (64, 16)]),
    'l2 64/4 l3 128/4 l4 64/16': lambda: chain([Z, Z, (64, 4), (128, 4), (64, 16)]),
    'l2 128/3 l3 128/4 l4 64/16': lambda: chain([Z, Z, (128, 3), (128, 4), (64, 16)]),
    'l2 128/6 l3 128/4 l4 64/16': lambda: chain([Z, Z, (128, 6), (128, 4), (64, 16)]),
    'l2 64/4 l3 128/4 l4 64/24': lambda: chain([Z, Z, (64, 4), (128, 4), (64, 24)]),
    'l2 64/6 l3 128/4 l4 64/16': lambda: chain([Z, Z, (64, 6), (128, 4), (64, 16)]),
    'l2 64/4 l3 128/8 l4 64/16': lambda: chain([Z, Z, (64, 4), (128, 8), (64, 16)]),
}
with torch.no_grad():
    ref = enc(x)
    for name, fn in VARIANTS.items():
        e = (fn() - ref).abs().max().item()
        assert e < 1e-5, (name, e)
    for _ in range(3):   # warm-up: clocks
        graph_time(lambda: enc(x), iters=10, reps=10)
    res = {k: [] for k in VARIANTS}
    for r in range(4):
        for name, fn in VARIANTS.items():
            res[name].append(graph_time(fn, iters=10, reps=5))
    for name, ts in res.items():
        print(f'{name:34s} min {min(ts):6.1f} us  median {sorted(ts)[len(ts) // 2]:6.1f}  '
              + ' '.join(f'{t:.1f}' for t in ts), flush=True)
