"""Per-layer AudioEncoder eval timing (B=64 x T=64, graph-replayed) under forced GEMM plans
(a2m_gemm_plan_override: tile 64 / 128, split-K counts), against the planner's own choice.
Diagnostic (tools/): prints one line per (layer, plan)."""
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
PLANS = [(0, 0)] + [(t, s) for t in (64, 128) for s in (1, 2, 3, 4, 6, 8, 16, 24)]
with torch.no_grad():
    total = graph_time(lambda: enc(x), iters=10, reps=3)
    print(f'encoder graph {total:.1f} us', flush=True)
    h = x.unsqueeze(-1)
    for i, (layer, c) in enumerate(zip(enc.conv, cols)):
        k, s, p = layer.geometry()
        last = i + 1 == len(enc.conv)
        fn = lambda h=h: F.conv2d_nhwc(h, layer.conv.weight, layer.conv.bias, s, tuple(p), bn=layer.bn_eval(),  # noqa: E731
                                       act=layer.act, cols=c, out_nhwc=not last, cache=layer._nhwc)
        Co, Ci = layer.conv.weight.shape[:2]
        Ho = (h.shape[1] + 2 * p[0] - k[0]) // s + 1
        fl = 2.0 * Co * Ci * k[0] * k[1] * 64 * Ho * (c[1] - c[0])
        ref = fn()
        for tile, split in (PLANS if i > 0 else [(0, 0)]):
            N.check(N.lib.a2m_gemm_plan_override(tile, split))
            try:
                out = fn()
                err = (out - ref).abs().max().item()
                t = graph_time(fn)
            except Exception as e:  # noqa: BLE001
                print(f'layer {i} tile {tile} split {split}: {e}', flush=True)
                continue
            finally:
                N.check(N.lib.a2m_gemm_plan_override(0, 0))
            print(f'layer {i} M={Co} N={64 * Ho * (c[1] - c[0])} K={Ci * k[0] * k[1]} tile {tile:3d} split {split:2d}: '
                  f'{t:7.1f} us {fl / t / 1e6:6.1f} TF  maxdiff {err:.2e}', flush=True)
        h = ref
    t = graph_time(lambda: F.interp_time(h, 64))
    print(f'interp {t:.1f} us', flush=True)
