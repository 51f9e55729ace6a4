"""Plan probe for the decoders' 1x1 projections (diagnostic): proj_in (256 -> J*64 over
[B][C][T], loader mode 3), proj_out (J*64 -> 256) and the logits, each under forced plans.
    python tools/proj_probe.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'audio-to-motion-generation_amd'))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from a2m import _native as NN  # noqa: E402
from a2m import functional as F  # noqa: E402
from tools.conv_ab import graph_time  # noqa: E402

dev = torch.device('cuda')
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(64, 256, 64, device=dev, generator=g)
for name, Co in [('hand proj_in', 2688), ('body proj_in', 640), ('hand logits', 84), ('body logits', 20)]:
    w = torch.randn(Co, 256, device=dev, generator=g) * 0.05
    b = torch.randn(Co, device=dev, generator=g)
    out = torch.empty(64, 64, Co, device=dev)
    fn = lambda: F.conv1d(x, w, b, out=out.permute(0, 2, 1))
    NN.lib.a2m_gemm_plan_override(0, 0)
    ref = fn().clone()
    t0 = graph_time(fn, iters=20, reps=5)
    line = f'{name} (M={Co}): default {t0:6.1f} us'
    for tile in (64, 128):
        for sp in (1, 2):
            NN.lib.a2m_gemm_plan_override(tile, sp)
            o = fn()
            e = ((o - ref).abs().max() / ref.abs().max()).item()
            t = graph_time(fn, iters=20, reps=5)
            line += f' | {tile}/{sp}: {t:6.1f}' + ('' if e < 1e-5 else ' MISMATCH')
    NN.lib.a2m_gemm_plan_override(0, 0)
    print(line, flush=True)

# the same hand proj_in with x as [B*T][C] rows (dense k-contiguous B, loader mode 0)
w = torch.randn(2688, 256, device=dev, generator=g) * 0.05
xr = x.permute(0, 2, 1).contiguous().view(4096, 256)
C = torch.empty(4096, 2688, device=dev)
fn = lambda: F.gemm(2688, 4096, 256, w, 256, 1, xr, 256, 1, C, 1, 2688)
fn()
print(f'hand proj_in, dense [B*T][C] operand: {graph_time(fn, iters=20, reps=5):6.1f} us', flush=True)
