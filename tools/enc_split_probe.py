"""AudioEncoder eval at B=64 x T=64, graph-replayed (diagnostic, tools/): the default chain
against (a) per-layer forced GEMM plans and (b) the batch split into halves on two streams
forked and joined inside the graph (so one half's latency-bound kernels overlap the other's
GEMMs).  Prints one line per variant."""
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


def chain(xx, plans=None):
    h = xx.unsqueeze(-1)
    for i, (layer, c) in enumerate(zip(enc.conv, cols)):
        k, s, p = layer.geometry()
        last = i + 1 == len(enc.conv)
        if plans is not None:
            N.check(N.lib.a2m_gemm_plan_override(*plans[i]))
        h = F.conv2d_nhwc(h, layer.conv.weight, layer.conv.bias, s, tuple(p), bn=layer.bn_eval(),
                          act=layer.act, cols=c, out_nhwc=not last, cache=layer._nhwc)
    N.check(N.lib.a2m_gemm_plan_override(0, 0))
    return F.interp_time(h, 64)


def split2(plans=None, parts=2):
    cur = torch.cuda.current_stream()
    side = [torch.cuda.Stream() for _ in range(parts - 1)]
    outs = []
    n = x.shape[0] // parts
    for j, st in enumerate(side):
        st.wait_stream(cur)
        with torch.cuda.stream(st):
            outs.append(chain(x[(j + 1) * n:(j + 2) * n], plans))
    outs.insert(0, chain(x[:n], plans))
    for st in side:
        cur.wait_stream(st)
    return outs


with torch.no_grad():
    ref = enc(x)
    for name, fn in [('default', lambda: enc(x)), ('chain', lambda: chain(x))]:
        print(f'{name:40s} {graph_time(fn, iters=10, reps=3):7.1f} us', flush=True)
    best = [(0, 0), (0, 0), (0, 0), (128, 4), (64, 24)]
    alt = [(0, 0), (0, 0), (128, 6), (128, 4), (64, 24)]
    alt2 = [(0, 0), (0, 0), (64, 4), (128, 4), (64, 16)]
    for name, pl in [('plans l3=128/4 l4=64/24', best), ('plans l2=128/6 l3=128/4 l4=64/24', alt),
                     ('plans l2=64/4 l3=128/4 l4=64/16', alt2)]:
        err = (chain(x, pl) - ref).abs().max().item()
        print(f'{name:40s} {graph_time(lambda: chain(x, pl), iters=10, reps=3):7.1f} us  maxdiff {err:.2e}', flush=True)
    for parts in (2, 4):
        outs = split2(parts=parts)
        err = (torch.cat(outs) - ref).abs().max().item()
        print(f'{"split" + str(parts):40s} {graph_time(lambda: split2(parts=parts), iters=10, reps=3):7.1f} us  maxdiff {err:.2e}',
              flush=True)
        for pl in (best, alt):
            print(f'{"split" + str(parts) + " + plans " + str(pl[2:]):40s} '
                  f'{graph_time(lambda: split2(pl, parts), iters=10, reps=3):7.1f} us', flush=True)
    # half-batch per-layer plan sweep (what the split chain's launches see)
    xh = x[:32]
    h = xh.unsqueeze(-1)
    for i, (layer, c) in enumerate(zip(enc.conv, cols)):
        k, s, p = layer.geometry()
        last = i + 1 == len(enc.conv)
        fn = lambda h=h: F.conv2d_nhwc(h, layer.conv.weight, layer.conv.bias, s, tuple(p), bn=layer.bn_eval(),  # noqa: E731
                                       act=layer.act, cols=c, out_nhwc=not last, cache=layer._nhwc)
        for tile, split in ([(0, 0)] + ([(t, sp) for t in (64, 128) for sp in (1, 2, 4, 6, 8, 16, 24)] if i else [])):
            N.check(N.lib.a2m_gemm_plan_override(tile, split))
            t = graph_time(fn)
            N.check(N.lib.a2m_gemm_plan_override(0, 0))
            print(f'B=32 layer {i} tile {tile:3d} split {split:2d}: {t:7.1f} us', flush=True)
        h = fn()
