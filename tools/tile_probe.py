"""Encoder conv plans (diagnostic): every AudioEncoder layer 1..4 run channels-last (NHWC in,
NHWC out; the last layer NCHW) with forced GEMM plans (a2m_gemm_plan_override: tile code x
splits), graph-replayed, checked against the default plan; plus the current default chain
(im2col + dense for K >= 2048).  Also the non-square tiles on dense GEMMs against fp64.
   A2M_GEMM_KS2_MODES=3 python tools/tile_probe.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'audio-to-motion-generation_amd'))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from a2m import _native as NN  # noqa: E402
from a2m import functional as F  # noqa: E402
from a2m.real_motion_model import SelfAttention_G  # noqa: E402
from tools.conv_ab import graph_time  # noqa: E402

dev = torch.device('cuda')


def rel(a, b):
    return ((a.double() - b.double()).abs().max() / b.double().abs().max()).item()


def live(t, c, nhwc):
    # only the live output columns are computed (the rest of the buffer is never written)
    return t[:, :, c[0]:c[1], :] if nhwc else t[..., c[0]:c[1]]


# dense GEMM correctness of every tile code
for M, N, K in [(128, 22528, 1024), (256, 5120, 2048), (300, 1000, 500)]:
    g = torch.Generator().manual_seed(M + N)
    A = torch.randn(M, K, generator=g)
    Bm = torch.randn(N, K, generator=g)
    ref = (A.double() @ Bm.double().t())
    for tile in (64, 128):
        NN.lib.a2m_gemm_plan_override(tile, 1)
        C = torch.empty(M, N, device=dev)
        F.gemm(M, N, K, A.to(dev), K, 1, Bm.to(dev), K, 1, C, N, 1)
        e = rel(C.cpu(), ref)
        print(f'dense {M}x{N}x{K} tile {tile}: rel err {e:.1e}', flush=True)
        assert e < 1e-5
NN.lib.a2m_gemm_plan_override(0, 0)

torch.manual_seed(0)
enc = SelfAttention_G(p=0.2).to(dev).eval().audio_encoder
x = torch.randn(64, 64, 128, device=dev)
cols = enc.live_columns(128)
with torch.no_grad():
    # the current default chain, per layer
    h = x.contiguous()
    tot = 0.0
    hs = [x.unsqueeze(-1)]
    cur = x.unsqueeze(-1)
    for i, (layer, c) in enumerate(zip(enc.conv, cols)):
        k, s, p = layer.geometry()
        last = i + 1 == len(enc.conv)
        fn = (lambda h=cur, layer=layer, c=c, k=k, s=s, p=p, last=last: F.conv2d_nhwc(
            h, layer.conv.weight, layer.conv.bias, s, tuple(p), bn=layer.bn_eval(), act=layer.act,
            cols=c, out_nhwc=not last, cache=layer._nhwc))
        cur = fn()
        hs.append(cur)
    full = graph_time(lambda: enc(x))
    print(f'encoder default chain (graph): {full:.1f} us', flush=True)
    for i in range(1, 5):
        layer, c = enc.conv[i], cols[i]
        k, s, p = layer.geometry()
        last = i == 4
        hin = hs[i]
        Co, Ci = layer.conv.weight.shape[:2]
        Ho = (hin.shape[1] + 2 * p[0] - k[0]) // s + 1
        fl = 2.0 * Co * Ci * k[0] * k[1] * 64 * Ho * (c[1] - c[0])

        def fn(hin=hin, layer=layer, c=c, s=s, p=p, last=last):
            return F.conv2d_nhwc(hin, layer.conv.weight, layer.conv.bias, s, tuple(p), bn=layer.bn_eval(),
                                 act=layer.act, cols=c, out_nhwc=not last, cache=layer._nhwc)
        NN.lib.a2m_gemm_plan_override(0, 0)
        ref = fn()
        t0 = graph_time(fn)
        print(f'layer {i} Ci={Ci} Co={Co} k={k} s={s} N={64 * Ho * (c[1] - c[0])}: nhwc default plan '
              f'{t0:7.1f} us ({fl / t0 / 1e6:5.1f} TF)', flush=True)
        best = (t0, 'default')
        for tile in (64, 128):
            for sp in (1, 2, 3, 4, 6, 8, 12, 16, 24, 32):
                if sp > 1 and (Ci * k[0] * k[1]) // sp < 256:
                    continue
                NN.lib.a2m_gemm_plan_override(tile, sp)
                try:
                    out = fn()
                    e = rel(live(out, c, not last), live(ref, c, not last))
                    t = graph_time(fn)
                except Exception as ex:  # noqa: BLE001
                    print(f'   tile {tile} split {sp}: {ex}')
                    continue
                flag = '' if e < 1e-5 else f'  MISMATCH {e:.1e}'
                print(f'   tile {tile:6d} split {sp:3d}: {t:7.1f} us ({fl / t / 1e6:5.1f} TF){flag}', flush=True)
                if e < 1e-5 and t < best[0]:
                    best = (t, f'tile {tile} split {sp}')
        NN.lib.a2m_gemm_plan_override(0, 0)
        print(f'  best layer {i}: {best[1]} {best[0]:.1f} us', flush=True)
