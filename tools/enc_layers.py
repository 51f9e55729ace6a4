"""Per-layer AudioEncoder eval timing (graph-replayed, B=64 x T=64): the NCHW chain (mode-2
gather / im2col + dense GEMM) against the channels-last chain (mode-4 runs).  Diagnostic."""
import sys
import torch
sys.path.insert(0, 'audio-to-motion-generation_amd')
from a2m import functional as F  # noqa: E402
from a2m.real_motion_model import SelfAttention_G  # noqa: E402
sys.path.insert(0, '.')
from tools.conv_ab import graph_time  # noqa: E402

torch.manual_seed(0)
enc = SelfAttention_G(p=0.2).cuda().eval().audio_encoder
x = torch.randn(64, 64, 128, device='cuda')
cols = enc.live_columns(128)
with torch.no_grad():
    hc, hn = x.unsqueeze(1), x.unsqueeze(-1)
    for i, (layer, c) in enumerate(zip(enc.conv, cols)):
        k, s, p = layer.geometry()
        last = i + 1 == len(enc.conv)
        fc = lambda h=hc: layer(h, cols=c)  # noqa: E731
        fn = lambda h=hn: F.conv2d_nhwc(h, layer.conv.weight, layer.conv.bias, s, tuple(p), bn=layer.bn_eval(),  # noqa: E731
                                        act=layer.act, cols=c, out_nhwc=not last, cache=layer._nhwc)
        tc, tn = graph_time(fc), graph_time(fn)
        Co, Ci = layer.conv.weight.shape[:2]
        Ho = (hc.shape[2] + 2 * p[0] - k[0]) // s + 1
        fl = 2.0 * Co * Ci * k[0] * k[1] * 64 * Ho * (c[1] - c[0])
        print(f'layer {i} Ci={Ci} Co={Co} k={k} s={s} cols={c}: nchw {tc:7.1f} us ({fl / tc / 1e6:5.1f} TF)  '
              f'nhwc {tn:7.1f} us ({fl / tn / 1e6:5.1f} TF)', flush=True)
        hc, hn = fc(), fn()
