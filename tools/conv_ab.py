"""conv1d (k=3, stride 1) timing: im2col + dense GEMM against the tap-chunked path (loader mode 5),
per engine precision, graph-replayed (device time per conv incl. the im2col launch).
usage: PREC=fp32,bf16x6 python tools/conv_ab.py [B,Ci,Co,T ...]   (diagnostic, tools/)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'audio-to-motion-generation_amd'))
import torch  # noqa: E402

import a2m  # noqa: E402
from a2m import functional as F  # noqa: E402

dev = torch.device('cuda')
SHAPES = [(64, 256, 256, 64), (64, 256, 512, 64), (64, 512, 1024, 32), (64, 1024, 2048, 16),
          (64, 2048, 1024, 32), (64, 1024, 512, 64)]
if len(sys.argv) > 1:
    SHAPES = [tuple(int(v) for v in a.split(',')) for a in sys.argv[1:]]
PRECS = os.environ.get('PREC', 'fp32').split(',')


def graph_time(fn, iters=20, reps=3):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(iters):
                fn()
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            g.replay()
        e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * iters)


def main():
    for B, Ci, Co, T in SHAPES:
        x = torch.randn(B, Ci, T, device=dev)
        w = torch.randn(Co, Ci, 3, device=dev) / (3 * Ci) ** 0.5
        b = torch.randn(Co, device=dev)
        y = torch.empty(B, Co, T, device=dev)
        ref = torch.nn.functional.conv1d(x.double().cpu(), w.double().cpu(), b.double().cpu(), padding=1)
        flops = 2.0 * B * T * Co * Ci * 3
        for prec in PRECS:
            a2m.set_gemm_precision(prec)
            for name, cache in (('im2col', None), ('tap', {})):
                us = graph_time(lambda: F.conv1d(x, w, b, 1, 1, act=F.ACT_LRELU, out=y, cache=cache))
                F.conv1d(x, w, b, 1, 1, out=y, cache=cache)
                err = ((y.double().cpu() - ref).abs().max() / ref.abs().max()).item()
                print(f'conv B={B} Ci={Ci} Co={Co} T={T} {prec:6s} {name:6s}: {us:7.1f} us '
                      f'{flops / us / 1e6:6.1f} TF  rel err {err:.1e}', flush=True)
    a2m.set_gemm_precision('fp32')


if __name__ == '__main__':
    main()
