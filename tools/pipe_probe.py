"""Per-launch A/B of the software-pipelined tile (gemm_pipe.h) against gemm_tile on the step's
one-wave-per-SIMD shapes (diagnostic).  Run twice, A2M_GEMM_PIPE=1 / 0:
    python tools/pipe_probe.py [bf16]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'audio-to-motion-generation_amd'))
sys.path.insert(0, REPO)
import torch  # noqa: E402

BF16 = 'bf16' in sys.argv[1:]
sys.argv[1:] = [a for a in sys.argv[1:] if a != 'bf16']   # tools.conv_ab reads the rest as shapes

from a2m import functional as F  # noqa: E402
from tools.conv_ab import graph_time  # noqa: E402

dev = torch.device('cuda')
tag = 'pipe' if os.environ.get('A2M_GEMM_PIPE', '1') != '0' else 'tile'
if BF16:
    import a2m
    a2m.set_gemm_precision('bf16')
    tag += '-bf16'
torch.manual_seed(0)
for M, N, K in [(256, 4096, 768), (256, 4096, 256), (256, 4096, 512), (2688, 4096, 256), (256, 4096, 2688),
                (512, 2048, 1024), (1024, 2048, 2048)]:
    A = torch.randn(M, K, device=dev)
    B = torch.randn(N, K, device=dev)
    C = torch.empty(M, N, device=dev)
    run = lambda: F.gemm(M, N, K, A, K, 1, B, K, 1, C, N, 1)  # noqa: E731
    us = graph_time(run)
    run()
    ref = (A.double() @ B.double().t())
    err = ((C.double() - ref).abs().max() / ref.abs().max()).item()
    print(f'{tag} gemm {M}x{N}x{K}: {us:7.1f} us {2.0 * M * N * K / us / 1e6:6.1f} TF err {err:.1e} '
          f'sum {C.double().sum().item():.10e}', flush=True)
for M, N, K in [(2688, 4096, 256), (640, 4096, 256), (104, 4096, 256)]:   # row-contiguous B (mode 3)
    A = torch.randn(M, K, device=dev)
    Bt = torch.randn(K, N, device=dev)
    C = torch.empty(M, N, device=dev)
    run = lambda: F.gemm(M, N, K, A, K, 1, Bt, 1, N, C, N, 1)  # noqa: E731
    us = graph_time(run)
    run()
    ref = (A.double() @ Bt.double())
    err = ((C.double() - ref).abs().max() / ref.abs().max()).item()
    print(f'{tag} gemm-kr {M}x{N}x{K}: {us:7.1f} us {2.0 * M * N * K / us / 1e6:6.1f} TF err {err:.1e} '
          f'sum {C.double().sum().item():.10e}', flush=True)
for B, Ci, Co, T in [(64, 256, 256, 64), (64, 512, 256, 64), (64, 256, 512, 64), (64, 1024, 512, 32),
                     (64, 2048, 1024, 16), (64, 512, 512, 64)]:
    x = torch.randn(B, Ci, T, device=dev)
    w = torch.randn(Co, Ci, 3, device=dev) / (3 * Ci) ** 0.5
    b = torch.randn(Co, device=dev)
    y = torch.empty(B, Co, T, device=dev)
    cache = {}
    run = lambda: F.conv1d(x, w, b, 1, 1, act=F.ACT_LRELU, out=y, cache=cache)  # noqa: E731
    us = graph_time(run)
    run()
    ref = torch.nn.functional.leaky_relu(torch.nn.functional.conv1d(x.double(), w.double(), b.double(), padding=1), 0.2)
    err = ((y.double() - ref).abs().max() / ref.abs().max()).item()
    print(f'{tag} conv1d B={B} Ci={Ci} Co={Co} T={T}: {us:7.1f} us {2.0 * B * T * Co * Ci * 3 / us / 1e6:6.1f} TF '
          f'err {err:.1e} sum {y.double().sum().item():.10e}', flush=True)
for B, Ci, Co, H, W, kh, kw, st, ph, pw in [(64, 64, 128, 128, 46, 3, 3, 2, 1, 1), (64, 128, 256, 64, 22, 3, 3, 2, 1, 1)]:
    x = torch.randn(B, H, W, Ci, device=dev)   # NHWC
    w = torch.randn(Co, Ci, kh, kw, device=dev) / (Ci * kh * kw) ** 0.5
    b = torch.randn(Co, device=dev)
    cache = {}
    try:
        run = lambda: F.conv2d_nhwc(x, w, b, st, (ph, pw), cache=cache)  # noqa: E731
        us = graph_time(run)
        y = run()
        ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).double(), w.double(), b.double(), stride=st, padding=(ph, pw))
        yy = y if y.shape == ref.shape else y.permute(0, 3, 1, 2)
        err = ((yy.double() - ref).abs().max() / ref.abs().max()).item()
        Ho, Wo = ref.shape[2], ref.shape[3]
        print(f'{tag} conv2d_nhwc B={B} Ci={Ci} Co={Co} {H}x{W}: {us:7.1f} us '
              f'{2.0 * B * Ho * Wo * Co * Ci * kh * kw / us / 1e6:6.1f} TF err {err:.1e}', flush=True)
    except Exception as e:  # signature probe
        print(f'{tag} conv2d_nhwc skipped: {e}', flush=True)
