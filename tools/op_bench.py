"""Per-op timing on the GPU (HIP events), for tuning: the G forward's dominant shapes.
usage: python tools/op_bench.py [filter]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'audio-to-motion-generation_amd'))
import torch  # noqa: E402

from a2m import functional as F  # noqa: E402
from a2m import skeleton as S  # noqa: E402

dev = torch.device('cuda')


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def conv_case(B, Ci, Co, T, k, s, p):
    x = torch.randn(B, Ci, T, device=dev)
    w = torch.randn(Co, Ci, k, device=dev) * 0.02
    b = torch.zeros(Co, device=dev)
    bn = (torch.ones(Co, device=dev), torch.zeros(Co, device=dev), torch.zeros(Co, device=dev),
          torch.ones(Co, device=dev), 1e-5)
    Tout = (T + 2 * p - k) // s + 1
    y = torch.empty(B, Co, Tout, device=dev)
    us = timeit(lambda: F.conv1d(x, w, b, s, p, bn=bn, act=F.ACT_LRELU, out=y))
    return us, 2.0 * Co * Ci * k * B * Tout


def convt_case(B, Ci, Co, T):
    x = torch.randn(B, Ci, T, device=dev)
    w = torch.randn(Ci, Co, 3, device=dev) * 0.02
    y = torch.empty(B, Co, 2 * T, device=dev)
    us = timeit(lambda: F.convt1d(x, w, None, out=y))
    return us, 2.0 * Co * Ci * 3 * B * T


def attn_case(B, C, T):
    x = torch.randn(B, C, T, device=dev)
    ws = [torch.randn(C // 8, C, device=dev) * 0.02, torch.zeros(C // 8, device=dev),
          torch.randn(C // 8, C, device=dev) * 0.02, torch.zeros(C // 8, device=dev),
          torch.randn(C, C, device=dev) * 0.02, torch.zeros(C, device=dev), torch.ones(1, device=dev)]
    y = torch.empty_like(x)
    us = timeit(lambda: F.self_attention(x, *ws, out=y))
    return us, 2.0 * B * T * C * (C + C // 4) + 4.0 * B * T * T * C


def graph_case(J, lo, kind, B=64, T=64):
    x = torch.randn(B * T * J, 64, device=dev)
    ptr, idx = [t.to(dev) for t in S.in_neighbour_csr(S.edge_index(lo, J), J)]
    w0 = torch.randn(256 if kind == 0 else 64, 64, device=dev) * 0.1
    w1 = torch.randn(64, 64, device=dev) * 0.1
    a = torch.randn(1, 4, 64, device=dev) * 0.1
    bias, lw, lb = torch.zeros(64, device=dev), torch.ones(64, device=dev), torch.zeros(64, device=dev)
    y = torch.empty_like(x)
    us = timeit(lambda: F.graph_layer(x, J, kind, ptr, idx, w0, w1, a, a, bias, lw, lb, out=y))
    return us, 2.0 * x.shape[0] * 64 * (256 if kind == 0 else 128)


def dense_case(M, N, K):
    A = torch.randn(M, K, device=dev)
    Bm = torch.randn(N, K, device=dev)
    C = torch.empty(M, N, device=dev)
    us = timeit(lambda: F.gemm(M, N, K, A, K, 1, Bm, K, 1, C, N, 1), iters=10)
    return us, 2.0 * M * N * K


def dense_nn_case(M, N, K):
    """B stored [K][N] (row-contiguous operand, the [B,C,T] activation orientation)."""
    A = torch.randn(M, K, device=dev)
    Bm = torch.randn(K, N, device=dev)
    C = torch.empty(M, N, device=dev)
    us = timeit(lambda: F.gemm(M, N, K, A, K, 1, Bm, 1, N, C, N, 1), iters=10)
    return us, 2.0 * M * N * K


def norm_case(B=256, T=64):
    from a2m import normalization as NZ
    pose = torch.randn(B, T, 104, device=dev)
    mean, std = torch.randn(104, device=dev), torch.rand(104, device=dev) + 0.5
    out = torch.empty_like(pose)
    us = timeit(lambda: NZ.necksub_normalize(pose, mean, std, out=out))
    return us, 2.0 * pose.numel() * 4 / 1e6 * 1e6  # bytes moved (reported as 'TFLOP/s' column = MB/us)


def pck_case(N=4096, K=52):
    from a2m.evaluation import compute_pck
    gt = torch.randn(N, 2, K, device=dev)
    pred = gt + 0.1 * torch.randn_like(gt)
    us = timeit(lambda: compute_pck(pred, gt))
    return us, 2.0 * gt.numel() * 4


CASES = {
    'unet.d0 256->512 k3 T64': lambda: conv_case(64, 256, 512, 64, 3, 1, 1),
    'unet.d1 512->512 k4s2 T64': lambda: conv_case(64, 512, 512, 64, 4, 2, 1),
    'unet.d2 512->1024 k3 T32': lambda: conv_case(64, 512, 1024, 32, 3, 1, 1),
    'unet.d3 1024->1024 k4s2 T32': lambda: conv_case(64, 1024, 1024, 32, 4, 2, 1),
    'unet.bott 1024->2048 k3 T16': lambda: conv_case(64, 1024, 2048, 16, 3, 1, 1),
    'unet.up1 2048->1024 k3 T32': lambda: conv_case(64, 2048, 1024, 32, 3, 1, 1),
    'unet.up3 1024->512 k3 T64': lambda: conv_case(64, 1024, 512, 64, 3, 1, 1),
    'dec 256->256 k3 T64': lambda: conv_case(64, 256, 256, 64, 3, 1, 1),
    'convT 2048->1024 T16': lambda: convt_case(64, 2048, 1024, 16),
    'convT 1024->512 T32': lambda: convt_case(64, 1024, 512, 32),
    'attn C2048 T16': lambda: attn_case(64, 2048, 16),
    'attn C2048 T32': lambda: attn_case(64, 2048, 32),
    'attn C256 T64': lambda: attn_case(64, 256, 64),
    'dense 4096^3': lambda: dense_case(4096, 4096, 4096),
    'dense up1 1024x2048x6144': lambda: dense_case(1024, 2048, 6144),
    'denseNN up1 1024x2048x6144': lambda: dense_nn_case(1024, 2048, 6144),
    'denseNN up3 512x4096x3072': lambda: dense_nn_case(512, 4096, 3072),
    'dense bott 2048x1024x3072': lambda: dense_case(2048, 1024, 3072),
    'dense up3 512x4096x3072': lambda: dense_case(512, 4096, 3072),
    'dense d2 1024x2048x1536': lambda: dense_case(1024, 2048, 1536),
    'dense dec 256x4096x768': lambda: dense_case(256, 4096, 768),
    'gat body': lambda: graph_case(10, 0, 0),
    'bytes: pose normalize B256 T64': norm_case,
    'bytes: pck N4096 K52': pck_case,
    'gat hand': lambda: graph_case(42, 10, 0),
    'gconv hand': lambda: graph_case(42, 10, 1),
}

if __name__ == '__main__':
    flt = sys.argv[1] if len(sys.argv) > 1 else ''
    tag = '/'.join(os.environ.get(k, '-') for k in ('A2M_GEMM_TILE', 'A2M_GEMM_SPLIT', 'A2M_GEMM_BK', 'A2M_GEMM_XCD'))
    for name, fn in CASES.items():
        if flt not in name:
            continue
        us, fl = fn()
        print(f'[{tag}] {name:32s} {us:9.1f} us  {fl / us / 1e6:7.2f} TFLOP/s', flush=True)
