"""Phase breakdown of the pipelined tile per block (diagnostic build _ab/stamps.so,
-DA2M_PIPE_STAMPS=1): shader-clock cycles of prologue / k loop / epilogue, the clock rate, and
the launch's block start skew, for the last of 20 graph-replayed launches of each shape.
    A2M_LIB=_ab/stamps.so python tools/pipe_stamps.py"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'audio-to-motion-generation_amd'))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from a2m import _native as NN  # noqa: E402
from a2m import functional as F  # noqa: E402
from tools.conv_ab import graph_time  # noqa: E402

dev = torch.device('cuda')
fn = NN.lib.a2m_debug_pipe_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros(4096 * 6, dtype=np.uint64)


def report(tag, nblocks):
    torch.cuda.synchronize()
    assert fn(buf.ctypes.data, buf.size) == 0
    s = buf[:nblocks * 6].reshape(nblocks, 6).astype(np.int64)
    pro, loop, epi = s[:, 1] - s[:, 0], s[:, 2] - s[:, 1], s[:, 3] - s[:, 2]
    rt = (s[:, 5] - s[:, 4]) * 10.0   # ns
    mhz = (s[:, 3] - s[:, 0]) / np.maximum(rt, 1) * 1e3
    start = (s[:, 4] - s[:, 4].min()) * 10.0
    end = (s[:, 5] - s[:, 4].min()) * 10.0
    print(f'{tag}: blocks {nblocks}  cycles prologue {np.median(pro):.0f} loop {np.median(loop):.0f} '
          f'epilogue {np.median(epi):.0f} (median; loop max {pro.max() + loop.max()})  clock {np.median(mhz):.0f} MHz  '
          f'start skew {np.median(start):.0f}/{start.max():.0f} ns  last end {end.max():.0f} ns', flush=True)


torch.manual_seed(0)
for M, N, K in [(256, 4096, 768), (256, 4096, 256), (256, 4096, 2688)]:
    A = torch.randn(M, K, device=dev)
    B = torch.randn(N, K, device=dev)
    C = torch.empty(M, N, device=dev)
    run = lambda: F.gemm(M, N, K, A, K, 1, B, K, 1, C, N, 1)  # noqa: E731
    us = graph_time(run)
    report(f'gemm {M}x{N}x{K} ({us:.1f} us/launch)', (M // 64) * (N // 64))
for B, Ci, Co, T in [(64, 256, 256, 64)]:
    x = torch.randn(B, Ci, T, device=dev)
    w = torch.randn(Co, Ci, 3, device=dev) / (3 * Ci) ** 0.5
    b = torch.randn(Co, device=dev)
    y = torch.empty(B, Co, T, device=dev)
    cache = {}
    run = lambda: F.conv1d(x, w, b, 1, 1, act=F.ACT_LRELU, out=y, cache=cache)  # noqa: E731
    us = graph_time(run)
    report(f'conv1d B={B} Ci={Ci} Co={Co} T={T} ({us:.1f} us/launch)', (Co // 64) * (B * T // 64))
