"""Sweep the GEMM engine's (tile, split-K) choice over the G forward's shapes (HIP events).
usage: python tools/gemm_tune.py [nt|nn]   -- nt: both operands k-contiguous (mode 0,0);
nn: B stored [K][N] (mode 0,3, the conv-activation orientation)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'audio-to-motion-generation_amd'))
import torch  # noqa: E402

from a2m import _native as N  # noqa: E402
from a2m import functional as F  # noqa: E402

dev = torch.device('cuda')
SHAPES = [(4096, 4096, 4096), (256, 4096, 768), (2560, 2048, 2048), (1024, 2048, 6144),
          (320, 4096, 256), (2560, 1024, 2048), (2688, 4096, 256), (512, 4096, 2304),
          (2048, 1024, 3072), (512, 4096, 3072), (1024, 1024, 4096), (256, 5120, 2048),
          (1024, 2048, 1536), (256, 512, 12288), (256, 4096, 2688), (512, 2048, 2048),
          (512, 4096, 768), (512, 2048, 1024), (640, 4096, 256), (256, 4096, 640)]


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    nn = len(sys.argv) > 1 and sys.argv[1] == 'nn'
    for M, Nn, K in SHAPES:
        A = torch.randn(M, K, device=dev)
        if nn:
            Bm = torch.randn(K, Nn, device=dev)
            run = lambda: F.gemm(M, Nn, K, A, K, 1, Bm, 1, Nn, C, Nn, 1)  # noqa: E731
        else:
            Bm = torch.randn(Nn, K, device=dev)
            run = lambda: F.gemm(M, Nn, K, A, K, 1, Bm, K, 1, C, Nn, 1)  # noqa: E731
        C = torch.empty(M, Nn, device=dev)
        fl = 2.0 * M * Nn * K
        N.check(N.lib.a2m_gemm_plan_override(0, 0))
        auto = timeit(run)
        res = []
        for tile in (64, 128):
            for s in (1, 2, 3, 4, 6, 8, 12, 16):
                if K // s < 128:
                    continue
                N.check(N.lib.a2m_gemm_plan_override(tile, s))
                res.append((timeit(run), tile, s))
        N.check(N.lib.a2m_gemm_plan_override(0, 0))
        res.sort()
        best = res[0]
        print(f'{M:5d} {Nn:5d} {K:5d}  auto {auto:7.1f} us {fl / auto / 1e6:6.1f} TF | best {best[0]:7.1f} us '
              f'{fl / best[0] / 1e6:6.1f} TF tile {best[1]} s {best[2]} | ' +
              ' '.join(f'{t}/{s}:{u:.0f}' for u, t, s in sorted(res, key=lambda r: (r[1], r[2]))), flush=True)


if __name__ == '__main__':
    main()
