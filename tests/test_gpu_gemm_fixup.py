"""The engine's in-launch split-K combine (A2M_GEMM_FIXUP=1, gemm_kernel.h: the last-arriving
split block of each output tile sums the write-through slabs in fixed order and runs the
epilogue) against the default separate reduce kernel.  The summation order is the reduce
kernel's (0 + slab 0 + slab 1 + ...), so the outputs must agree bit for bit over split plans
on both tile sizes, the tap-conv and dense loaders, a batched launch, the BN + LeakyReLU
epilogue and the m-contiguous (staged through LDS) output -- and stay equal over repeated
launches (the arrival counters must come back to 0).  The switch is read once per process,
so the combined path runs in a child process."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _cases():
    """(both processes) seeded split-K launches; returns their outputs (CPU)."""
    import conftest  # noqa: F401  (sys.path for the package)
    from a2m import functional as F
    outs = []
    g = torch.Generator().manual_seed(5)
    # tap-chunked conv1d, UNet-like: M = 1024, N = 256, K = 3072 (128-tile split plans)
    x = torch.randn(16, 1024, 16, generator=g).to(DEV)
    w = (torch.randn(1024, 1024, 3, generator=g) / np.sqrt(3072)).to(DEV)
    b = torch.randn(1024, generator=g).to(DEV)
    outs.append(F.conv1d(x, w, b, 1, 1, cache={}))
    # dense 1x1 (linear): M = 256, N = 64, K = 4096 (64-tile split plans)
    x = torch.randn(64, 4096, generator=g).to(DEV)
    w = (torch.randn(256, 4096, generator=g) / 64).to(DEV)
    outs.append(F.linear(x, w, torch.randn(256, generator=g).to(DEV)))
    # BN-eval + LeakyReLU epilogue into an m-contiguous view ([B, T, Co] buffer seen as [B, Co, T])
    B, Ci, Co, T = 4, 2048, 256, 16
    x = torch.randn(B, Ci, T, generator=g).to(DEV)
    w = (torch.randn(Co, Ci, 3, generator=g) / np.sqrt(3 * Ci)).to(DEV)
    bn = tuple(t.to(DEV) for t in (torch.rand(Co, generator=g) + 0.5, torch.randn(Co, generator=g),
                                   torch.randn(Co, generator=g) * 0.1, torch.rand(Co, generator=g) + 0.5)) + (1e-5,)
    buf = torch.zeros(B, T, Co, device=DEV)
    F.conv1d(x, w, None, 1, 1, bn=bn, act=F.ACT_LRELU, slope=0.2, out=buf.permute(0, 2, 1), cache={})
    outs.append(buf)
    # batched launch: two independent [128 x 4096] x [4096 x 96] products
    A = torch.randn(2, 128, 4096, generator=g).to(DEV)
    Bm = torch.randn(2, 96, 4096, generator=g).to(DEV)
    C = torch.empty(2, 128, 96, device=DEV)
    F.gemm(128, 96, 4096, A, 4096, 1, Bm, 4096, 1, C, 96, 1, batch=2, a_bs=128 * 4096,
           b_bs=96 * 4096, c_bs=128 * 96)
    outs.append(C)
    # the first case again (the counters of the first launches must be back at 0)
    torch.cuda.synchronize()
    return [o.cpu() for o in outs]


def test_in_launch_split_combine_bitwise(tmp_path):
    out = str(tmp_path / 'fixup.pt')
    code = ('import sys, torch; sys.path[:0] = %r\n'
            'from test_gpu_gemm_fixup import _cases\n'
            'a = _cases(); b = _cases()\n'
            'assert all(torch.equal(x, y) for x, y in zip(a, b)), "repeat differs"\n'
            'torch.save(a, %r)\n' % ([os.path.dirname(os.path.abspath(__file__))], out))
    env = dict(os.environ, A2M_GEMM_FIXUP='1', A2M_GEMM_FIXUP_KB='100000', A2M_GEMM_LOG='1')
    p = subprocess.run([sys.executable, '-c', code], env=env, capture_output=True, text=True, timeout=180)
    assert p.returncode == 0, p.stderr[-3000:]
    assert '(in-launch)' in p.stderr, 'no launch took the in-launch combine'
    got = torch.load(out, weights_only=True)
    ref = _cases()
    for i, (a, r) in enumerate(zip(got, ref)):
        assert torch.equal(a, r), (i, (a - r).abs().max().item())
