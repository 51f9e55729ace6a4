"""The software-pipelined 64x64 tiles -- gemm_pipe.h (fp32) and gemm_pipe_bf16.h (bf16 operands)
-- against gemm_tile, the engine's reference tile, on every operand mode they take: dense rows
(mode 0), row-contiguous [K][N] operands (mode 3), the tap-chunked conv1d (mode 5, three taps)
and ConvTranspose phases (mode 5, two taps with a shift), channels-last conv rows (mode 6), the
1-D conv weight gradients (mode-4 runs on both sides, x as stride-2 runs for stride-2 convs), plain
[K][M] A operands; ragged M / N / K, one and several split-K slabs, float4 and scalar epilogues.

Both tiles compute the same products in the same order, so the results are bitwise equal, except
fp32 dense rows, whose gemm_tile path is the two-wave-group tile (KS = 2: the k halves summed in a
different order, fp32 rounding apart).  a2m_gemm_pipe_override switches the tile per call.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


@pytest.fixture
def eng():
    import a2m
    from a2m import _native as N
    yield a2m, N
    N.check(N.lib.a2m_gemm_pipe_override(-1))
    N.check(N.lib.a2m_gemm_plan_override(0, 0))
    a2m.set_gemm_precision('fp32')


def _rand(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(DEV)


def _rel(a, ref):
    return ((a.double() - ref).abs().max() / ref.abs().max()).item()


def _case_gemm(M, N, K):
    A, B = _rand(M, K, seed=1), _rand(N, K, seed=2)
    C = torch.empty(M, N, device=DEV)

    def run():
        from a2m import functional as F
        return F.gemm(M, N, K, A, K, 1, B, K, 1, C, N, 1)
    return run, A.double() @ B.double().t(), True


def _case_gemm_kr(M, N, K):
    A, Bt = _rand(M, K, seed=3), _rand(K, N, seed=4)
    C = torch.empty(M, N, device=DEV)

    def run():
        from a2m import functional as F
        return F.gemm(M, N, K, A, K, 1, Bt, 1, N, C, N, 1)
    return run, A.double() @ Bt.double(), False


def _case_gemm_at(M, N, K, b_rows):
    """A as a plain [K][M] operand (mode 3), B dense [N][K] rows or [K][N] (mode 3): the weight
    gradients of the linears and graph layers."""
    At = _rand(K, M, seed=16)
    B = _rand(N, K, seed=17) if b_rows else _rand(K, N, seed=18)
    C = torch.empty(M, N, device=DEV)

    def run():
        from a2m import functional as F
        return F.gemm(M, N, K, At, 1, M, B, K if b_rows else 1, 1 if b_rows else N, C, N, 1)
    ref = At.double().t() @ (B.double().t() if b_rows else B.double())
    return run, ref, False


def _case_conv1d(B, Ci, Co, T):
    x = _rand(B, Ci, T, seed=5)
    w = _rand(Co, Ci, 3, seed=6, scale=(3 * Ci) ** -0.5)
    b = _rand(Co, seed=7)
    y = torch.empty(B, Co, T, device=DEV)
    cache = {}

    def run():
        from a2m import functional as F
        return F.conv1d(x, w, b, 1, 1, act=F.ACT_LRELU, out=y, cache=cache)
    ref = torch.nn.functional.leaky_relu(
        torch.nn.functional.conv1d(x.double(), w.double(), b.double(), padding=1), 0.2)
    return run, ref, False


def _case_convt(B, Ci, Co, Tin):
    x = _rand(B, Ci, Tin, seed=8)
    w = _rand(Ci, Co, 4, seed=9, scale=(2 * Ci) ** -0.5)
    b = _rand(Co, seed=10)
    cache = {}

    def run():
        from a2m import functional as F
        return F.convt1d(x, w, b, stride=2, pad=1, out_pad=0, cache=cache)
    ref = torch.nn.functional.conv_transpose1d(x.double(), w.double(), b.double(), stride=2, padding=1)
    return run, ref, False


def _case_nhwc(B, Ci, Co, H, W):
    x = _rand(B, H, W, Ci, seed=11)
    w = _rand(Co, Ci, 3, 3, seed=12, scale=(9 * Ci) ** -0.5)
    b = _rand(Co, seed=13)
    cache = {}

    def run():
        from a2m import functional as F
        return F.conv2d_nhwc(x, w, b, 2, (1, 1), cache=cache)
    ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).double(), w.double(), b.double(), stride=2,
                                     padding=(1, 1)).permute(0, 2, 3, 1)
    return run, ref, False


def _case_wgrad1d(B, Ci, Co, T, k, pad, stride=1):
    Tout = (T + 2 * pad - k) // stride + 1
    x = _rand(B, Ci, T, seed=14)
    dy = _rand(B, Co, Tout, seed=15)

    def run():
        from a2m import functional as F
        return F.conv_wgrad(dy, x, (Co, Ci, k), stride, pad)
    ref = torch.nn.grad.conv1d_weight(x.double(), (Co, Ci, k), dy.double(), stride=stride, padding=pad)
    return run, ref, False


CASES = {
    'gemm_200x1000x768': lambda: _case_gemm(200, 1000, 768),
    'gemm_130x998x320': lambda: _case_gemm(130, 998, 320),      # scalar epilogue (N % 4 != 0)
    'gemm_kr_130x4096x300': lambda: _case_gemm_kr(130, 4096, 300),
    'gemm_kr_64x512x2688': lambda: _case_gemm_kr(64, 512, 2688),
    'conv1d_b16_128to192_t64': lambda: _case_conv1d(16, 128, 192, 64),
    'conv1d_b8_256to128_t16': lambda: _case_conv1d(8, 256, 128, 16),
    'convt_b8_128to64_t32': lambda: _case_convt(8, 128, 64, 32),
    'nhwc_b4_64to96_20x22': lambda: _case_nhwc(4, 64, 96, 20, 22),
    # A in mode 3 (plain [K][M]) with dense or mode-3 B
    'gemm_at_128x1000x700_rows': lambda: _case_gemm_at(128, 1000, 700, True),
    'gemm_at_64x64x20000_kr': lambda: _case_gemm_at(64, 64, 20000, False),
    'gemm_at_256x2688x512_kr': lambda: _case_gemm_at(256, 2688, 512, False),
    # mode 4 on both operands (the 1-D conv weight gradients): padding taps cross the run edges
    'wgrad_b8_48to80_t64_k3': lambda: _case_wgrad1d(8, 48, 80, 64, 3, 1),
    'wgrad_b6_130to70_t32_k3': lambda: _case_wgrad1d(6, 130, 70, 32, 3, 1),
    'wgrad_b4_64to64_t96_k1': lambda: _case_wgrad1d(4, 64, 64, 96, 1, 0),
    'wgrad_b4_32to40_t64_k5': lambda: _case_wgrad1d(4, 32, 40, 64, 5, 2),
    # runs shorter than the k-tile (a tile spans several clips' runs)
    'wgrad_b16_64to48_t16_k3': lambda: _case_wgrad1d(16, 64, 48, 16, 3, 1),
    'wgrad_b24_32to36_t4_k3': lambda: _case_wgrad1d(24, 32, 36, 4, 3, 1),
    'wgrad_b10_40to40_t20_k3': lambda: _case_wgrad1d(10, 40, 40, 20, 3, 1),
    # stride-2 convs: x read as stride-2 runs (gemm_tile gathers them, mode 1)
    'wgrad_s2_b8_48to64_t64_k4': lambda: _case_wgrad1d(8, 48, 64, 64, 4, 1, 2),
    'wgrad_s2_b12_40to36_t32_k3': lambda: _case_wgrad1d(12, 40, 36, 32, 3, 1, 2),
    'wgrad_s2_b16_64to64_t16_k4': lambda: _case_wgrad1d(16, 64, 64, 16, 4, 1, 2),
}


@pytest.mark.parametrize('prec', ['fp32', 'bf16'])
@pytest.mark.parametrize('split', [0, 3])
@pytest.mark.parametrize('case', sorted(CASES))
def test_pipe_tile_matches_gemm_tile(eng, prec, split, case):
    a2m, N = eng
    a2m.set_gemm_precision(prec)
    N.check(N.lib.a2m_gemm_plan_override(64, split))
    run, ref, dense_rows = CASES[case]()
    outs = []
    for mode in (1, 0):
        N.check(N.lib.a2m_gemm_pipe_override(mode))
        outs.append(run().clone())
    torch.cuda.synchronize()
    pipe, tile = outs
    tol = 1e-4 if prec == 'fp32' else 2e-2
    assert _rel(pipe, ref) < tol and _rel(tile, ref) < tol
    if prec == 'fp32' and dense_rows:
        assert _rel(pipe, tile.double()) < 1e-5
    else:
        assert torch.equal(pipe, tile), f'{case} {prec} split {split}: max diff {(pipe - tile).abs().max().item()}'
