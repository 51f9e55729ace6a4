"""Tap-chunked conv1d (a2m_conv1d_tap_fwd_f32, GEMM loader mode 5) at fp32 and bf16 operand precision.

The tap path is the forward of nn.Conv1d(k, stride=1, padding=(k-1)/2) (model_layers.py:75-120,
the ConvNormRelu / ResBlock convs of the UNet and both decoders) without an im2col matrix: the
B loader stages each channel chunk's x window once and re-stores it shifted per tap.  It must
agree with an fp64 convolution at fp32 accuracy, wrap nothing across clip boundaries, and
match the im2col path it replaces.
"""
import os

import numpy as np
import pytest
import torch

from conftest import golden, rel_err

pytestmark = pytest.mark.gpu
DEV = 'cuda'

# fp32-class accuracy against fp64, relative to max |ref| (measured ~1e-6 at K <= 6144)
TOL32 = 1e-5


def _conv_ref(x, w, b, pad):
    return torch.nn.functional.conv1d(x.double(), w.double(), None if b is None else b.double(),
                                      padding=pad)


@pytest.mark.parametrize('prec', ['fp32', 'bf16'])
@pytest.mark.parametrize('B,Ci,Co,T,k', [(64, 256, 256, 64, 3), (8, 512, 1024, 32, 3),
                                         (5, 1024, 2048, 16, 3), (1, 256, 512, 16, 3),
                                         (3, 64, 96, 8, 5), (2, 32, 20, 4, 3)])
def test_tap_conv1d_matches_fp64(prec, B, Ci, Co, T, k):
    import a2m
    from a2m import functional as F
    g = torch.Generator().manual_seed(B * 7 + Ci + T)
    x = torch.randn(B, Ci, T, generator=g)
    w = torch.randn(Co, Ci, k, generator=g) / np.sqrt(Ci * k)
    b = torch.randn(Co, generator=g)
    pad = (k - 1) // 2
    with a2m.gemm_precision(prec):
        if Ci % a2m._native.lib.a2m_conv1d_tap_chunk():
            pytest.skip('Ci not a multiple of the k-tile at this precision')
        cache = {}
        y = F.conv1d(x.to(DEV), w.to(DEV), b.to(DEV), 1, pad, cache=cache)
        assert 'w' in cache, 'tap path not taken'
    ref = _conv_ref(x, w, b, pad)
    if prec == 'bf16':
        ref = _conv_ref(x.bfloat16().float(), w.bfloat16().float(), b, pad)
    e = rel_err(y.cpu().double(), ref)
    assert e < TOL32, e


_HALO_CASES = [(64, 256, 256, 64), (8, 512, 1024, 32), (5, 1024, 2048, 16), (1, 256, 512, 16),
               (3, 128, 64, 16), (16, 256, 128, 64)]


def _tap_cases():
    """(both processes) the tap-path outputs of _HALO_CASES (the last with the BN + LeakyReLU
    epilogue), on seeded inputs."""
    from a2m import functional as F
    outs = []
    for i, (B, Ci, Co, T) in enumerate(_HALO_CASES):
        g = torch.Generator().manual_seed(100 + i)
        x = torch.randn(B, Ci, T, generator=g).to(DEV)
        w = (torch.randn(Co, Ci, 3, generator=g) / np.sqrt(3 * Ci)).to(DEV)
        b = torch.randn(Co, generator=g).to(DEV)
        kw = {}
        if i == len(_HALO_CASES) - 1:
            kw = dict(bn=tuple(t.to(DEV) for t in (torch.rand(Co, generator=g) + 0.5, torch.randn(Co, generator=g),
                                                   torch.randn(Co, generator=g) * 0.1,
                                                   torch.rand(Co, generator=g) + 0.5)) + (1e-5,),
                      act=F.ACT_LRELU, slope=0.2)
        cache = {}
        outs.append(F.conv1d(x, w, b, 1, 1, cache=cache, **kw).cpu())
        assert 'w' in cache, 'tap path not taken'
    return outs


def test_tap_conv1d_halo_layout_bitwise(tmp_path):
    """The halo B layout (3 taps, pad 1, clips of T >= 16: the window stored once with a zero row
    around every clip, each tap read at a row shift; the default) feeds the MFMAs the same
    operands in the same order as the per-tap re-stored window (A2M_GEMM_HALO=0, computed in a
    child process since the switch is read once): bit-identical outputs, including ragged
    batches (B = 5 clips of 16 leave a partial tile), split-K plans and the BN epilogue."""
    import subprocess
    import sys
    out = str(tmp_path / 'nohalo.pt')
    code = ('import sys, torch; sys.path[:0] = %r\n'
            'import conftest\n'
            'from test_gpu_tapconv import _tap_cases\n'
            'torch.save(_tap_cases(), %r)\n' % ([os.path.dirname(os.path.abspath(__file__))], out))
    p = subprocess.run([sys.executable, '-c', code], env=dict(os.environ, A2M_GEMM_HALO='0'),
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-3000:]
    ref = torch.load(out, weights_only=True)
    got = _tap_cases()
    for case, a, r in zip(_HALO_CASES, got, ref):
        assert torch.equal(a, r), (case, (a - r).abs().max().item())


def test_tap_conv1d_epilogue_views_and_cache():
    """BN-eval + LeakyReLU epilogue, x a channel slice of a concat buffer, out a strided view;
    the packed weights are rebuilt when the weight changes in place."""
    from a2m import functional as F
    g = torch.Generator().manual_seed(3)
    B, Ci, Co, T = 16, 256, 128, 64
    cat = torch.randn(B, 2 * Ci, T, generator=g).to(DEV)
    x = cat[:, Ci:]
    w = (torch.randn(Co, Ci, 3, generator=g) * 0.05).to(DEV)
    bias = torch.randn(Co, generator=g).to(DEV)
    bn = tuple(t.to(DEV) for t in (torch.rand(Co) + 0.5, torch.randn(Co), torch.randn(Co) * 0.1,
                                   torch.rand(Co) + 0.5)) + (1e-5,)
    outbuf = torch.zeros(B, T, 2 * Co, device=DEV)
    out = outbuf[:, :, Co:].permute(0, 2, 1)
    cache = {}
    F.conv1d(x, w, bias, 1, 1, bn=bn, act=F.ACT_LRELU, slope=0.2, out=out, cache=cache)
    ref = F.conv1d(x, w, bias, 1, 1, bn=bn, act=F.ACT_LRELU, slope=0.2)   # im2col path
    assert rel_err(out.cpu(), ref.cpu()) < 1e-6
    assert outbuf[:, :, :Co].abs().max().item() == 0.0
    with torch.no_grad():
        w.mul_(-1.0)
    F.conv1d(x, w, bias, 1, 1, bn=bn, act=F.ACT_LRELU, slope=0.2, out=out, cache=cache)
    ref = F.conv1d(x, w, bias, 1, 1, bn=bn, act=F.ACT_LRELU, slope=0.2)
    assert rel_err(out.cpu(), ref.cpu()) < 1e-6


def test_tap_conv1d_rejects_ineligible():
    """T that does not tile the 64-row GEMM tile (the long-form 480-frame clips) or a chunk
    packed for another precision is refused by the C-ABI (the Python layer then takes the
    im2col path)."""
    import a2m
    from a2m import _native as N
    from a2m import functional as F
    x = torch.randn(2, 64, 480, device=DEV)
    w = torch.randn(64, 64, 3, device=DEV)
    cache = {}
    y = F.conv1d(x, w, None, 1, 1, cache=cache)
    assert 'w' not in cache
    assert rel_err(y.cpu().double(), _conv_ref(x.cpu(), w.cpu(), None, 1)) < TOL32
    x = torch.randn(2, 64, 64, device=DEV)
    packed, chunk = F.conv1d_tap_packed(w)
    with a2m.gemm_precision('bf16'):
        rc = N.lib.a2m_conv1d_tap_fwd_f32(x.data_ptr(), 64 * 64, 64, 2, 64, 64, packed.data_ptr(),
                                          chunk, None, 64, 3, 1, None, None, None, None, 1e-5, 0,
                                          0.2, y.data_ptr(), 64 * 64, 64, 1, None, 0, None)
    assert rc == N.A2M_EINVAL and 'chunk' in N.last_error()


@pytest.mark.parametrize('B,Ci,Co,H,W,k,s,p,cols', [
    (4, 1, 64, 64, 128, (4, 4), 2, (1, 1), (9, 55)),      # encoder conv0 (mel, Ci = 1)
    (3, 64, 128, 32, 64, (4, 4), 2, (1, 1), (5, 27)),     # conv1
    (2, 128, 256, 16, 32, (4, 4), 2, (1, 1), (3, 13)),    # conv2
    (3, 32, 64, 10, 14, (3, 3), 1, (1, 1), (2, 11)),      # Ci = one k-tile
    (2, 256, 512, 8, 16, (3, 3), 1, (1, 1), (4, 12)),     # conv3
    (2, 512, 256, 8, 8, (3, 8), 1, (1, 0), (0, 1)),       # conv4 (3 x 8 kernel, W_out = 1)
    (2, 12, 20, 9, 11, (3, 3), 2, (1, 1), None)])
@pytest.mark.parametrize('out_nhwc', [True, False])
def test_conv2d_nhwc_matches_fp64(B, Ci, Co, H, W, k, s, p, cols, out_nhwc):
    """Channels-last conv2d (a2m_conv2d_nhwc_fwd_f32) against an fp64 convolution, on the
    computed column range: Ci = 1 (conv0) through the direct kernel; Ci a multiple of the k-tile
    through loader mode 6 (per-tap channel runs); other Ci through mode 4 (unit-stride runs of
    kw*Ci floats)."""
    from a2m import functional as F
    g = torch.Generator().manual_seed(B + Ci + Co + H)
    x = torch.randn(B, Ci, H, W, generator=g)
    w = torch.randn(Co, Ci, *k, generator=g) / np.sqrt(Ci * k[0] * k[1])
    b = torch.randn(Co, generator=g)
    ref = torch.nn.functional.conv2d(x.double(), w.double(), b.double(), stride=s, padding=p)
    lo, hi = cols if cols is not None else (0, ref.shape[-1])
    xn = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    y = F.conv2d_nhwc(xn, w.to(DEV), b.to(DEV), s, p, cols=cols, out_nhwc=out_nhwc, cache={})
    y = (y.permute(0, 3, 1, 2) if out_nhwc else y).cpu().double()
    e = rel_err(y[..., lo:hi], ref[..., lo:hi])
    assert e < TOL32, e


def _bn_ref(y, bn, act, slope=0.2):
    w, b_, rm, rv, eps = bn
    sh = (1, -1, 1, 1)
    z = (y - rm.double().view(sh)) / torch.sqrt(rv.double().view(sh) + eps) * w.double().view(sh) + b_.double().view(sh)
    return torch.where(z > 0, z, slope * z) if act else z


def test_conv2d_nhwc_unaligned_input_takes_run_loader():
    """An input that is 4- but not 16-byte aligned (a view one float into a buffer) with Ci a
    multiple of the k-tile: the float4 channel-run loader (mode 6) needs 16-byte alignment, so
    the conv takes the k-run loader (mode 4) and still matches fp64."""
    from a2m import functional as F
    g = torch.Generator().manual_seed(7)
    B, Ci, Co, H, W = 2, 64, 128, 16, 20
    x = torch.randn(B, Ci, H, W, generator=g)
    w = torch.randn(Co, Ci, 4, 4, generator=g) / np.sqrt(Ci * 16)
    b = torch.randn(Co, generator=g)
    ref = torch.nn.functional.conv2d(x.double(), w.double(), b.double(), stride=2, padding=1)
    xn = x.permute(0, 2, 3, 1).contiguous()
    buf = torch.empty(xn.numel() + 1, device=DEV)
    xv = buf[1:].view(xn.shape)
    xv.copy_(xn.to(DEV))
    assert xv.data_ptr() % 16 == 4
    y = F.conv2d_nhwc(xv, w.to(DEV), b.to(DEV), 2, (1, 1), cache={})
    assert rel_err(y.permute(0, 3, 1, 2).cpu().double(), ref) < TOL32


@pytest.mark.parametrize('Co,stride,act,mfma', [(64, 1, True, 1), (1024, 2, True, 1), (64, 2, False, 0),
                                                (1024, 1, True, 0), (96, 2, True, 1)])
def test_conv2d_c1_bn_act_stride(Co, stride, act, mfma):
    """The encoder's Ci = 1 first conv (4 x 4) in its direct kernels -- the MFMA one
    (conv2d_c1_mfma_kernel, default for channels-last outputs) and, with A2M_C1_MFMA=0, the VALU
    one -- at stride 1 and 2, with the BatchNorm-eval affine and LeakyReLU epilogue, and at
    Co = 1024, against fp64."""
    import subprocess
    import sys
    import json
    env = dict(os.environ, A2M_C1_MFMA=str(mfma))
    code = (
        'import sys, json, torch, numpy as np; sys.path[:0] = %r\n'
        'from test_gpu_tapconv import _c1_case\n'
        'print(json.dumps(_c1_case(%d, %d, %r)))\n' % ([os.path.dirname(os.path.abspath(__file__))], Co, stride, act))
    p = subprocess.run([sys.executable, '-c', code], env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-3000:]
    e = json.loads(p.stdout.strip().splitlines()[-1])
    assert e < TOL32, e


def _c1_case(Co, stride, act):
    """(child process: A2M_C1_MFMA is read once per process) conv0-shaped conv vs fp64."""
    import conftest  # noqa: F401  (sys.path for the package)
    from a2m import functional as F
    g = torch.Generator().manual_seed(Co + stride)
    B, H, W = 3, 64, 128
    x = torch.randn(B, 1, H, W, generator=g) * 2 - 3
    w = torch.randn(Co, 1, 4, 4, generator=g) / 4
    b = torch.randn(Co, generator=g)
    bn = (torch.rand(Co, generator=g) + 0.5, torch.randn(Co, generator=g), torch.randn(Co, generator=g) * 0.1,
          torch.rand(Co, generator=g) + 0.5, 1e-5)
    ref = torch.nn.functional.conv2d(x.double(), w.double(), b.double(), stride=stride, padding=1)
    ref = _bn_ref(ref, bn, act)
    y = F.conv2d_nhwc(x.permute(0, 2, 3, 1).contiguous().to(DEV), w.to(DEV), b.to(DEV), stride, (1, 1),
                      bn=tuple(t.to(DEV) for t in bn[:4]) + (bn[4],), act=F.ACT_LRELU if act else F.ACT_NONE,
                      cache={})
    return rel_err(y.permute(0, 3, 1, 2).cpu().double(), ref)


@pytest.mark.parametrize('B,T,split', [(64, 64, 0), (3, 64, 1), (2, 480, 0), (1, 33, 0), (5, 100, 3)])
def test_conv2d_nhwc_interp_equals_conv_then_interp(B, T, split):
    """The encoder's last conv with its time resample fused into the GEMM reduce
    (a2m_conv2d_nhwc_interp_fwd_f32) equals conv2d_nhwc (the live column, NCHW) followed by
    interp_time bit for bit -- at the bench shape, long-form H = 60 (configs[3]), odd T, and
    with the planner forced to one split (the tile writes a raw slab) or three."""
    from a2m import functional as F
    from a2m import _native as N
    g = torch.Generator().manual_seed(B * 1000 + T)
    H = T // 8
    x = torch.randn(B, H, 16, 512, generator=g).to(DEV)   # conv3's NHWC output [B, H, 16, 512]
    w = (torch.randn(256, 512, 3, 8, generator=g) / np.sqrt(512 * 24)).to(DEV)
    b = torch.randn(256, generator=g).to(DEV)
    bn = tuple(t.to(DEV) for t in (torch.rand(256, generator=g) + 0.5, torch.randn(256, generator=g),
                                     torch.randn(256, generator=g) * 0.1, torch.rand(256, generator=g) + 0.5)) + (1e-5,)
    cache = {}
    N.check(N.lib.a2m_gemm_plan_override(64 if split else 0, split))
    try:
        y = F.conv2d_nhwc(x, w, b, 1, (1, 3), bn=bn, act=F.ACT_LRELU, cols=(7, 8), out_nhwc=False, cache=cache)
        ref = F.interp_time(y, T)
        fused = F.conv2d_nhwc_interp(x, w, b, 1, (1, 3), T, 7, bn=bn, act=F.ACT_LRELU, cache=cache)
    finally:
        N.check(N.lib.a2m_gemm_plan_override(0, 0))
    torch.cuda.synchronize()
    assert fused.shape == (B, 256, T)
    assert torch.equal(fused, ref), (fused - ref).abs().max().item()


def test_conv2d_nhwc_interp_rejects_non_live_column():
    """A column the resample does not read with weight 1 is refused (A2M_EINVAL), not computed."""
    from a2m import functional as F
    x = torch.randn(1, 8, 16, 512, device=DEV)
    w = torch.randn(256, 512, 3, 8, device=DEV)
    with pytest.raises(Exception, match='live column'):
        F.conv2d_nhwc_interp(x, w, None, 1, (1, 3), 64, 6, cache={})


def test_encoder_eval_fused_interp_matches_golden_chain():
    """AudioEncoder eval through the fused last layer equals the unfused chain bit for bit."""
    import a2m.model_layers as ML
    from a2m.real_motion_model import SelfAttention_G
    torch.manual_seed(0)
    enc = SelfAttention_G(p=0.0).to(DEV).eval().audio_encoder
    x = torch.randn(4, 64, 128, device=DEV)
    with torch.no_grad():
        fused = enc(x)
        ML._ENC_FUSED_INTERP = False
        try:
            ref = enc(x)
        finally:
            ML._ENC_FUSED_INTERP = True
    assert torch.equal(fused, ref), (fused - ref).abs().max().item()
