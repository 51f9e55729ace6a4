"""Grouped decoder launches: the body and hand decoders' same-shape layers as one launch each
(a2m_conv1d_tap_group_fwd_f32, a2m_self_attention_eval_group_f32; real_motion_model.py
SelfAttention_G._decoders_grouped).  Each grouped op is held to the single-problem op it
replaces on the same inputs, including shared inputs (group stride 0) and problems laid out in
reverse / separate allocations (negative or arbitrary group strides); the generator's eval
forward with grouping on is held to the ungrouped forward and to the reference's pose
(tests/golden g_eval fixtures, via test_gpu_eval)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _rel(a, b):
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def _bn(C, g):
    return (torch.rand(C, device=DEV, generator=g) + 0.5, torch.randn(C, device=DEV, generator=g) * 0.1,
            torch.randn(C, device=DEV, generator=g) * 0.1, torch.rand(C, device=DEV, generator=g) + 0.5, 1e-5)


@pytest.mark.parametrize('layout', ['separate', 'shared_x', 'reversed_out'])
@pytest.mark.parametrize('B,C,T', [(64, 256, 64), (3, 256, 32), (1, 128, 16)])
def test_conv1d_tap_group(layout, B, C, T):
    from a2m import functional as F
    g = torch.Generator(device=DEV).manual_seed(7)
    ws = [torch.randn(C, C, 3, device=DEV, generator=g) * 0.05 for _ in range(2)]
    bs = [torch.randn(C, device=DEV, generator=g) * 0.1 for _ in range(2)]
    bns = [_bn(C, g) for _ in range(2)]
    x0 = torch.randn(B, C, T, device=DEV, generator=g)
    xs = [x0, x0] if layout == 'shared_x' else [x0, torch.randn(B, C, T, device=DEV, generator=g)]
    caches = [{}, {}]
    ref = [F.conv1d(xs[i], ws[i], bs[i], 1, 1, bn=bns[i], act=F.ACT_LRELU, cache=caches[i]) for i in range(2)]
    packed = torch.stack([F.conv1d_tap_packed(ws[i], caches[i])[0] for i in range(2)])
    chunk = F.N.lib.a2m_conv1d_tap_chunk()
    st = lambda k: torch.stack([bns[i][k] for i in range(2)])
    bn = (st(0), st(1), st(2), st(3), 1e-5)
    buf = torch.full((2, B, C, T), float('nan'), device=DEV)
    outs = [buf[1], buf[0]] if layout == 'reversed_out' else [buf[0], buf[1]]
    F.conv1d_tap_group(xs, packed, chunk, torch.stack(bs), C, 3, 1, bn, F.ACT_LRELU, 0.2, outs)
    torch.cuda.synchronize()
    for i in range(2):
        assert not torch.isnan(outs[i]).any()
        # the grouped launch may plan a different split-K (fp32 sums reassociated over K = 3C)
        assert _rel(outs[i], ref[i]) < 1e-5, (i, _rel(outs[i], ref[i]))


@pytest.mark.parametrize('B,C,T', [(64, 256, 64), (5, 128, 32)])
@pytest.mark.parametrize('with_res', [False, True])
def test_self_attention_group(B, C, T, with_res):
    from a2m import functional as F
    g = torch.Generator(device=DEV).manual_seed(11)
    W = []
    for i in range(2):
        W.append([torch.randn(C // 8, C, device=DEV, generator=g) * 0.05, torch.randn(C // 8, device=DEV, generator=g) * 0.1,
                  torch.randn(C // 8, C, device=DEV, generator=g) * 0.05, torch.randn(C // 8, device=DEV, generator=g) * 0.1,
                  torch.randn(C, C, device=DEV, generator=g) * 0.05, torch.randn(C, device=DEV, generator=g) * 0.1,
                  torch.tensor([0.3 + 0.4 * i], device=DEV)])
    # problem 0's x in its own allocation, problem 1's inside a larger buffer: arbitrary stride
    x0 = torch.randn(B, C, T, device=DEV, generator=g)
    big = torch.randn(3, B, C, T, device=DEV, generator=g)
    xs = [x0, big[2]]
    res = [torch.randn(B, C, T, device=DEV, generator=g) for _ in range(2)] if with_res else None
    ref = [F.self_attention(xs[i], *W[i], res=res[i] if res else None) for i in range(2)]
    qkv = [F.stacked_qkv(*W[i][:6]) for i in range(2)]
    out = torch.full((2, B, C, T), float('nan'), device=DEV)
    F.self_attention_group(xs, torch.stack([q[0] for q in qkv]), torch.stack([q[1] for q in qkv]),
                           torch.cat([W[i][6] for i in range(2)]), list(out), res=res)
    torch.cuda.synchronize()
    for i in range(2):
        assert _rel(out[i], ref[i]) < 1e-6, (i, _rel(out[i], ref[i]))


@pytest.mark.parametrize('mode', [1, 2])
@pytest.mark.parametrize('B,T', [(64, 64), (2, 32)])
def test_generator_grouped_vs_branches(B, T, mode, monkeypatch):
    from a2m import real_motion_model as R
    torch.manual_seed(3)
    g = R.SelfAttention_G(time_steps=T).to(DEV).eval()
    # non-trivial gammas / BN statistics so every grouped layer contributes
    with torch.no_grad():
        for m in g.modules():
            if isinstance(m, torch.nn.BatchNorm1d):
                m.running_mean.normal_(0, 0.1)
                m.running_var.uniform_(0.5, 1.5)
            if hasattr(m, 'gamma') and isinstance(m.gamma, torch.nn.Parameter):
                m.gamma.fill_(0.5)
    audio = torch.randn(B, T, 128, device=DEV)
    with torch.no_grad():
        feats = g.unet(g.audio_encoder(audio))
        monkeypatch.setattr(R, '_GROUPED', mode)
        assert g._groupable(feats)
        y1, l1 = g(audio)
        monkeypatch.setattr(R, '_GROUPED', 0)
        y0, l0 = g(audio)
    torch.cuda.synchronize()
    assert _rel(y1, y0) < 1e-5, _rel(y1, y0)
    assert abs(l1[-1].item() - l0[-1].item()) <= 1e-5 * max(1.0, abs(l0[-1].item()))
