"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle / reference goldens.

Tolerance: north_star's 1e-4 relative fp32, measured as max|gpu - ref| / max|ref| per tensor.
Per-op tests compare with a plain PyTorch fp32 CPU computation of the same op.
"""
import numpy as np
import pytest
import torch

from conftest import golden, rel_err

pytestmark = pytest.mark.gpu
TOL = 1e-4
DEV = 'cuda'


def _rand(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).float()


# ------------------------------------------------------------------------------ log-mel
def test_logmel_build_config_vs_reference():
    from a2m.mel_features import log_mel_batch
    z = golden('mel.npz')
    wav = torch.from_numpy(z['mel_build_wave']).to(DEV)
    out = log_mel_batch(wav).cpu().numpy()
    assert out.shape == (2, 64, 128)
    assert rel_err(out, z['mel_build_out']) < TOL


def test_logmel_batch_vs_oracle_full_frames():
    """Register-FFT kernel (fft_len 2048) over a batch of 16 synthetic clips, 64 and 70 frames,
    including a strided clip view (clip_stride != n_samples), vs the float64 numpy oracle."""
    from a2m.mel_features import log_mel_batch
    from oracle import mel as omel, synth
    for frames, seed in ((64, 11), (70, 12)):
        n = synth.samples_for_frames(frames)
        wav = synth.speech_like(16, n + 37, seed=seed)
        dev = torch.from_numpy(wav).to(DEV)[:, 5:5 + n]  # strided rows, odd start offset
        out = log_mel_batch(dev).cpu().numpy()
        for c in (0, 7, 15):
            ref = omel.log_mel(wav[c, 5:5 + n], **omel.BUILD_CFG)
            assert out.shape[1:] == ref.shape
            assert rel_err(out[c], ref) < TOL, (frames, c)
    # window 2000 < fft_len 2048 (zero-padded frames: the kernel's table-window variant)
    cfg = dict(omel.BUILD_CFG, window_secs=0.125)
    wav = synth.speech_like(3, 40000, seed=13)
    out = log_mel_batch(torch.from_numpy(wav).to(DEV), window_length_secs=0.125).cpu().numpy()
    for c in range(3):
        assert rel_err(out[c], omel.log_mel(wav[c], **cfg)) < TOL


def test_logmel_reference_signature_and_edges():
    from a2m.mel_features import log_mel_spectrogram
    z = golden('mel.npz')
    out = log_mel_spectrogram(z['mel_repr_wave'], audio_sample_rate=16000, log_offset=0.01,
                              window_length_secs=0.025, hop_length_secs=0.010, num_mel_bins=64,
                              lower_edge_hertz=125, upper_edge_hertz=7500)
    assert out.shape == z['mel_repr_out'].shape and rel_err(out, z['mel_repr_out']) < TOL
    # reference defaults: 8 kHz, 20 mels, log_offset 0 (fft 256 -> radix-2 + radix-4 stages)
    out = log_mel_spectrogram(z['mel_default_wave'])
    assert rel_err(out, z['mel_default_out']) < TOL
    build = dict(audio_sample_rate=16000, log_offset=0.01, window_length_secs=0.128,
                 hop_length_secs=1 / 15, num_mel_bins=128, lower_edge_hertz=125.0, upper_edge_hertz=7500.0)
    assert rel_err(log_mel_spectrogram(z['mel_oneframe_wave'], **build), z['mel_oneframe_out']) < TOL
    assert log_mel_spectrogram(z['mel_oneframe_wave'][:2047], **build).shape == (0, 128)
    with pytest.raises(ValueError, match='Nyquist'):
        log_mel_spectrogram(z['mel_oneframe_wave'], **{**build, 'upper_edge_hertz': 9000.0})


def test_logmel_half_even_rates_vs_reference():
    """44.1 kHz and 22.05 kHz, where int(round(sr * secs)) lands on .5 (window 1102.5 -> 1102,
    hop 220.5 -> 220, mel_features.py:212-213): frame count and values against the
    reference's own outputs (tests/golden/mel_rates.npz)."""
    from a2m.mel_features import log_mel_spectrogram
    z = golden('mel_rates.npz')
    for i, (sr, ws, hs, nm, lo, hi) in enumerate(z['cases']):
        ref = z[f'out{i}']
        out = log_mel_spectrogram(z[f'wave{i}'], audio_sample_rate=int(sr), log_offset=0.01,
                                  window_length_secs=ws, hop_length_secs=hs, num_mel_bins=int(nm),
                                  lower_edge_hertz=lo, upper_edge_hertz=hi)
        assert out.shape == ref.shape, (i, out.shape, ref.shape)
        assert rel_err(out, ref) < TOL, (i, rel_err(out, ref))


# ------------------------------------------------------------------------------ per op
@pytest.mark.parametrize('B,Ci,Co,T,k,s,p', [(3, 16, 24, 20, 3, 1, 1), (2, 32, 64, 17, 4, 2, 1),
                                             (4, 40, 8, 9, 1, 1, 0), (2, 256, 512, 64, 3, 1, 1),
                                             (2, 104, 64, 63, 4, 2, 1), (1, 7, 130, 5, 3, 1, 1)])
def test_conv1d_bn_act(B, Ci, Co, T, k, s, p):
    from a2m import functional as F
    x, w, b = _rand(B, Ci, T, seed=1), _rand(Co, Ci, k, seed=2, scale=0.3), _rand(Co, seed=3)
    bw, bb, rm, rv = _rand(Co, seed=4).abs() + 0.5, _rand(Co, seed=5), _rand(Co, seed=6), _rand(Co, seed=7).abs() + 0.5
    ref = torch.nn.functional.conv1d(x, w, b, stride=s, padding=p)
    ref = torch.nn.functional.batch_norm(ref, rm, rv, bw, bb, False, 0.0, 1e-5)
    ref = torch.nn.functional.leaky_relu(ref, 0.2)
    d = [t.to(DEV) for t in (x, w, b, bw, bb, rm, rv)]
    out = F.conv1d(d[0], d[1], d[2], s, p, bn=(d[3], d[4], d[5], d[6], 1e-5), act=F.ACT_LRELU)
    assert rel_err(out.cpu(), ref) < TOL


def test_conv1d_strided_views_and_linear():
    from a2m import functional as F
    x = _rand(3, 50, 12, seed=8)
    w, b = _rand(30, 20, 3, seed=9, scale=0.2), _rand(30, seed=10)
    big = torch.zeros(3, 90, 12)
    ref = torch.nn.functional.conv1d(x[:, 10:30], w, b, padding=1)
    xd, bd = x.to(DEV), big.to(DEV)
    F.conv1d(xd[:, 10:30], w.to(DEV), b.to(DEV), 1, 1, out=bd[:, 40:70])
    assert rel_err(bd[:, 40:70].cpu(), ref) < TOL and bd[:, :40].abs().max() == 0
    xl, wl, bl = _rand(37, 640, seed=11), _rand(256, 640, seed=12, scale=0.05), _rand(256, seed=13)
    out = F.linear(xl.to(DEV), wl.to(DEV), bl.to(DEV))
    assert rel_err(out.cpu(), torch.nn.functional.linear(xl, wl, bl)) < TOL
    # [B, C, T] -> [B, T, O] (proj_in layout) and transposed input (D's first conv)
    xt = _rand(2, 63, 104, seed=14)
    w1 = _rand(64, 104, 4, seed=15, scale=0.1)
    ref = torch.nn.functional.conv1d(xt.transpose(1, 2), w1, None, stride=2, padding=1)
    out = F.conv1d(xt.to(DEV).transpose(1, 2), w1.to(DEV), None, 2, 1)
    assert rel_err(out.cpu(), ref) < TOL


@pytest.mark.parametrize('B,Ci,Co,T', [(2, 64, 32, 8), (3, 2048, 1024, 16), (2, 1024, 512, 32),
                                        (2, 40, 24, 7)])
def test_convt1d_bn_relu(B, Ci, Co, T):
    from a2m import functional as F
    x, w, b = _rand(B, Ci, T, seed=20), _rand(Ci, Co, 3, seed=21, scale=0.1), _rand(Co, seed=22)
    bw, bb, rm, rv = _rand(Co, seed=23).abs() + .5, _rand(Co, seed=24), _rand(Co, seed=25), _rand(Co, seed=26).abs() + .5
    ref = torch.nn.functional.conv_transpose1d(x, w, b, stride=2, padding=1, output_padding=1)
    ref = torch.relu(torch.nn.functional.batch_norm(ref, rm, rv, bw, bb, False, 0.0, 1e-5))
    d = [t.to(DEV) for t in (x, w, b, bw, bb, rm, rv)]
    out = F.convt1d(d[0], d[1], d[2], bn=(d[3], d[4], d[5], d[6], 1e-5), act=F.ACT_RELU)
    assert out.shape == ref.shape and rel_err(out.cpu(), ref) < TOL


@pytest.mark.parametrize('ks,stride,pad,op,T', [(3, 2, 1, 1, 16), (4, 2, 1, 0, 8), (5, 2, 2, 1, 32),
                                                (3, 1, 1, 0, 16), (6, 4, 1, 0, 4), (2, 2, 0, 0, 64)])
def test_convt1d_tap_path(ks, stride, pad, op, T):
    """The tap-chunked ConvTranspose1d (a2m_convt1d_tap_fwd_f32, loader mode 5 per output
    phase) against torch and against the gathered per-phase path on the same inputs."""
    from a2m import functional as F
    from a2m import _native as NN
    B, Ci, Co = 3, 96, 40
    x, w, b = _rand(B, Ci, T, seed=27), _rand(Ci, Co, ks, seed=28, scale=0.1), _rand(Co, seed=29)
    ref = torch.nn.functional.conv_transpose1d(x, w, b, stride=stride, padding=pad, output_padding=op)
    xd, wd, bd = x.to(DEV), w.to(DEV), b.to(DEV)
    assert F._convt_tap_eligible(xd, stride, ref.shape[2])
    out = F.convt1d(xd, wd, bd, stride, pad, op)
    assert out.shape == ref.shape and rel_err(out.cpu(), ref) < TOL
    Tout = ref.shape[2]
    packed = F.convt_packed(wd, stride, pad)
    gathered = torch.empty(B, Co, Tout, device=DEV)
    F._with_ws(xd.device, lambda wp, wn: NN.lib.a2m_convt1d_packed_fwd_f32(
        F._p(xd), xd.stride(0), xd.stride(1), B, Ci, T, F._p(packed), F._p(bd), Co, ks, stride, pad, op,
        *F._bn_args(None), F.ACT_NONE, 0.2, F._p(gathered), gathered.stride(0), gathered.stride(1), wp, wn,
        F._stream()))
    assert rel_err(out.cpu(), gathered.cpu()) < TOL


@pytest.mark.parametrize('Ci,Co,k,stride,pad,H,W,cols', [
    (128, 128, (4, 4), 2, (1, 1), 16, 32, (3, 13)),    # AudioEncoder conv3 geometry, LDS patch
    (256, 128, (3, 3), 1, (1, 1), 8, 16, (4, 12)),     # conv4 geometry
    (256, 128, (3, 8), 1, (0, 0), 8, 16, (4, 5)),      # conv5 geometry (one live column)
    (1024, 128, (4, 4), 1, (1, 1), 6, 12, (0, 13)),    # wide K, every column
])
def test_conv2d_im2col_paths(Ci, Co, k, stride, pad, H, W, cols):
    """Column-range conv2d on the im2col + dense GEMM path (Co >= 128, K >= 2048; one live
    column takes the k-split im2col grid) against torch on the live columns."""
    from a2m import functional as F
    x, w, b = _rand(2, Ci, H, W, seed=33), _rand(Co, Ci, *k, seed=34, scale=0.05), _rand(Co, seed=35)
    assert Ci * k[0] * k[1] >= 2048
    ref = torch.nn.functional.conv2d(x, w, b, stride=stride, padding=pad)
    lo, hi = cols
    hi = min(hi, ref.shape[3])
    out = torch.full(ref.shape, float('nan'), device=DEV)
    F.conv2d(x.to(DEV), w.to(DEV), b.to(DEV), stride, pad, cols=(lo, hi), out=out)
    assert rel_err(out[..., lo:hi].cpu(), ref[..., lo:hi]) < TOL


def test_conv2d_column_range():
    from a2m import functional as F
    x, w, b = _rand(2, 8, 16, 32, seed=30), _rand(12, 8, 4, 4, seed=31, scale=0.2), _rand(12, seed=32)
    ref = torch.nn.functional.conv2d(x, w, b, stride=2, padding=1)
    out = torch.full(ref.shape, float('nan'), device=DEV)
    F.conv2d(x.to(DEV), w.to(DEV), b.to(DEV), 2, (1, 1), cols=(3, 11), out=out)
    assert rel_err(out[..., 3:11].cpu(), ref[..., 3:11]) < TOL
    assert torch.isnan(out[..., :3]).all() and torch.isnan(out[..., 11:]).all()
    w2 = _rand(6, 8, 3, 8, seed=33, scale=0.2)
    ref2 = torch.nn.functional.conv2d(x, w2, None, stride=1, padding=(1, 3))
    out2 = F.conv2d(x.to(DEV), w2.to(DEV), None, 1, (1, 3))
    assert rel_err(out2.cpu(), ref2) < TOL
    # Co >= 128: the explicit 2-D im2col + dense GEMM path (encoder layers), with and without
    # a live-column window, stride 2 / k4 and stride 1 / (3, 8) kernels
    x3 = _rand(3, 64, 16, 24, seed=34)
    for w3, s3, p3, cols in ((_rand(128, 64, 4, 4, seed=35, scale=0.05), 2, (1, 1), (2, 9)),
                             (_rand(128, 64, 3, 8, seed=36, scale=0.05), 1, (1, 3), None)):
        ref3 = torch.nn.functional.conv2d(x3, w3, None, stride=s3, padding=p3)
        out3 = torch.zeros(ref3.shape, device=DEV)
        F.conv2d(x3.to(DEV), w3.to(DEV), None, s3, p3, cols=cols, out=out3)
        lo, hi = cols if cols else (0, ref3.shape[-1])
        assert rel_err(out3[..., lo:hi].cpu(), ref3[..., lo:hi]) < TOL


def test_interp_time():
    from a2m import functional as F
    x = _rand(2, 5, 8, 15, seed=40)
    ref = torch.nn.functional.interpolate(x, size=(64, 1), mode='bilinear').squeeze(-1)
    assert rel_err(F.interp_time(x.to(DEV), 64).cpu(), ref) < TOL
    x2 = _rand(1, 3, 60, 15, seed=41)
    ref2 = torch.nn.functional.interpolate(x2, size=(480, 1), mode='bilinear').squeeze(-1)
    assert rel_err(F.interp_time(x2.to(DEV), 480).cpu(), ref2) < TOL
    # T % 4 != 0: one output per thread instead of float4 runs
    ref3 = torch.nn.functional.interpolate(x, size=(62, 1), mode='bilinear').squeeze(-1)
    assert rel_err(F.interp_time(x.to(DEV), 62).cpu(), ref3) < TOL


@pytest.mark.parametrize('B,C,T', [(2, 256, 64), (2, 2048, 16), (1, 64, 480), (3, 16, 5), (64, 256, 64),
                                   (3, 128, 36), (2, 2048, 32), (3, 2048, 4), (2, 512, 12), (4, 2048, 20)])
def test_self_attention(B, C, T):
    """Eval path: (B, 256, 64) / (B, 128, 36) run the fused QKV + attention kernel
    (a2m_self_attention_eval_f32); C = 2048 / 512 at T <= 32 the wide attention core
    (attn_core_wide_kernel, the UNet's and D's SelfAttention(2048)); the others the packed
    QKV GEMM + core / general path.  The attention matrix kept for the backward pass is
    checked against Q^T K softmax on the host."""
    from a2m import functional as F
    from oracle import model as OM
    x, res = _rand(B, C, T, seed=50), _rand(B, C, T, seed=51)
    sd = {'a.query_conv.weight': _rand(C // 8, C, 1, seed=52, scale=C ** -0.5),
          'a.query_conv.bias': _rand(C // 8, seed=53, scale=0.1),
          'a.key_conv.weight': _rand(C // 8, C, 1, seed=54, scale=C ** -0.5),
          'a.key_conv.bias': _rand(C // 8, seed=55, scale=0.1),
          'a.value_conv.weight': _rand(C, C, 1, seed=56, scale=C ** -0.5),
          'a.value_conv.bias': _rand(C, seed=57, scale=0.1), 'a.gamma': torch.tensor([0.37])}
    ref = OM.self_attention(OM.Ctx(sd), 'a', x) + res
    d = {k: v.to(DEV) for k, v in sd.items()}
    out = F.self_attention(x.to(DEV), d['a.query_conv.weight'], d['a.query_conv.bias'],
                           d['a.key_conv.weight'], d['a.key_conv.bias'], d['a.value_conv.weight'],
                           d['a.value_conv.bias'], d['a.gamma'], res=res.to(DEV))
    assert rel_err(out.cpu(), ref) < TOL
    from a2m import _native as N
    if N.lib.a2m_self_attention_eval_fits(C, T):  # the fused kernel equals the packed path
        save = {}
        out2 = F.self_attention(x.to(DEV), d['a.query_conv.weight'], d['a.query_conv.bias'],
                                d['a.key_conv.weight'], d['a.key_conv.bias'], d['a.value_conv.weight'],
                                d['a.value_conv.bias'], d['a.gamma'], res=res.to(DEV), save=save)
        assert 'qkv' in save and rel_err(out.cpu(), out2.cpu()) < 2e-6
    if N.lib.a2m_self_attention_eval_fits(C, T) and C % 128 == 0:
        # the fused kernel's V chunks of 64 channels (the default) and of 128 (Q / K once per two
        # 64-channel chunks): the same operations per output element, so bitwise equal, fp32 and
        # bf16 operand modes
        # In bf16 mode also with the module cache, i.e. the stacked weights' cached bf16 copy
        # staged as is (a2m_self_attention_eval_ex_f32): the values the kernel would round to.
        outs = {}
        try:
            for prec in (0, 1):
                N.check(N.lib.a2m_set_gemm_precision(prec))
                for nv in (64, 128):
                    N.check(N.lib.a2m_set_attn_eval_chunk(nv))
                    for cached in ((False, True) if prec == 1 else (False,)):
                        outs[prec, nv, cached] = F.self_attention(
                            x.to(DEV), d['a.query_conv.weight'], d['a.query_conv.bias'], d['a.key_conv.weight'],
                            d['a.key_conv.bias'], d['a.value_conv.weight'], d['a.value_conv.bias'], d['a.gamma'],
                            res=res.to(DEV), cache={} if cached else None).cpu()
        finally:
            N.lib.a2m_set_attn_eval_chunk(64)
            N.lib.a2m_set_gemm_precision(0)
        outs = {k[:2] if not k[2] else k: v for k, v in outs.items()}
        assert torch.equal(outs[1, 64], outs[1, 64, True]) and torch.equal(outs[1, 128], outs[1, 128, True])
        assert torch.equal(outs[0, 64], outs[0, 128]) and torch.equal(outs[1, 64], outs[1, 128])
        assert torch.equal(outs[0, 64], out.cpu())
        assert N.lib.a2m_set_attn_eval_chunk(96) == N.A2M_EINVAL
    save = {}
    F.self_attention(x.to(DEV), d['a.query_conv.weight'], d['a.query_conv.bias'], d['a.key_conv.weight'],
                     d['a.key_conv.bias'], d['a.value_conv.weight'], d['a.value_conv.bias'], d['a.gamma'],
                     res=res.to(DEV), save=save)
    q = torch.einsum('oc,bct->bot', sd['a.query_conv.weight'][..., 0], x) + sd['a.query_conv.bias'][None, :, None]
    k = torch.einsum('oc,bct->bot', sd['a.key_conv.weight'][..., 0], x) + sd['a.key_conv.bias'][None, :, None]
    att = torch.softmax(torch.einsum('bci,bcj->bij', q.double(), k.double()), dim=-1)
    assert rel_err(save['attn'].cpu(), att) < TOL


def test_derived_weight_caches_follow_updates():
    """The eval path caches stacked QKV and phase-packed convT weights; torch in-place updates
    (version counters) and FlatAdam's HIP update (weights epoch) must both invalidate them."""
    from a2m.model_layers import ConvTranspose1D, SelfAttention
    from a2m.optim import FlatAdam
    from oracle import model as OM
    torch.manual_seed(3)
    att, ct = SelfAttention(32), ConvTranspose1D(16, 8)
    with torch.no_grad():
        att.gamma.fill_(0.5)
    att, ct = att.to(DEV).eval(), ct.to(DEV).eval()
    x, xc = _rand(2, 32, 12, seed=60).to(DEV), _rand(2, 16, 6, seed=61).to(DEV)

    def refs():
        sd = {'a.' + k: v.detach().cpu() for k, v in att.state_dict().items()}
        ra = OM.self_attention(OM.Ctx(sd), 'a', x.cpu())
        c, n = ct.conv_transpose, ct.bn
        rc = torch.nn.functional.conv_transpose1d(xc.cpu(), c.weight.detach().cpu(), c.bias.detach().cpu(),
                                                  stride=2, padding=1, output_padding=1)
        rc = torch.relu(torch.nn.functional.batch_norm(rc, n.running_mean.cpu(), n.running_var.cpu(),
                                                       n.weight.detach().cpu(), n.bias.detach().cpu(),
                                                       False, 0.0, 1e-5))
        return ra, rc

    with torch.no_grad():
        for step in range(3):
            ra, rc = refs()
            assert rel_err(att(x).cpu(), ra) < TOL and rel_err(ct(xc).cpu(), rc) < TOL, step
            if step == 0:   # torch in-place update
                att.value_conv.weight.mul_(-1.5)
                att.key_conv.weight.add_(0.05)
                ct.conv_transpose.weight.mul_(2.0)
    opt_a, opt_c = FlatAdam(att.parameters(), lr=0.05), FlatAdam(ct.parameters(), lr=0.05)
    with torch.no_grad():   # re-seated parameters: caches rebuilt on the flat buffers
        ra, rc = refs()
        assert rel_err(att(x).cpu(), ra) < TOL and rel_err(ct(xc).cpu(), rc) < TOL
    for o in (opt_a, opt_c):   # the HIP update leaves data_ptr and _version unchanged
        o.flat_grad.copy_(torch.randn_like(o.flat_grad))
        o.step()
    with torch.no_grad():
        ra, rc = refs()
        assert rel_err(att(x).cpu(), ra) < TOL and rel_err(ct(xc).cpu(), rc) < TOL
    # load_state_dict writes through p.copy_ under no_grad; its post-hook bumps the epoch too
    sa = {k: v.clone() * (1.3 if k.endswith('weight') else 1.0) for k, v in att.state_dict().items()}
    sc = {k: v.clone() * (0.7 if k.endswith('weight') else 1.0) for k, v in ct.state_dict().items()}
    att.load_state_dict(sa)
    ct.load_state_dict(sc)
    with torch.no_grad():
        ra, rc = refs()
        assert rel_err(att(x).cpu(), ra) < TOL and rel_err(ct(xc).cpu(), rc) < TOL
    # a write through p.data (e.g. an EMA) is invisible to torch's version counter: the writer
    # calls bump_weights_epoch() (documented contract, functional.py)
    from a2m import functional as F
    att.value_conv.weight.data.mul_(0.5)
    ct.conv_transpose.weight.data.mul_(-1.0)
    F.bump_weights_epoch()
    with torch.no_grad():
        ra, rc = refs()
        assert rel_err(att(x).cpu(), ra) < TOL and rel_err(ct(xc).cpu(), rc) < TOL


def test_channel_attention_layernorm_mean_repeat():
    from a2m import functional as F
    from oracle import model as OM
    x = _rand(3, 256, 64, seed=60)
    sd = {'c.fc.0.weight': _rand(32, 256, seed=61, scale=0.06), 'c.fc.0.bias': _rand(32, seed=62, scale=0.1),
          'c.fc.2.weight': _rand(256, 32, seed=63, scale=0.2), 'c.fc.2.bias': _rand(256, seed=64, scale=0.1)}
    ref = OM.channel_attention(OM.Ctx(sd), 'c', x)
    d = [sd[k].to(DEV) for k in ('c.fc.0.weight', 'c.fc.0.bias', 'c.fc.2.weight', 'c.fc.2.bias')]
    assert rel_err(F.channel_attention(x.to(DEV), *d).cpu(), ref) < TOL
    # the fused (C, T) = (256, 64) kernel in place (y aliasing x), with its weights vector
    xi = x.to(DEV).clone()
    att = torch.empty(3, 256, device=DEV)
    F.channel_attention(xi, *d, out=xi, att=att)
    assert rel_err(xi.cpu(), ref) < TOL
    ra = ref / x
    assert rel_err(att.cpu(), ra[:, :, 0]) < 1e-5
    # the generic two-kernel path (other shapes)
    x2 = _rand(2, 128, 40, seed=68)
    sd2 = {'c.fc.0.weight': _rand(16, 128, seed=69, scale=0.08), 'c.fc.0.bias': _rand(16, seed=70, scale=0.1),
           'c.fc.2.weight': _rand(128, 16, seed=71, scale=0.2), 'c.fc.2.bias': _rand(128, seed=72, scale=0.1)}
    ref2 = OM.channel_attention(OM.Ctx(sd2), 'c', x2)
    d2 = [sd2[k].to(DEV) for k in ('c.fc.0.weight', 'c.fc.0.bias', 'c.fc.2.weight', 'c.fc.2.bias')]
    assert rel_err(F.channel_attention(x2.to(DEV), *d2).cpu(), ref2) < TOL
    rows = _rand(3 * 64, 256, seed=65)
    w, b = _rand(256, seed=66).abs() + .5, _rand(256, seed=67)
    ref = torch.nn.functional.layer_norm(rows, (256,), w, b).view(3, 64, 256).permute(0, 2, 1)
    out = F.layernorm_to_bct(rows.to(DEV), w.to(DEV), b.to(DEV), 64)
    assert rel_err(out.cpu(), ref) < TOL
    assert rel_err(F.mean_time(x.to(DEV)[:, 100:200]).cpu(), x[:, 100:200].mean(2)) < TOL
    buf = torch.zeros(3, 20, 4, device=DEV)
    F.repeat_time(x.to(DEV)[:, :10, 0].contiguous(), buf[:, 10:])
    assert torch.equal(buf[:, 10:].cpu(), x[:, :10, :1].expand(3, 10, 4)) and buf[:, :10].abs().max() == 0


@pytest.mark.parametrize('B,T,D', [(3, 64, 256), (2, 32, 200), (2, 20, 256), (1, 16, 512)])
def test_layernorm_to_bct_paths(B, T, D):
    """LayerNorm of [B*T][D] rows written as [B][D][T] (the decoders' permute), values and the
    saved mean / rstd, against torch, for D up to the kernel's 512 and ragged D / T."""
    from a2m import functional as F
    rows = _rand(B * T, D, seed=68)
    w, b = _rand(D, seed=69).abs() + .5, _rand(D, seed=70)
    ref = torch.nn.functional.layer_norm(rows, (D,), w, b).view(B, T, D).permute(0, 2, 1)
    stats = {}
    out = F.layernorm_to_bct(rows.to(DEV), w.to(DEV), b.to(DEV), T, stats=stats)
    assert out.shape == ref.shape and rel_err(out.cpu(), ref) < TOL
    assert rel_err(stats['mean'].cpu(), rows.mean(1)) < TOL
    var = rows.var(1, unbiased=False)
    assert rel_err(stats['rstd'].cpu(), 1.0 / torch.sqrt(var + 1e-5)) < TOL


@pytest.mark.parametrize('part,J,lo', [('body', 10, 0), ('hand', 42, 10)])
def test_graph_layers_vs_oracle(part, J, lo):
    from a2m import functional as F
    from a2m import skeleton as S
    from oracle import model as OM
    Fr = 37
    x = _rand(Fr * J, 64, seed=70)
    ei = S.edge_index(lo, J)
    edges = OM.expand_edges(ei, J, Fr)
    ptr, idx = S.in_neighbour_csr(ei, J)
    lw, asrc, adst, bias = _rand(256, 64, seed=71, scale=0.15), _rand(1, 4, 64, seed=72, scale=0.3), \
        _rand(1, 4, 64, seed=73, scale=0.3), _rand(64, seed=74, scale=0.1)
    lnw, lnb = _rand(64, seed=75).abs() + .5, _rand(64, seed=76, scale=0.1)
    g = OM._gat_fn(x, edges, lw, asrc, adst, bias, 4)
    ref = torch.nn.functional.leaky_relu(torch.nn.functional.layer_norm(g, (64,), lnw, lnb), 0.2) + x
    dv = lambda t: t.to(DEV)
    out = F.graph_layer(dv(x), J, 0, dv(ptr), dv(idx), dv(lw), None, dv(asrc), dv(adst), dv(bias), dv(lnw), dv(lnb))
    assert rel_err(out.cpu(), ref) < TOL
    bare = F.graph_layer(dv(x), J, 0, dv(ptr), dv(idx), dv(lw), None, dv(asrc), dv(adst), dv(bias),
                         None, None, norm_res=False)
    assert rel_err(bare.cpu(), g) < TOL
    wr, br, wo = _rand(64, 64, seed=77, scale=0.12), _rand(64, seed=78, scale=0.1), _rand(64, 64, seed=79, scale=0.12)
    sd = {'g.lin_rel.weight': wr, 'g.lin_rel.bias': br, 'g.lin_root.weight': wo}
    gc = OM.graph_conv(OM.Ctx(sd), 'g', x, edges)
    ref = torch.nn.functional.leaky_relu(torch.nn.functional.layer_norm(gc, (64,), lnw, lnb), 0.2) + x
    out = F.graph_layer(dv(x), J, 1, dv(ptr), dv(idx), dv(wr), dv(wo), None, None, dv(br), dv(lnw), dv(lnb))
    assert rel_err(out.cpu(), ref) < TOL


@pytest.mark.parametrize('part,J,lo', [('body', 10, 0), ('hand', 42, 10)])
def test_graph_stack_vs_oracle(part, J, lo):
    """The fused 5-layer eval stack (a2m_graph_stack_fwd_f32: GAT, GraphConv, GAT, GraphConv,
    GAT, each + LN64 + LeakyReLU + residual, node tile resident in LDS) against the oracle's
    layer-by-layer PyG restatement, on a frame count that leaves a partial last workgroup."""
    from a2m import functional as F
    from a2m import skeleton as S
    from oracle import model as OM
    Fr = 29
    x = _rand(Fr * J, 64, seed=80)
    ei = S.edge_index(lo, J)
    edges = OM.expand_edges(ei, J, Fr)
    ptr, idx = S.in_neighbour_csr(ei, J)
    dv = lambda t: t.to(DEV)  # noqa: E731
    ref, layers = x, []
    for L in range(5):
        lnw, lnb = _rand(64, seed=90 + L).abs() + .5, _rand(64, seed=95 + L, scale=0.1)
        if L % 2 == 0:
            lw, asrc, adst, bias = _rand(256, 64, seed=100 + L, scale=0.15), \
                _rand(1, 4, 64, seed=110 + L, scale=0.3), _rand(1, 4, 64, seed=120 + L, scale=0.3), \
                _rand(64, seed=130 + L, scale=0.1)
            g = OM._gat_fn(ref, edges, lw, asrc, adst, bias, 4)
            U = F.graph_att_proj(dv(lw), dv(asrc), dv(adst))
            layers.append((0, dv(lw), None, U, dv(bias), dv(lnw), dv(lnb)))
        else:
            wr, br, wo = _rand(64, 64, seed=140 + L, scale=0.12), _rand(64, seed=150 + L, scale=0.1), \
                _rand(64, 64, seed=160 + L, scale=0.12)
            g = OM.graph_conv(OM.Ctx({'g.lin_rel.weight': wr, 'g.lin_rel.bias': br,
                                      'g.lin_root.weight': wo}), 'g', ref, edges)
            layers.append((1, dv(wr), dv(wo), None, dv(br), dv(lnw), dv(lnb)))
        ref = torch.nn.functional.leaky_relu(torch.nn.functional.layer_norm(g, (64,), lnw, lnb), 0.2) + ref
    out = F.graph_stack(dv(x), J, dv(ptr), dv(idx), layers)
    e = rel_err(out.cpu(), ref)
    assert e < TOL, e


@pytest.mark.parametrize('part,J,lo', [('body', 10, 0), ('hand', 42, 10)])
def test_graph_stack_bf16_mode(part, J, lo):
    """The stack in bf16 operand mode (configs[4]: the layer products on the bf16 MFMA, as
    torch.autocast runs GATConv / GraphConv's linears in bf16) against the fp32 oracle at a
    bf16-level tolerance, and against the fp32 kernel."""
    import a2m
    from a2m import functional as F
    from a2m import skeleton as S
    from oracle import model as OM
    Fr = 29
    x = _rand(Fr * J, 64, seed=80)
    ei = S.edge_index(lo, J)
    edges = OM.expand_edges(ei, J, Fr)
    ptr, idx = S.in_neighbour_csr(ei, J)
    dv = lambda t: t.to(DEV)  # noqa: E731
    ref, layers = x, []
    for L in range(5):
        lnw, lnb = _rand(64, seed=90 + L).abs() + .5, _rand(64, seed=95 + L, scale=0.1)
        if L % 2 == 0:
            lw, asrc, adst, bias = _rand(256, 64, seed=100 + L, scale=0.15), \
                _rand(1, 4, 64, seed=110 + L, scale=0.3), _rand(1, 4, 64, seed=120 + L, scale=0.3), \
                _rand(64, seed=130 + L, scale=0.1)
            g = OM._gat_fn(ref, edges, lw, asrc, adst, bias, 4)
            U = F.graph_att_proj(dv(lw), dv(asrc), dv(adst))
            layers.append((0, dv(lw), None, U, dv(bias), dv(lnw), dv(lnb)))
        else:
            wr, br, wo = _rand(64, 64, seed=140 + L, scale=0.12), _rand(64, seed=150 + L, scale=0.1), \
                _rand(64, 64, seed=160 + L, scale=0.12)
            g = OM.graph_conv(OM.Ctx({'g.lin_rel.weight': wr, 'g.lin_rel.bias': br,
                                      'g.lin_root.weight': wo}), 'g', ref, edges)
            layers.append((1, dv(wr), dv(wo), None, dv(br), dv(lnw), dv(lnb)))
        ref = torch.nn.functional.leaky_relu(torch.nn.functional.layer_norm(g, (64,), lnw, lnb), 0.2) + ref
    out32 = F.graph_stack(dv(x), J, dv(ptr), dv(idx), layers).cpu()
    # the layer weights' cached bf16 copies (a2m_to_bf16_f32: the same RNE values torch's cast
    # gives) feed the k loops the values it would round itself: bitwise the same stack output
    wh = [F.graph_weights_bf16(Lr[1], Lr[2], {}) for Lr in layers]
    for Lr, (h0, h1) in zip(layers, wh):
        assert torch.equal(h0.cpu(), Lr[1].cpu().to(torch.bfloat16))
        assert h1 is None or torch.equal(h1.cpu(), Lr[2].cpu().to(torch.bfloat16))
    odd = dv(_rand(7, seed=170))
    assert torch.equal(F.to_bf16(odd).cpu(), odd.cpu().to(torch.bfloat16))
    prev = a2m.set_gemm_precision('bf16')
    try:
        out16 = F.graph_stack(dv(x), J, dv(ptr), dv(idx), layers).cpu()
        out16h = F.graph_stack(dv(x), J, dv(ptr), dv(idx), layers, wh=wh).cpu()
    finally:
        a2m.set_gemm_precision(prev)
    assert torch.equal(out16, out16h)
    assert torch.equal(F.graph_stack(dv(x), J, dv(ptr), dv(idx), layers, wh=wh).cpu(), out32)  # fp32 ignores wh
    e16, e32 = rel_err(out16, ref), rel_err(out32, ref)
    print(f'{part}: bf16 stack vs oracle {e16:.2e}, fp32 stack {e32:.2e}')
    assert e32 < TOL and 1e-6 < e16 < 3e-2, (e16, e32)


def test_pose_losses_vs_reference():
    from a2m import functional as F
    z = golden('losses.npz')
    out = F.pose_losses(torch.from_numpy(z['gen']).to(DEV), torch.from_numpy(z['real']).to(DEV)).cpu()
    assert rel_err(out[0], z['bone']) < TOL and rel_err(out[1], z['angle']) < TOL
    out2 = F.pose_losses(torch.from_numpy(z['gen']).to(DEV)).cpu()
    assert rel_err(out2[1], z['angle']) < TOL and out2[0].item() == 0.0  # no real pose: bone 0


def test_angle_loss_methods_vs_reference(g_state):
    """SelfAttention_G.compute_{bone_length, hand_joint_angle, body_joint_angle,
    comprehensive_angle}_loss (real_motion_model.py:307-461) against the reference's values,
    on device and on host tensors, and differentiable in gen_pose."""
    from a2m.real_motion_model import SelfAttention_G
    z = golden('losses.npz')
    g = SelfAttention_G(p=0.0).to(DEV)
    gen, real = torch.from_numpy(z['gen']), torch.from_numpy(z['real'])
    for dev in (DEV, 'cpu'):
        gd, rd = gen.to(dev), real.to(dev)
        vals = {'bone': g.compute_bone_length_loss(rd, gd), 'hand': g.compute_hand_joint_angle_loss(gd),
                'body': g.compute_body_joint_angle_loss(gd), 'angle': g.compute_comprehensive_angle_loss(gd)}
        for k, v in vals.items():
            assert v.device.type == torch.device(dev).type, (k, dev)
            assert rel_err(v.detach().cpu(), z[k]) < TOL, (k, dev)
    from oracle import model as OM
    for name, fn, ref_fn in (('hand', g.compute_hand_joint_angle_loss, OM.hand_angle_loss),
                             ('body', g.compute_body_joint_angle_loss, OM.body_angle_loss)):
        x = gen.clone().to(DEV).requires_grad_(True)
        fn(x).backward()
        x64 = gen.double().requires_grad_(True)
        ref_fn(x64).backward()
        assert rel_err(x.grad.cpu().double(), x64.grad) < 2e-5, name
    assert g.compute_body_joint_angle_loss(gen[..., :100].to(DEV)).item() == 0.0   # :403-404


def test_host_tensor_entry_generator_and_discriminator(g_state, d_state):
    """generate_motion_video.py:235-257: a generator constructed on the host, loaded from a
    checkpoint, called on host tensors, left in train mode under no_grad.  The module moves
    itself to the GPU once; results come back on the host; eval-mode values match the
    device path."""
    from a2m.real_motion_model import SelfAttention_D, SelfAttention_G
    z = golden('g_eval_b2t64.npz')
    g = SelfAttention_G(p=0.0)
    g.load_state_dict(g_state, strict=False)
    audio = torch.from_numpy(z['audio'])
    with torch.no_grad():
        pose, losses = g(audio)          # train mode, as the script leaves it
    assert pose.device.type == 'cpu' and all(l.device.type == 'cpu' for l in losses)
    assert next(g.parameters()).is_cuda and pose.shape == (2, 64, 104) and torch.isfinite(pose).all()
    g.load_state_dict(g_state, strict=False)   # the train-mode call moved the BN running stats
    g.eval()
    with torch.no_grad():
        pose_e, losses_e = g(audio, real_pose=torch.from_numpy(z['real_pose']))
    assert pose_e.device.type == 'cpu' and len(losses_e) == 2
    assert rel_err(pose_e, z['pose']) < TOL
    d = SelfAttention_D(out_channels=64, p=0.0)
    d.load_state_dict(d_state, strict=False)
    d.eval()
    with torch.no_grad():
        dr, aux = d(torch.diff(torch.from_numpy(z['real_pose']), dim=1))
    assert dr.device.type == 'cpu' and aux == [] and rel_err(dr, z['d_real']) < TOL


# ------------------------------------------------------------------------------ full model
def _g(g_state):
    from a2m.real_motion_model import SelfAttention_G
    m = SelfAttention_G(p=0.0)
    m.load_state_dict(g_state, strict=False)
    return m.to(DEV).eval()


def test_generator_eval_vs_reference(g_state):
    z = golden('g_eval_b2t64.npz')
    m = _g(g_state)
    with torch.no_grad():
        out, losses = m(torch.from_numpy(z['audio']).to(DEV), real_pose=torch.from_numpy(z['real_pose']).to(DEV))
        feats = m.audio_encoder(torch.from_numpy(z['audio']).to(DEV))
        ref_feats = m.unet(feats)
    assert rel_err(feats.cpu(), z['act/audio_encoder']) < TOL
    assert rel_err(ref_feats.cpu(), z['act/unet']) < TOL
    assert rel_err(out.cpu(), z['pose']) < TOL
    assert rel_err(losses[0].cpu(), z['bone']) < TOL
    assert rel_err(losses[1].cpu(), z['angle']) < TOL


def test_generator_longform_vs_reference(g_state):
    z = golden('g_eval_b1t480.npz')
    m = _g(g_state)
    with torch.no_grad():
        out, losses = m(torch.from_numpy(z['audio']).to(DEV))
    assert rel_err(out.cpu(), z['pose']) < TOL
    assert len(losses) == 1 and rel_err(losses[0].cpu(), z['angle']) < TOL


def test_mel_plus_generator_end_to_end(g_state):
    """wave -> HIP log-mel -> HIP generator vs reference mel_features + reference G."""
    from a2m.mel_features import log_mel_batch
    zm, z = golden('mel.npz'), golden('g_eval_b2t64.npz')
    m = _g(g_state)
    with torch.no_grad():
        mel = log_mel_batch(torch.from_numpy(zm['mel_build_wave']).to(DEV))
        out, _ = m(mel, real_pose=torch.from_numpy(z['real_pose']).to(DEV))
    assert rel_err(out.cpu(), z['pose']) < TOL


def test_discriminator_eval_vs_reference(d_state):
    from a2m.real_motion_model import SelfAttention_D
    z = golden('g_eval_b2t64.npz')
    d = SelfAttention_D(out_channels=64, p=0.0)
    d.load_state_dict(d_state, strict=False)
    d = d.to(DEV).eval()
    with torch.no_grad():
        out, _ = d(torch.diff(torch.from_numpy(z['real_pose']), dim=1).to(DEV))
    assert rel_err(out.cpu(), z['d_real']) < TOL


def test_full_size_batch_invariance(g_state):
    """B=64 x T=64 (the bench workload): every clip's output equals the same clip run alone
    (clips are independent in eval mode) and is finite."""
    from a2m.mel_features import log_mel_batch
    from oracle import synth
    m = _g(g_state)
    wav = torch.from_numpy(synth.speech_like(64, synth.samples_for_frames(64), seed=3)).to(DEV)
    with torch.no_grad():
        mel = log_mel_batch(wav)
        out, losses = m(mel)
        solo, _ = m(mel[17:18])
        solo2, _ = m(mel[63:64])
    assert torch.isfinite(out).all() and torch.isfinite(losses[0])
    assert rel_err(out[17:18].cpu(), solo.cpu()) < TOL
    assert rel_err(out[63:64].cpu(), solo2.cpu()) < TOL


def test_headline_b64_bench_step_vs_reference(g_state):
    """configs[1] at its real size: the exact bench step (bench.infer_step: HIP log-mel over
    64 resident 69,269-sample waveforms + SelfAttention_G eval, captured in one HIP graph by
    bench.capture_step and replayed) against the reference's own mel and pose for the same
    waveforms (tests/golden/g_eval_b64t64.npz, oracle/make_fixtures_r2.py)."""
    import bench
    from a2m.mel_features import log_mel_batch
    from a2m.real_motion_model import SelfAttention_G
    from oracle import synth
    z = golden('g_eval_b64t64.npz')
    wav = synth.speech_like(64, synth.samples_for_frames(64), seed=int(z['seed']))
    wave = torch.from_numpy(wav).to(DEV)
    g = SelfAttention_G(p=0.0)
    g.load_state_dict(g_state, strict=False)
    g = g.to(DEV).eval()
    with torch.no_grad():
        graph, out = bench.capture_step(torch.device(DEV), bench.infer_step(g, wave))
        out.zero_()
        graph.replay()
        graph.replay()
        torch.cuda.synchronize()
        mel = log_mel_batch(wave)
    assert out.shape == (64, 64, 104)
    assert rel_err(mel.cpu().numpy(), z['mel']) < TOL
    assert rel_err(out.cpu().numpy(), z['pose']) < TOL, rel_err(out.cpu().numpy(), z['pose'])
