"""Device ops: thin wrappers that hand torch tensors' device pointers / strides / the current
HIP stream to liba2m_hip.so.  PyTorch is used only for allocation and views.

Every function requires fp32 tensors on a ROCm device; there is no CPU path.
"""
import ctypes
import re

import torch

from . import _native as N

ACT_NONE, ACT_RELU, ACT_LRELU = 0, 1, 2

_NULL = None


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _check_dev(*ts):
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError('a2m ops need device tensors (no CPU fallback); got a CPU tensor')
        if t.dtype != torch.float32:
            raise TypeError(f'a2m ops compute in fp32; got {t.dtype}')


class _Workspace:
    """One growable scratch buffer per device (ops on one stream run in order)."""

    def __init__(self):
        self.buf = {}

    def get(self, device, nbytes=0):
        key = torch.device(device).index or 0
        cur = self.buf.get(key)
        if cur is None or cur.numel() < nbytes:
            size = max(nbytes, 64 << 20, 0 if cur is None else 2 * cur.numel())
            cur = torch.empty(size, dtype=torch.uint8, device=device)
            self.buf[key] = cur
        return cur


WS = _Workspace()


def _with_ws(device, call):
    ws = WS.get(device)
    for _ in range(4):
        rc = call(ctypes.c_void_p(ws.data_ptr()), ws.numel())
        if rc != N.A2M_EWS:
            N.check(rc)
            return
        m = re.search(r'<\s*(\d+)', N.last_error())
        need = int(m.group(1)) if m else 2 * ws.numel()
        ws = WS.get(device, need)
    N.check(rc)


def _bn_args(bn):
    if bn is None:
        return [None, None, None, None, 1e-5]
    w, b, rm, rv, eps = bn
    return [_p(w), _p(b), _p(rm), _p(rv), float(eps)]


# ------------------------------------------------------------------------------ convs
def conv1d(x, w, b=None, stride=1, pad=0, bn=None, act=ACT_NONE, slope=0.2, out=None):
    """x: [B, Ci, Tin] (any strides), w: [Co, Ci, k] (or [Co, Ci] for a linear / 1x1).
    Returns / fills out [B, Co, Tout] (any strides)."""
    _check_dev(x, w, b, out)
    B, Ci, Tin = x.shape
    Co, ks = w.shape[0], (w.shape[2] if w.dim() == 3 else 1)
    assert w.shape[1] == Ci and w.is_contiguous()
    Tout = (Tin + 2 * pad - ks) // stride + 1
    if out is None:
        out = torch.empty(B, Co, Tout, device=x.device, dtype=x.dtype)
    assert tuple(out.shape) == (B, Co, Tout), (out.shape, (B, Co, Tout))
    xs, ys = list(x.stride()), list(out.stride())
    if B == 1:  # batch stride is irrelevant; make single-batch row views look uniform
        xs[0], ys[0] = Tin * xs[2], Tout * ys[2]
    _with_ws(x.device, lambda wp, wn: N.lib.a2m_conv1d_fwd_f32(
        _p(x), xs[0], xs[1], xs[2], B, Ci, Tin, _p(w), _p(b), Co, ks, stride, pad,
        *_bn_args(bn), act, slope, _p(out), ys[0], ys[1], ys[2], wp, wn, _stream()))
    return out


def linear(x, w, b=None, out=None):
    """y = x W^T + b over the last dim of x ([..., I] -> [..., O])."""
    lead = x.shape[:-1]
    x2 = x.reshape(-1, x.shape[-1])
    R = x2.shape[0]
    y = out if out is not None else torch.empty(*lead, w.shape[0], device=x.device, dtype=x.dtype)
    y2 = y.view(R, w.shape[0])
    conv1d(x2.t().unsqueeze(0), w, b, out=y2.t().unsqueeze(0))
    return y


def convt1d(x, w, b=None, stride=2, pad=1, out_pad=1, bn=None, act=ACT_NONE, slope=0.2, out=None):
    """x: [B, Ci, Tin] (t contiguous), w: [Ci, Co, k]."""
    _check_dev(x, w, b, out)
    B, Ci, Tin = x.shape
    assert x.stride(2) == 1 and w.is_contiguous() and w.shape[0] == Ci
    Co, ks = w.shape[1], w.shape[2]
    Tout = (Tin - 1) * stride - 2 * pad + ks + out_pad
    if out is None:
        out = torch.empty(B, Co, Tout, device=x.device, dtype=x.dtype)
    assert tuple(out.shape) == (B, Co, Tout) and out.stride(2) == 1
    _with_ws(x.device, lambda wp, wn: N.lib.a2m_convt1d_fwd_f32(
        _p(x), x.stride(0), x.stride(1), B, Ci, Tin, _p(w), _p(b), Co, ks, stride, pad, out_pad,
        *_bn_args(bn), act, slope, _p(out), out.stride(0), out.stride(1), wp, wn, _stream()))
    return out


def conv2d(x, w, b=None, stride=1, pad=(0, 0), bn=None, act=ACT_NONE, slope=0.2, cols=None, out=None):
    """x contiguous [B, Ci, H, W]; computes output columns cols=(lo, hi) only (default all)."""
    _check_dev(x, w, b, out)
    assert x.is_contiguous() and w.is_contiguous()
    B, Ci, H, W = x.shape
    Co, _, kh, kw = w.shape
    ph, pw = pad
    Ho, Wo = (H + 2 * ph - kh) // stride + 1, (W + 2 * pw - kw) // stride + 1
    lo, hi = cols if cols is not None else (0, Wo)
    if out is None:
        out = torch.empty(B, Co, Ho, Wo, device=x.device, dtype=x.dtype)
    assert tuple(out.shape) == (B, Co, Ho, Wo) and out.is_contiguous()
    _with_ws(x.device, lambda wp, wn: N.lib.a2m_conv2d_fwd_f32(
        _p(x), B, Ci, H, W, _p(w), _p(b), Co, kh, kw, stride, ph, pw, *_bn_args(bn), act, slope,
        _p(out), Ho, Wo, lo, hi, wp, wn, _stream()))
    return out


def interp_time(x, T, out=None):
    _check_dev(x)
    assert x.is_contiguous()
    B, C, H, W = x.shape
    if out is None:
        out = torch.empty(B, C, T, device=x.device, dtype=x.dtype)
    N.check(N.lib.a2m_interp_time_f32(_p(x), B, C, H, W, _p(out), T, _stream()))
    return out


def mean_time(x, out=None):
    _check_dev(x, out)
    B, C, T = x.shape
    assert x.stride(2) == 1
    if out is None:
        out = torch.empty(B, C, device=x.device)
    N.check(N.lib.a2m_mean_time_f32(_p(x), x.stride(0), x.stride(1), B, C, T, _p(out), _stream()))
    return out


def repeat_time(x, out):
    """out[b, c, t] = x[b, c] for a [B, C, T] (t-contiguous) view `out`."""
    _check_dev(x, out)
    B, C, T = out.shape
    assert x.is_contiguous() and tuple(x.shape) == (B, C) and out.stride(2) == 1
    N.check(N.lib.a2m_repeat_time_f32(_p(x), B, C, T, _p(out), out.stride(0), out.stride(1), _stream()))
    return out


# ------------------------------------------------------------------------- attention
def self_attention(x, wq, bq, wk, bk, wv, bv, gamma, res=None, out=None, save=None):
    """SelfAttention forward.  x, res, out: [B, C, T] with t contiguous and channel stride T.
    `save`, if a dict, receives the qkv and attention intermediates."""
    _check_dev(x, wq, wk, wv, gamma, res, out)
    B, C, T = x.shape
    assert x.stride(2) == 1 and x.stride(1) == T
    if out is None:
        out = torch.empty(B, C, T, device=x.device, dtype=x.dtype)
    assert out.stride(0) == x.stride(0) and out.stride(1) == T and out.stride(2) == 1
    if res is not None:
        assert res.stride() == out.stride()
    qkv = torch.empty(B, C // 4 + C, T, device=x.device, dtype=x.dtype)
    attn = torch.empty(B, T, T, device=x.device, dtype=x.dtype)
    _with_ws(x.device, lambda wp, wn: N.lib.a2m_self_attention_fwd_f32(
        _p(x), x.stride(0), B, C, T, _p(wq), _p(bq), _p(wk), _p(bk), _p(wv), _p(bv), _p(gamma),
        _p(res), _p(out), out.stride(0), _p(qkv), _p(attn), wp, wn, _stream()))
    if save is not None:
        save['qkv'], save['attn'] = qkv, attn
    return out


def channel_attention(x, w1, b1, w2, b2, out=None, att=None):
    _check_dev(x, w1, b1, w2, b2, out)
    assert x.is_contiguous()
    B, C, T = x.shape
    if out is None:
        out = torch.empty_like(x)
    N.check(N.lib.a2m_channel_attention_fwd_f32(_p(x), B, C, T, _p(w1), _p(b1), w1.shape[0],
                                                _p(w2), _p(b2), _p(out), _p(att), _stream()))
    return out


def layernorm_to_bct(x, w, b, T, eps=1e-5, out=None, stats=None):
    """x: [B*T, D] rows -> LayerNorm over D -> written as [B, D, T] (the decoders' permute)."""
    _check_dev(x, w, b, out)
    assert x.is_contiguous()
    R, D = x.shape
    if out is None:
        out = torch.empty(R // T, D, T, device=x.device, dtype=x.dtype)
    mean = rstd = None
    if stats is not None:
        mean = torch.empty(R, device=x.device)
        rstd = torch.empty(R, device=x.device)
        stats['mean'], stats['rstd'] = mean, rstd
    N.check(N.lib.a2m_layernorm_fwd_f32(_p(x), R, D, _p(w), _p(b), eps, _p(out), T, out.stride(0),
                                        out.stride(1), out.stride(2), _p(mean), _p(rstd), _stream()))
    return out


# ------------------------------------------------------------------------- graph layer
def graph_layer(x, J, kind, nbr_ptr, nbr_idx, w0, w1, att_src, att_dst, bias, ln_w, ln_b,
                slope=0.2, out=None, pre_ln=None, norm_res=True):
    """x: [F*J, 64] contiguous node features; kind 0 = GATConv(heads 4, mean), 1 = GraphConv."""
    _check_dev(x, w0, w1, att_src, att_dst, bias, ln_w, ln_b, out)
    assert x.is_contiguous() and x.shape[1] == 64 and x.shape[0] % J == 0
    F = x.shape[0] // J
    if out is None:
        out = torch.empty_like(x)
    _with_ws(x.device, lambda wp, wn: N.lib.a2m_graph_layer_fwd_f32(
        _p(x), F, J, kind, int(norm_res), _p(nbr_ptr), _p(nbr_idx), _p(w0), _p(w1), _p(att_src),
        _p(att_dst), _p(bias), _p(ln_w), _p(ln_b), slope, _p(out), None, _p(pre_ln), wp, wn, _stream()))
    return out


# ------------------------------------------------------------------------- losses
def pose_losses(gen, real=None):
    """Returns a [2] tensor: (bone loss or 0 if real is None, comprehensive angle loss)."""
    _check_dev(gen, real)
    B, T, Fd = gen.shape
    assert Fd == 104 and gen.stride(2) == 1
    out = torch.zeros(2, device=gen.device)
    rs = real.stride() if real is not None else (0, 0, 1)
    if real is not None:
        assert real.stride(2) == 1
    _with_ws(gen.device, lambda wp, wn: N.lib.a2m_pose_losses_f32(
        _p(gen), gen.stride(0), gen.stride(1), _p(real), rs[0], rs[1], B, T, _p(out), wp, wn,
        _stream()))
    return out


# ------------------------------------------------------------------------- log-mel
class LogMelPlan:
    """Device-resident window / twiddle / banded-filterbank plan for one front-end config."""
    _cache = {}

    def __init__(self, sample_rate, window_secs, hop_secs, n_mels, lower_hz, upper_hz, device):
        win, hop, nfft = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        N.check(N.lib.a2m_logmel_geometry(sample_rate, window_secs, hop_secs, ctypes.byref(win),
                                          ctypes.byref(hop), ctypes.byref(nfft)), value_error=True)
        self.window, self.hop, self.fft_len, self.n_mels = win.value, hop.value, nfft.value, n_mels
        nbytes = N.lib.a2m_logmel_plan_bytes(sample_rate, window_secs, hop_secs, n_mels, lower_hz, upper_hz)
        host = torch.zeros(max(nbytes, 16), dtype=torch.uint8)
        N.check(N.lib.a2m_logmel_plan_build(sample_rate, window_secs, hop_secs, n_mels, lower_hz,
                                            upper_hz, ctypes.c_void_p(host.data_ptr()), host.numel()),
                value_error=True)
        self.dev = host.to(device)

    @classmethod
    def get(cls, sample_rate, window_secs, hop_secs, n_mels, lower_hz, upper_hz, device):
        key = (int(sample_rate), float(window_secs), float(hop_secs), int(n_mels), float(lower_hz),
               float(upper_hz), str(torch.device(device)))
        if key not in cls._cache:
            cls._cache[key] = cls(*key[:6], device)
        return cls._cache[key]

    def num_frames(self, n_samples):
        return int(N.lib.a2m_logmel_num_frames(n_samples, self.window, self.hop))


def log_mel(wave, plan, log_offset, out=None):
    """wave [C, S] fp32 device tensor (s contiguous) -> [C, F, n_mels]."""
    _check_dev(wave, out)
    assert wave.dim() == 2 and wave.stride(1) == 1
    C, S = wave.shape
    F = plan.num_frames(S)
    if out is None:
        out = torch.empty(C, F, plan.n_mels, device=wave.device, dtype=torch.float32)
    N.check(N.lib.a2m_logmel_f32(_p(wave), C, wave.stride(0), S, plan.window, plan.hop, plan.fft_len,
                                 plan.n_mels, _p(plan.dev), float(log_offset), _p(out), _stream()))
    return out
