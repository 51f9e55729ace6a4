"""Device ops: thin wrappers that hand torch tensors' device pointers / strides / the current
HIP stream to liba2m_hip.so.  PyTorch is used only for allocation and views.

Every function requires fp32 tensors on a ROCm device; there is no CPU path.
"""
import ctypes
import os
import re

import torch

from . import _native as N

ACT_NONE, ACT_RELU, ACT_LRELU = 0, 1, 2

_native_lib = N.lib


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
    """One growable scratch buffer per (device, stream): ops on one stream run in order, and
    streams that run concurrently (the generator's body / hand branches) get their own."""

    def __init__(self):
        self.buf = {}

    def get(self, device, nbytes=0):
        device = torch.device(device)
        key = (device.index or 0, torch.cuda.current_stream(device).cuda_stream)
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
        # composite ops report the need of their inner GEMM only, so grow by at least 2x
        m = re.search(r'<\s*(\d+)', N.last_error())
        need = int(m.group(1)) if m else 0
        ws = WS.get(device, max(need, 2 * ws.numel()))
    N.check(rc)


def _bn_args(bn):
    if bn is None:
        return [None, None, None, None, 1e-5]
    w, b, rm, rv, eps = bn
    return [_p(w), _p(b), _p(rm), _p(rv), float(eps)]


# ------------------------------------------------------------------------------ convs
# module flags (tests reach the alternative routes by flipping them): tap-chunked conv1d /
# ConvTranspose phases (the gathered im2col routes measured 5-11 % slower per layer)
_TAP_CONV = True
_TAP_CONVT = True


def _tap_eligible(x, ks, stride, pad, Ci):
    T = x.shape[2]
    return (_TAP_CONV and ks > 1 and stride == 1 and 2 * pad == ks - 1 and x.stride(2) == 1 and
            T % 4 == 0 and 64 % T == 0 and pad < T and x.data_ptr() % 16 == 0 and
            (x.stride(0) % 4 == 0 or x.shape[0] == 1) and x.stride(1) % 4 == 0)


def conv1d_tap_packed(w, cache=None):
    """Tap-chunked conv1d weights [Co][Ci/chunk][k][chunk] for the engine's current k-tile
    (a2m_conv1d_tap_pack_f32), cached in `cache` per weight version and chunk."""
    chunk = N.lib.a2m_conv1d_tap_chunk()
    key = _wkey((w,)) + (chunk,)
    if cache is not None and cache.get('key') == key:
        return cache['w'], chunk
    Co, Ci, ks = w.shape
    packed = torch.empty(Co * Ci * ks, device=w.device)
    N.check(N.lib.a2m_conv1d_tap_pack_f32(_p(w), Co, Ci, ks, chunk, _p(packed), _stream()))
    if cache is not None:
        cache.update(key=key, w=packed)
    return packed, chunk


def conv1d(x, w, b=None, stride=1, pad=0, bn=None, act=ACT_NONE, slope=0.2, out=None, cache=None):
    """x: [B, Ci, Tin] (any strides), w: [Co, Ci, k] (or [Co, Ci] for a linear / 1x1).
    Returns / fills out [B, Co, Tout] (any strides).  With `cache` (a dict owned by the module),
    stride-1 same-padded convs over clips that tile the GEMM's 64 rows run on the tap-chunked
    path (a2m_conv1d_tap_fwd_f32: no im2col matrix; packed weights kept in `cache`)."""
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
    if cache is not None and _tap_eligible(x, ks, stride, pad, Ci) and \
            Ci % N.lib.a2m_conv1d_tap_chunk() == 0:
        packed, chunk = conv1d_tap_packed(w, cache)
        _with_ws(x.device, lambda wp, wn: N.lib.a2m_conv1d_tap_fwd_f32(
            _p(x), xs[0], xs[1], B, Ci, Tin, _p(packed), chunk, _p(b), Co, ks, pad,
            *_bn_args(bn), act, slope, _p(out), ys[0], ys[1], ys[2], wp, wn, _stream()))
        return out
    _with_ws(x.device, lambda wp, wn: N.lib.a2m_conv1d_fwd_f32(
        _p(x), xs[0], xs[1], xs[2], B, Ci, Tin, _p(w), _p(b), Co, ks, stride, pad,
        *_bn_args(bn), act, slope, _p(out), ys[0], ys[1], ys[2], wp, wn, _stream()))
    return out


def _group_stride(ts):
    """Element offset between consecutive problems of a grouped launch (uniform spacing; the
    tensors may live in different allocations -- the kernels only add g * stride)."""
    if len(ts) == 1:
        return 0
    d = ts[1].data_ptr() - ts[0].data_ptr()
    for i in range(2, len(ts)):
        assert ts[i].data_ptr() - ts[i - 1].data_ptr() == d, 'grouped operands must be evenly spaced'
    assert d % 16 == 0
    return d // 4


def conv1d_tap_group(xs, packed, chunk, bias, Co, ks, pad, bn, act, slope, outs):
    """G same-shape tap-chunked conv1d problems in one launch (a2m_conv1d_tap_group_fwd_f32).
    xs / outs: lists of G [B, Ci, T] / [B, Co, T] views with equal strides; packed [G, n] and
    bias / BN tensors [G, Co] stacked per problem (see group_params)."""
    x0, y0 = xs[0], outs[0]
    _check_dev(x0, y0, packed)
    B, Ci, T = x0.shape
    assert all(x.stride() == x0.stride() and x.shape == x0.shape for x in xs)
    assert all(y.stride() == y0.stride() and tuple(y.shape) == (B, Co, T) for y in outs)
    assert _tap_eligible(x0, ks, 1, pad, Ci) and Ci % chunk == 0 and chunk == N.lib.a2m_conv1d_tap_chunk()
    G = len(xs)
    xs_g, ys_g = _group_stride(xs), _group_stride(outs)
    xsb, ysb = x0.stride(0), y0.stride(0)
    if B == 1:
        xsb, ysb = T * x0.stride(2), T * y0.stride(2)
    _with_ws(x0.device, lambda wp, wn: N.lib.a2m_conv1d_tap_group_fwd_f32(
        _p(x0), xs_g, xsb, x0.stride(1), G, B, Ci, T, _p(packed), packed.stride(0), chunk, _p(bias), Co,
        ks, pad, *_bn_args(bn), act, slope, _p(y0), ys_g, ysb, y0.stride(1), y0.stride(2), wp, wn,
        _stream()))
    return outs


def linear(x, w, b=None, out=None):
    """y = x W^T + b over the last dim of x ([..., I] -> [..., O])."""
    lead = x.shape[:-1]
    x2 = x.reshape(-1, x.shape[-1])
    R = x2.shape[0]
    y = out if out is not None else torch.empty(*lead, w.shape[0], device=x.device, dtype=x.dtype)
    y2 = y.view(R, w.shape[0])
    conv1d(x2.t().unsqueeze(0), w, b, out=y2.t().unsqueeze(0))
    return y


def convt_packed(w, stride, pad, cache=None):
    """Phase-packed ConvTranspose1d weights (a2m_convt1d_pack_f32), cached in `cache`."""
    key = _wkey((w,)) + (stride, pad)
    if cache is not None and cache.get('key') == key:
        return cache['w']
    Ci, Co, ks = w.shape
    packed = torch.empty(Ci * Co * ks, device=w.device)
    N.check(N.lib.a2m_convt1d_pack_f32(_p(w), Ci, Co, ks, stride, pad, _p(packed), _stream()))
    if cache is not None:
        cache.update(key=key, w=packed)
    return packed


def convt_tap_packed(w, stride, pad, cache=None):
    """Per-phase tap-chunked ConvTranspose1d weights for the engine's current k-tile
    (a2m_convt1d_tap_pack_f32), cached in `cache` per weight version and chunk."""
    chunk = N.lib.a2m_conv1d_tap_chunk()
    key = _wkey((w,)) + (stride, pad, 'tap', chunk)
    if cache is not None and cache.get('key') == key:
        return cache['w'], chunk
    Ci, Co, ks = w.shape
    packed = torch.empty(Ci * Co * ks, device=w.device)
    N.check(N.lib.a2m_convt1d_tap_pack_f32(_p(w), Ci, Co, ks, stride, pad, chunk, _p(packed), _stream()))
    if cache is not None:
        cache.update(key=key, w=packed)
    return packed, chunk


def _convt_tap_eligible(x, stride, Tout):
    B, Ci, Tin = x.shape
    return (_TAP_CONVT and Tout == stride * Tin and Tin % 4 == 0 and 64 % Tin == 0 and
            Ci % N.lib.a2m_conv1d_tap_chunk() == 0 and x.data_ptr() % 16 == 0 and
            x.stride(0) % 4 == 0 and x.stride(1) % 4 == 0)


def convt1d(x, w, b=None, stride=2, pad=1, out_pad=1, bn=None, act=ACT_NONE, slope=0.2, out=None,
            cache=None):
    """x: [B, Ci, Tin] (t contiguous), w: [Ci, Co, k]; `cache` keeps the packed weights.
    Clip lengths that tile the engine's 64 rows run each output phase as a tap-chunked conv1d
    (a2m_convt1d_tap_fwd_f32), others the per-phase gathered GEMM (a2m_convt1d_packed_fwd_f32)."""
    _check_dev(x, w, b, out)
    B, Ci, Tin = x.shape
    assert x.stride(2) == 1 and w.is_contiguous() and w.shape[0] == Ci
    Co, ks = w.shape[1], w.shape[2]
    Tout = (Tin - 1) * stride - 2 * pad + ks + out_pad
    if out is None:
        out = torch.empty(B, Co, Tout, device=x.device, dtype=x.dtype)
    assert tuple(out.shape) == (B, Co, Tout) and out.stride(2) == 1
    if _convt_tap_eligible(x, stride, Tout):
        packed, chunk = convt_tap_packed(w, stride, pad, cache)
        _with_ws(x.device, lambda wp, wn: N.lib.a2m_convt1d_tap_fwd_f32(
            _p(x), x.stride(0), x.stride(1), B, Ci, Tin, _p(packed), chunk, _p(b), Co, ks, stride, pad,
            out_pad, *_bn_args(bn), act, slope, _p(out), out.stride(0), out.stride(1), wp, wn, _stream()))
        return out
    packed = convt_packed(w, stride, pad, cache)
    _with_ws(x.device, lambda wp, wn: N.lib.a2m_convt1d_packed_fwd_f32(
        _p(x), x.stride(0), x.stride(1), B, Ci, Tin, _p(packed), _p(b), Co, ks, stride, pad, out_pad,
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


def conv2d_nhwc_packed(w, cache=None):
    """[Co][kh][kw][Ci] conv2d weights (a2m_conv2d_pack_nhwc_f32), cached per weight version."""
    key = _wkey((w,))
    if cache is not None and cache.get('key') == key:
        return cache['w']
    Co, Ci, kh, kw = w.shape
    packed = torch.empty(Co * kh * kw * Ci, device=w.device)
    N.check(N.lib.a2m_conv2d_pack_nhwc_f32(_p(w), Co, Ci, kh, kw, _p(packed), _stream()))
    if cache is not None:
        cache.update(key=key, w=packed)
    return packed


def conv2d_nhwc(x, w, b=None, stride=1, pad=(0, 0), bn=None, act=ACT_NONE, slope=0.2, cols=None,
                out_nhwc=True, cache=None):
    """Channels-last conv2d: x contiguous NHWC [B, H, W, Ci], w [Co, Ci, kh, kw] (packed and
    cached in `cache`); returns NHWC [B, Ho, Wo, Co] (or NCHW with out_nhwc=False) with only
    the output columns cols = (lo, hi) computed."""
    _check_dev(x, w, b)
    assert x.is_contiguous() and w.is_contiguous()
    B, H, W, Ci = x.shape
    Co, _, kh, kw = w.shape
    ph, pw = pad
    Ho, Wo = (H + 2 * ph - kh) // stride + 1, (W + 2 * pw - kw) // stride + 1
    lo, hi = cols if cols is not None else (0, Wo)
    packed = conv2d_nhwc_packed(w, cache)
    out = torch.empty((B, Ho, Wo, Co) if out_nhwc else (B, Co, Ho, Wo), device=x.device, dtype=x.dtype)
    _with_ws(x.device, lambda wp, wn: N.lib.a2m_conv2d_nhwc_fwd_f32(
        _p(x), B, Ci, H, W, _p(packed), _p(b), Co, kh, kw, stride, ph, pw, *_bn_args(bn), act,
        slope, _p(out), int(out_nhwc), Ho, Wo, lo, hi, wp, wn, _stream()))
    return out


def conv2d_nhwc_interp(x, w, b, stride, pad, T, col, bn=None, act=ACT_NONE, slope=0.2, cache=None, out=None):
    """The encoder's last conv restricted to its one live output column `col`, with the
    bilinear time resample to T fused into the GEMM's reduce: [B, Co, T], equal bit for bit to
    interp_time(conv2d_nhwc(..., cols=(col, col + 1), out_nhwc=False), T)."""
    _check_dev(x, w, b, out)
    assert x.is_contiguous() and w.is_contiguous()
    B, H, W, Ci = x.shape
    Co, _, kh, kw = w.shape
    ph, pw = pad
    Ho, Wo = (H + 2 * ph - kh) // stride + 1, (W + 2 * pw - kw) // stride + 1
    packed = conv2d_nhwc_packed(w, cache)
    if out is None:
        out = torch.empty(B, Co, T, device=x.device, dtype=x.dtype)
    assert out.is_contiguous() and tuple(out.shape) == (B, Co, T)
    _with_ws(x.device, lambda wp, wn: N.lib.a2m_conv2d_nhwc_interp_fwd_f32(
        _p(x), B, Ci, H, W, _p(packed), _p(b), Co, kh, kw, stride, ph, pw, *_bn_args(bn), act,
        slope, _p(out), T, Ho, Wo, col, wp, wn, _stream()))
    return out


def bct_to_btc(x, out=None):
    """[B, C, T] (channel stride T) -> [B, T, C] contiguous (a2m_bct_to_btc_f32, T <= 64)."""
    _check_dev(x, out)
    B, C, T = x.shape
    assert x.stride(2) == 1 and x.stride(1) == T
    if out is None:
        out = torch.empty(B, T, C, device=x.device, dtype=x.dtype)
    assert out.is_contiguous() and tuple(out.shape) == (B, T, C)
    N.check(N.lib.a2m_bct_to_btc_f32(_p(x), x.stride(0), B, C, T, _p(out), _stream()))
    return out


def interp_time(x, T, out=None):
    _check_dev(x)
    assert x.is_contiguous()
    B, C, H, W = x.shape
    if out is None:
        out = torch.empty(B, C, T, device=x.device, dtype=x.dtype)
    N.check(N.lib.a2m_interp_time_f32(_p(x), B, C, H, W, _p(out), T, _stream()))
    return out


def mean_time(x, out=None, scale=1.0):
    """out[b, c] = scale * mean_t x[b, c, t]."""
    _check_dev(x, out)
    B, C, T = x.shape
    assert x.stride(2) == 1
    if out is None:
        out = torch.empty(B, C, device=x.device)
    N.check(N.lib.a2m_mean_time_f32(_p(x), x.stride(0), x.stride(1), B, C, T, scale, _p(out), _stream()))
    return out


def repeat_time(x, out, scale=1.0):
    """out[b, c, t] = scale * x[b, c] for a [B, C, T] (t-contiguous) view `out`."""
    _check_dev(x, out)
    B, C, T = out.shape
    assert x.is_contiguous() and tuple(x.shape) == (B, C) and out.stride(2) == 1
    N.check(N.lib.a2m_repeat_time_f32(_p(x), B, C, T, scale, _p(out), out.stride(0), out.stride(1),
                                      _stream()))
    return out


# ------------------------------------------------------------------------- attention
# Derived weight layouts (stacked QKV, phase-packed convT) are cached under
# (epoch, data_ptr, _version) keys.  Parameters written outside torch's version counters --
# FlatAdam's HIP update, or any in-place write through `p.data` (p.data.copy_, an EMA) --
# must call bump_weights_epoch(); FlatAdam.step() does, and every module that caches bumps it
# from a load_state_dict post-hook.  torch.optim updates and p.copy_() under no_grad bump
# the parameter's own _version and need nothing.
WEIGHTS_EPOCH = [0]


def bump_weights_epoch(*_):
    WEIGHTS_EPOCH[0] += 1


def _wkey(ts):
    return (WEIGHTS_EPOCH[0],) + tuple(None if t is None else (t.data_ptr(), t._version) for t in ts)


def _adjacent_view(ts, shape):
    """A view of shape `shape` over the tensors `ts` when they lie back to back in one storage
    (each contiguous, in order), else None."""
    t0 = ts[0]
    off = t0.storage_offset()
    for t in ts:
        if not t.is_contiguous() or t.untyped_storage().data_ptr() != t0.untyped_storage().data_ptr() or \
                t.storage_offset() != off:
            return None
        off += t.numel()
    stride = [1] * len(shape)
    for i in range(len(shape) - 2, -1, -1):
        stride[i] = stride[i + 1] * shape[i + 1]
    return torch.as_strided(t0.detach(), shape, stride, t0.storage_offset())


def stacked_qkv(wq, bq, wk, bk, wv, bv, cache=None):
    """[C/4 + C][C] stacked q/k/v weights and [C/4 + C] biases (cached in `cache` if given).
    When the weights (and the biases) already lie back to back in memory -- FlatAdam places a
    SelfAttention's parameters that way (optim.flat_order) -- the stack is a view: no copy launch
    each training step, and a captured graph reads the live weights."""
    C = wq.shape[1]
    w = _adjacent_view((wq, wk, wv), (C // 4 + C, C))
    b = _adjacent_view((bq, bk, bv), (C // 4 + C,)) if w is not None else None
    if w is not None and b is not None:
        return w, b
    key = _wkey((wq, bq, wk, bk, wv, bv))
    if cache is not None and cache.get('key') == key:
        return cache['w'], cache['b']
    w = torch.empty(C // 4 + C, C, device=wq.device)
    b = torch.empty(C // 4 + C, device=wq.device)
    N.check(N.lib.a2m_stack_qkv_f32(_p(wq), _p(bq), _p(wk), _p(bk), _p(wv), _p(bv), C, _p(w), _p(b),
                                    _stream()))
    if cache is not None:
        cache.update(key=key, w=w, b=b)
    return w, b


_ATTN_EVAL_FUSED = True
# bf16 operand mode: the fused eval attention with its projection on the bf16 MFMA
# (False: the engine's bf16 QKV GEMM + the attention core, as in round 4; tests compare the two)
_ATTN_EVAL_BF16 = True
# bf16 mode: the fused eval attention stages a cached bf16 copy of its stacked weights
_ATTN_BF16_WEIGHTS = True


def self_attention(x, wq, bq, wk, bk, wv, bv, gamma, res=None, out=None, save=None, cache=None):
    """SelfAttention forward.  x, res, out: [B, C, T] with t contiguous and channel stride T.
    `save`, if a dict, receives the qkv and attention intermediates; `cache` (a dict owned by
    the module) keeps the stacked QKV weights between calls."""
    _check_dev(x, wq, wk, wv, gamma, res, out)
    B, C, T = x.shape
    assert x.stride(2) == 1 and x.stride(1) == T
    if out is None:
        out = torch.empty(B, C, T, device=x.device, dtype=x.dtype)
    assert out.stride(0) == x.stride(0) and out.stride(1) == T and out.stride(2) == 1
    if res is not None:
        assert res.stride() == out.stride()
    wqkv, bqkv = stacked_qkv(wq, bq, wk, bk, wv, bv, cache)
    if save is None and _ATTN_EVAL_FUSED and N.lib.a2m_self_attention_eval_fits(C, T) and \
            x.stride(0) % 4 == 0 and x.data_ptr() % 16 == 0 and \
            N.lib.a2m_get_gemm_precision() in ((0, 1) if _ATTN_EVAL_BF16 else (0,)):
        # inference: q/k/v projections fused into the attention core, one launch (bf16 mode: the
        # stacked weights' bf16 copy, cached per weight version, when the module keeps a cache)
        wh = None
        if cache is not None and _ATTN_BF16_WEIGHTS and N.lib.a2m_get_gemm_precision() == 1:
            key = _wkey((wq, bq, wk, bk, wv, bv))
            if cache.get('hkey') != key:
                cache.update(hkey=key, wh=to_bf16(wqkv.contiguous()))
            wh = cache['wh']
        N.check(N.lib.a2m_self_attention_eval_ex_f32(_p(x), x.stride(0), B, C, T, _p(wqkv), _p(bqkv), _p(gamma),
                                                     _p(res), _p(out), out.stride(0), _p(wh), _stream()))
        return out
    qkv = torch.empty(B, C // 4 + C, T, device=x.device, dtype=x.dtype)
    attn = torch.empty(B, T, T, device=x.device, dtype=x.dtype)
    _with_ws(x.device, lambda wp, wn: N.lib.a2m_self_attention_packed_fwd_f32(
        _p(x), x.stride(0), B, C, T, _p(wqkv), _p(bqkv), _p(gamma),
        _p(res), _p(out), out.stride(0), _p(qkv), _p(attn), wp, wn, _stream()))
    if save is not None:
        save['qkv'], save['attn'] = qkv, attn
    return out


def self_attention_group(xs, wqkv, bqkv, gamma, outs, res=None):
    """G SelfAttention eval problems in one launch (a2m_self_attention_eval_group_f32): xs / outs
    / res lists of G [B, C, T] views (channel stride T, equal batch strides), wqkv [G, C/4 + C, C],
    bqkv [G, C/4 + C], gamma [G] stacked per problem."""
    x0, y0 = xs[0], outs[0]
    _check_dev(x0, y0, wqkv, bqkv, gamma)
    B, C, T = x0.shape
    assert N.lib.a2m_self_attention_eval_fits(C, T) and N.lib.a2m_get_gemm_precision() == 0
    for t in list(xs) + list(outs) + list(res or []):
        assert tuple(t.shape) == (B, C, T) and t.stride() == x0.stride() and t.stride(1) == T
    assert x0.stride(0) % 4 == 0 and x0.data_ptr() % 16 == 0
    assert wqkv.is_contiguous() and bqkv.is_contiguous() and gamma.is_contiguous()
    N.check(N.lib.a2m_self_attention_eval_group_f32(
        _p(x0), _group_stride(xs), x0.stride(0), len(xs), B, C, T, _p(wqkv), _p(bqkv), _p(gamma),
        _p(res[0]) if res else None, _group_stride(res) if res else 0, _p(y0), _group_stride(outs),
        _stream()))
    return outs


def channel_attention(x, w1, b1, w2, b2, out=None, att=None):
    _check_dev(x, w1, b1, w2, b2, out)
    assert x.is_contiguous()
    B, C, T = x.shape
    if out is None:
        out = torch.empty_like(x)
    if att is None:
        att = torch.empty(B, C, device=x.device)
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


def graph_att_proj(w0, att_src, att_dst, cache=None):
    """[8][64] GAT attention projections (a2m_graph_att_proj_f32), cached per weight version."""
    key = _wkey((w0, att_src, att_dst))
    if cache is not None and cache.get('key') == key:
        return cache['U']
    U = torch.empty(8, 64, device=w0.device)
    N.check(N.lib.a2m_graph_att_proj_f32(_p(w0), _p(att_src), _p(att_dst), _p(U), _stream()))
    if cache is not None:
        cache.update(key=key, U=U)
    return U


def to_bf16(x, out=None):
    """bf16 (RNE) copy of a contiguous fp32 tensor (a2m_to_bf16_f32)."""
    _check_dev(x, out)
    assert x.is_contiguous() and x.dtype == torch.float32
    if out is None:
        out = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
    N.check(N.lib.a2m_to_bf16_f32(_p(x), _p(out), x.numel(), _stream()))
    return out


def graph_weights_bf16(w0, w1, cache):
    """bf16 copies of a graph layer's weights for the bf16 operand mode's fused stack, cached in
    `cache` per weight version (w1 may be None: GAT)."""
    key = _wkey((w0, w1))
    if cache.get('key') != key:
        cache.update(key=key, h0=to_bf16(w0.detach()), h1=None if w1 is None else to_bf16(w1.detach()))
    return cache['h0'], cache['h1']


def graph_stack(x, J, nbr_ptr, nbr_idx, layers, slope=0.2, out=None, wh=None):
    """Fused eval stack of graph layers (a2m_graph_stack_fwd_ex_f32).  x: [F*J, 64] contiguous;
    layers: list of (kind, w0, w1, U, bias, ln_w, ln_b) with U from graph_att_proj for GAT;
    wh: optional per-layer (w0, w1) bf16 copies (graph_weights_bf16) for the bf16 operand mode."""
    _check_dev(x, out)
    assert x.is_contiguous() and x.shape[1] == 64 and x.shape[0] % J == 0 and 0 < len(layers) <= 8
    F = x.shape[0] // J
    if out is None:
        out = torch.empty_like(x)
    n = len(layers)
    ptrs = lambda i: (ctypes.c_void_p * n)(*[_p(L[i]) for L in layers])  # noqa: E731
    kinds = (ctypes.c_int32 * n)(*[L[0] for L in layers])
    hp = [None, None] if wh is None else \
        [(ctypes.c_void_p * n)(*[_p(h[i]) for h in wh]) for i in (0, 1)]
    N.check(N.lib.a2m_graph_stack_fwd_ex_f32(_p(x), F, J, _p(nbr_ptr), _p(nbr_idx), n, kinds,
                                             ptrs(1), ptrs(2), ptrs(3), ptrs(4), ptrs(5), ptrs(6),
                                             hp[0], hp[1], slope, _p(out), _stream()))
    return out


# ------------------------------------------------------------------------- losses
ANGLE_W = (0.7, 0.3)   # compute_comprehensive_angle_loss (real_motion_model.py:449-461)


def pose_losses(gen, real=None, angle_w=ANGLE_W):
    """Returns a [2] tensor: (bone loss or 0 if real is None, angle loss weighted
    angle_w[0] * hand + angle_w[1] * body)."""
    _check_dev(gen, real)
    B, T, Fd = gen.shape
    assert Fd == 104 and gen.stride(2) == 1
    out = torch.empty(2, device=gen.device)  # the final kernel writes both entries
    rs = real.stride() if real is not None else (0, 0, 1)
    if real is not None:
        assert real.stride(2) == 1
    _with_ws(gen.device, lambda wp, wn: N.lib.a2m_pose_losses_w_f32(
        _p(gen), gen.stride(0), gen.stride(1), _p(real), rs[0], rs[1], B, T, angle_w[0], angle_w[1],
        _p(out), wp, wn, _stream()))
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


# =============================================================================== training
DROP_NONE, DROP_BEFORE, DROP_BEFORE_CH, DROP_AFTER = 0, 1, 2, 3


def _bcl(t):
    """(B, C, L, stride_b, stride_c) of a [B, C, ...] tensor whose trailing dims are contiguous."""
    B, C = t.shape[0], t.shape[1]
    L = 1
    for s in t.shape[2:]:
        L *= s
    inner = 1
    for d in range(t.dim() - 1, 1, -1):
        assert t.stride(d) == inner, 'trailing dims must be contiguous'
        inner *= t.shape[d]
    return B, C, L, t.stride(0), t.stride(1)


# SyncBatchNorm: when a process group is set, training BatchNorm all-reduces its
# per-channel statistics (float64 sums) across the group in the forward and backward, so ranks
# normalise over the whole data-parallel batch like the single-device step.  Every rank must
# hold the same number of clips (n_total = world * local count).
_sync_bn_group = None


def set_sync_bn_group(group):
    """Process group for SyncBN (torch.distributed default group: pass `dist.group.WORLD`), or
    None for per-rank statistics (the default).  Returns the previous setting."""
    global _sync_bn_group
    prev, _sync_bn_group = _sync_bn_group, group
    return prev


def _sync_world():
    if _sync_bn_group is None:
        return 0
    if hasattr(_sync_bn_group, 'all_reduce_sum'):   # an in-process group (tests/test_gpu_syncbn.py)
        w = _sync_bn_group.size()
    else:
        import torch.distributed as dist
        w = dist.get_world_size(_sync_bn_group)
    return w if w > 1 else 0


def _allreduce_sum_(t):
    if hasattr(_sync_bn_group, 'all_reduce_sum'):
        _sync_bn_group.all_reduce_sum(t)
        return
    import torch.distributed as dist
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=_sync_bn_group)


def bn_train(x, gamma, beta, rmean, rvar, momentum, eps, p, mode, seed, act, slope=0.2, out=None):
    """Training-mode BatchNorm fused with dropout and activation; updates rmean / rvar."""
    _check_dev(x, gamma, beta, rmean, rvar, out)
    B, C, L, xsb, xsc = _bcl(x)
    if out is None:
        out = torch.empty(x.shape, device=x.device)
    _, _, _, ysb, ysc = _bcl(out)
    mean = torch.empty(C, device=x.device)
    rstd = torch.empty(C, device=x.device)
    world = _sync_world()
    if world:
        sums = torch.empty(C, 2, device=x.device, dtype=torch.float64)
        _with_ws(x.device, lambda wp, wn: N.lib.a2m_bn_sync_stats_f32(
            _p(x), xsb, xsc, B, C, L, p, mode, seed, _p(sums), wp, wn, _stream()))
        _allreduce_sum_(sums)
        N.check(N.lib.a2m_bn_sync_apply_f32(
            _p(x), xsb, xsc, B, C, L, _p(sums), B * L * world, _p(gamma), _p(beta), _p(rmean), _p(rvar),
            momentum, eps, p, mode, seed, act, slope, _p(out), ysb, ysc, _p(mean), _p(rstd), _stream()))
        return out, mean, rstd
    _with_ws(x.device, lambda wp, wn: N.lib.a2m_bn_train_fwd_f32(
        _p(x), xsb, xsc, B, C, L, _p(gamma), _p(beta), _p(rmean), _p(rvar), momentum, eps, p, mode,
        seed, act, slope, _p(out), ysb, ysc, _p(mean), _p(rstd), wp, wn, _stream()))
    return out, mean, rstd


def bn_eval(x, gamma, beta, rmean, rvar, eps, act, slope=0.2, out=None, p=0.0, mode=0, seed=0):
    """Eval-mode BatchNorm (running statistics, not updated) fused with the activation (and the
    caller's dropout, DROP_* mode), for a forward with gradients; returns (out, mean, rstd) for
    bn_eval_bwd."""
    _check_dev(x, gamma, beta, rmean, rvar, out)
    B, C, L, xsb, xsc = _bcl(x)
    if out is None:
        out = torch.empty(x.shape, device=x.device)
    _, _, _, ysb, ysc = _bcl(out)
    mean = torch.empty(C, device=x.device)
    rstd = torch.empty(C, device=x.device)
    N.check(N.lib.a2m_bn_eval_fwd_f32(_p(x), xsb, xsc, B, C, L, _p(gamma), _p(beta), _p(rmean), _p(rvar),
                                      eps, p, mode, seed, act, slope, _p(out), ysb, ysc, _p(mean), _p(rstd),
                                      _stream()))
    return out, mean, rstd


def bn_eval_bwd(dy, x, gamma, beta, mean, rstd, act, slope=0.2, want_bias=True, p=0.0, mode=0, seed=0):
    """Backward of bn_eval: (dx, dgamma, dbeta, dbias) with the statistics held fixed."""
    _check_dev(dy, x)
    B, C, L, xsb, xsc = _bcl(x)
    _, _, _, dsb, dsc = _bcl(dy)
    dx = torch.empty(x.shape, device=x.device)
    dg = torch.empty(C, device=x.device) if gamma is not None else None
    db = torch.empty(C, device=x.device) if beta is not None else None
    dbias = torch.empty(C, device=x.device) if want_bias else None
    _with_ws(x.device, lambda wp, wn: N.lib.a2m_bn_eval_bwd_f32(
        _p(dy), dsb, dsc, _p(x), xsb, xsc, B, C, L, _p(gamma), _p(beta), _p(mean), _p(rstd), p, mode, seed,
        act, slope, _p(dx), _p(dg), _p(db), _p(dbias), wp, wn, _stream()))
    return dx, dg, db, dbias


def bn_train_bwd(dy, x, gamma, beta, mean, rstd, p, mode, seed, act, slope=0.2, want_bias=True):
    _check_dev(dy, x)
    B, C, L, xsb, xsc = _bcl(x)
    _, _, _, dsb, dsc = _bcl(dy)
    dx = torch.empty(x.shape, device=x.device)
    dg = torch.empty(C, device=x.device) if gamma is not None else None
    db = torch.empty(C, device=x.device) if beta is not None else None
    dbias = torch.empty(C, device=x.device) if want_bias else None
    world = _sync_world()
    if world:
        sums = torch.empty(C, 2, device=x.device, dtype=torch.float64)
        _with_ws(x.device, lambda wp, wn: N.lib.a2m_bn_sync_bwd_stats_f32(
            _p(dy), dsb, dsc, _p(x), xsb, xsc, B, C, L, _p(gamma), _p(beta), _p(mean), _p(rstd), p, mode,
            seed, act, slope, _p(sums), _p(dg), _p(db), wp, wn, _stream()))
        _allreduce_sum_(sums)
        _with_ws(x.device, lambda wp, wn: N.lib.a2m_bn_sync_bwd_apply_f32(
            _p(dy), dsb, dsc, _p(x), xsb, xsc, B, C, L, _p(gamma), _p(beta), _p(mean), _p(rstd), p, mode,
            seed, act, slope, _p(sums), B * L * world, _p(dx), _p(dbias), wp, wn, _stream()))
        return dx, dg, db, dbias
    _with_ws(x.device, lambda wp, wn: N.lib.a2m_bn_train_bwd_f32(
        _p(dy), dsb, dsc, _p(x), xsb, xsc, B, C, L, _p(gamma), _p(beta), _p(mean), _p(rstd), p, mode,
        seed, act, slope, _p(dx), _p(dg), _p(db), _p(dbias), wp, wn, _stream()))
    return dx, dg, db, dbias


def _as4d(t):
    return t.unsqueeze(2) if t.dim() == 3 else t


def conv_dgrad(dy, w, x_shape, stride, pad, dx=None, accumulate=False):
    """dX of conv{1,2}d(x, w, stride, pad); dy contiguous [B, Co, (Ho,) Wo]."""
    _check_dev(dy, w, dx)
    dy = dy.contiguous()
    d4 = _as4d(dy)
    w4 = w.unsqueeze(2) if w.dim() == 3 else w
    B, Co, Ho, Wo = d4.shape
    _, Ci, kh, kw = w4.shape
    if len(x_shape) == 3:
        H, W, sh, sw, ph, pw = 1, x_shape[2], 1, stride, 0, pad
    else:
        H, W = x_shape[2], x_shape[3]
        sh = sw = stride
        ph, pw = pad
    if dx is None:
        dx = torch.empty(x_shape, device=dy.device)
    x4 = _as4d(dx)
    _with_ws(dy.device, lambda wp, wn: N.lib.a2m_conv2d_dgrad_f32(
        _p(dy), B, Co, Ho, Wo, _p(w), Ci, H, W, kh, kw, sh, sw, ph, pw, _p(dx), x4.stride(0),
        x4.stride(1), x4.stride(2), x4.stride(3), int(accumulate), wp, wn, _stream()))
    return dx


def conv_wgrad(dy, x, w_shape, stride, pad, dw=None, accumulate=False):
    """dW of conv{1,2}d(x, w, stride, pad); dy contiguous."""
    _check_dev(dy, x, dw)
    dy = dy.contiguous()
    d4, x4 = _as4d(dy), _as4d(x)
    B, Co, Ho, Wo = d4.shape
    _, Ci, H, W = x4.shape
    if len(w_shape) == 3:
        kh, kw, sh, sw, ph, pw = 1, w_shape[2], 1, stride, 0, pad
    else:
        kh, kw = w_shape[2], w_shape[3]
        sh = sw = stride
        ph, pw = pad
    if dw is None:
        dw = torch.empty(w_shape, device=dy.device)
    _with_ws(dy.device, lambda wp, wn: N.lib.a2m_conv2d_wgrad_f32(
        _p(dy), B, Co, Ho, Wo, _p(x), x4.stride(0), x4.stride(1), x4.stride(2), x4.stride(3), Ci, H, W,
        kh, kw, sh, sw, ph, pw, _p(dw), int(accumulate), wp, wn, _stream()))
    return dw


def gemm(M, N, K, A, a_m, a_k, B, b_n, b_k, C, c_m, c_n, N1=1, K1=1, batch=1, a_bs=0, b_bs=0, c_bs=0,
         bias=None, accumulate=False):
    """C[m][n] (+)= sum_k A(m,k) B(n,k) (+bias[m]).  a_k/b_k/b_n/c_n are (outer, inner) stride
    pairs when K1 / N1 > 1 (k = k0*K1 + k1, n = n0*N1 + n1), plain ints otherwise."""
    _check_dev(A, B, C, bias)
    ak0, ak1 = a_k if isinstance(a_k, tuple) else (a_k, 0)
    bk0, bk1 = b_k if isinstance(b_k, tuple) else (b_k, 0)
    bn0, bn1 = b_n if isinstance(b_n, tuple) else (b_n, 0)
    cn0, cn1 = c_n if isinstance(c_n, tuple) else (c_n, 0)
    lib, n_cols = _native_lib, N  # the argument N shadows the module alias
    _with_ws(C.device, lambda wp, wn: lib.a2m_gemm_f32(
        M, n_cols, N1, K, K1, batch, _p(A), a_bs, a_m, ak0, ak1, _p(B), b_bs, bn0, bn1, bk0, bk1, _p(C),
        c_bs, c_m, cn0, cn1, _p(bias), 1.0, int(accumulate), wp, wn, _stream()))
    return C


def sum_bt(x, out=None, accumulate=False):
    """out[c] = sum over (b, t) of x [B, C, T] (t stride arbitrary)."""
    _check_dev(x, out)
    B, C, T = x.shape
    if out is None:
        out = torch.empty(C, device=x.device)
    N.check(N.lib.a2m_sum_bt_f32(_p(x), x.stride(0), x.stride(1), x.stride(2), B, C, T, _p(out),
                                 int(accumulate), _stream()))
    return out


def dropout(x, p, seed, out=None):
    _check_dev(x, out)
    assert x.is_contiguous()
    if out is None:
        out = torch.empty_like(x)
    N.check(N.lib.a2m_dropout_f32(_p(x), x.numel(), p, seed, _p(out), _stream()))
    return out


def layernorm_bwd(dy_bct, x_rows, w, mean, rstd, T):
    _check_dev(dy_bct, x_rows, w, mean, rstd)
    R, D = x_rows.shape
    dx = torch.empty_like(x_rows)
    dw = torch.empty(D, device=x_rows.device)
    db = torch.empty(D, device=x_rows.device)
    s = dy_bct.stride()
    _with_ws(x_rows.device, lambda wp, wn: N.lib.a2m_layernorm_bwd_f32(
        _p(dy_bct), s[0], s[1], s[2], T, _p(x_rows), R, D, _p(w), _p(mean), _p(rstd), _p(dx), _p(dw),
        _p(db), wp, wn, _stream()))
    return dx, dw, db


def self_attention_bwd(dy, x, weights, qkv, attn):
    wq, bq, wk, bk, wv, bv, gamma = weights
    _check_dev(dy, x, qkv, attn)
    B, C, T = x.shape
    dy = dy.contiguous()
    assert x.stride(0) == dy.stride(0) and x.stride(1) == T and x.stride(2) == 1
    dx = torch.empty(B, C, T, device=x.device)
    # one buffer each for the weight and bias gradients: the library then reduces all three
    # projections in one GEMM / one bias pass (train_attn.hip, packed_w / packed_b)
    Cq = wq.shape[0]
    dwcat = torch.empty(2 * Cq + C, C, device=x.device)
    dwq, dwk, dwv = dwcat[:Cq].view_as(wq), dwcat[Cq:2 * Cq].view_as(wk), dwcat[2 * Cq:].view_as(wv)
    if bq is not None and bk is not None and bv is not None:
        dbcat = torch.empty(2 * Cq + C, device=x.device)
        dbq, dbk, dbv = dbcat[:Cq], dbcat[Cq:2 * Cq], dbcat[2 * Cq:]
    else:
        dbq = torch.empty_like(bq) if bq is not None else None
        dbk = torch.empty_like(bk) if bk is not None else None
        dbv = torch.empty_like(bv) if bv is not None else None
    dg = torch.empty(1, device=x.device)
    need = N.lib.a2m_self_attention_bwd_ws_bytes(B, C, T)
    WS.get(x.device, need)
    _with_ws(x.device, lambda wp, wn: N.lib.a2m_self_attention_bwd_f32(
        _p(dy), _p(x), x.stride(0), B, C, T, _p(wq), _p(bq), _p(wk), _p(bk), _p(wv), _p(bv), _p(gamma),
        _p(qkv), _p(attn), _p(dx), _p(dwq), _p(dbq), _p(dwk), _p(dbk), _p(dwv), _p(dbv), _p(dg), wp, wn,
        _stream()))
    return dx, (dwq, dbq, dwk, dbk, dwv, dbv, dg)


def channel_attention_bwd(dy, x, w1, b1, w2, b2):
    _check_dev(dy, x)
    x = x.contiguous()
    dy = dy.contiguous()
    B, C, T = x.shape
    dx = torch.empty_like(x)
    g = [torch.empty_like(t) for t in (w1, b1, w2, b2)]
    _with_ws(x.device, lambda wp, wn: N.lib.a2m_channel_attention_bwd_f32(
        _p(dy), _p(x), B, C, T, _p(w1), _p(b1), w1.shape[0], _p(w2), _p(b2), _p(dx), *[_p(t) for t in g],
        wp, wn, _stream()))
    return dx, g


def graph_layer_bwd(x, dy, J, kind, nbr_ptr, nbr_idx, w0, w1, att_src, att_dst, bias, ln_w, ln_b,
                    slope=0.2, norm_res=True, pre_ln=None):
    """pre_ln: the forward's saved pre-LayerNorm output (graph_layer(..., pre_ln=)); None = the
    backward recomputes it."""
    _check_dev(x, dy, pre_ln)
    dy = dy.contiguous()
    F = x.shape[0] // J
    dx = torch.empty_like(x)
    dw0 = torch.empty_like(w0)
    dw1 = torch.empty_like(w1) if w1 is not None else None
    das = torch.empty_like(att_src) if att_src is not None else None
    dad = torch.empty_like(att_dst) if att_dst is not None else None
    dbias = torch.empty_like(bias)
    dlw = torch.empty_like(ln_w) if norm_res else None
    dlb = torch.empty_like(ln_b) if norm_res else None
    _with_ws(x.device, lambda wp, wn: N.lib.a2m_graph_layer_bwd_saved_f32(
        _p(x), _p(dy), _p(pre_ln), F, J, kind, int(norm_res), _p(nbr_ptr), _p(nbr_idx), _p(w0), _p(w1), _p(att_src),
        _p(att_dst), _p(bias), _p(ln_w), _p(ln_b), slope, _p(dx), _p(dw0), _p(dw1), _p(das), _p(dad),
        _p(dbias), _p(dlw), _p(dlb), wp, wn, _stream()))
    return dx, dw0, dw1, das, dad, dbias, dlw, dlb


def interp_time_bwd(dy, H, W):
    _check_dev(dy)
    dy = dy.contiguous()
    B, C, T = dy.shape
    dx = torch.empty(B, C, H, W, device=dy.device)
    N.check(N.lib.a2m_interp_time_bwd_f32(_p(dy), B, C, H, W, _p(dx), T, _stream()))
    return dx


def pose_losses_bwd(gen, real, grad_out, dgen, angle_w=ANGLE_W):
    _check_dev(gen, real, grad_out, dgen)
    B, T, _ = gen.shape
    rs = real.stride() if real is not None else (0, 0, 1)
    _with_ws(gen.device, lambda wp, wn: N.lib.a2m_pose_losses_w_bwd_f32(
        _p(gen), gen.stride(0), gen.stride(1), _p(real), rs[0], rs[1], B, T, angle_w[0], angle_w[1],
        _p(grad_out.contiguous()), _p(dgen), wp, wn, _stream()))
    return dgen


def motion_losses(fake, real, grad_terms=None):
    """terms = [L1(motion), smoothness, jerk] (version5_model_train.py:216-248); with
    grad_terms (device [3]) also dfake = sum_i grad_terms[i] dterms[i]/dfake."""
    _check_dev(fake, real, grad_terms)
    fake = fake.contiguous()
    real = real.contiguous() if real is not None else None
    B, T, Fd = fake.shape
    terms = torch.empty(3, device=fake.device)
    dfake = torch.empty_like(fake) if grad_terms is not None else None
    gt = grad_terms.contiguous() if grad_terms is not None else None
    _with_ws(fake.device, lambda wp, wn: N.lib.a2m_motion_losses_f32(
        _p(fake), _p(real), B, T, Fd, _p(terms), _p(gt), _p(dfake), wp, wn, _stream()))
    return terms, dfake


def mse_loss(pred, target, grad_loss=None, want_grad=False):
    """loss = mean (pred - target)^2; dpred = grad_loss * 2 (pred - target) / n if wanted."""
    _check_dev(pred, target, grad_loss)
    pred, target = pred.contiguous(), target.contiguous()
    loss = torch.empty((), device=pred.device)
    d = torch.empty_like(pred) if (want_grad or grad_loss is not None) else None
    _with_ws(pred.device, lambda wp, wn: N.lib.a2m_mse_loss_f32(
        _p(pred), _p(target), pred.numel(), _p(loss), _p(grad_loss), _p(d), wp, wn, _stream()))
    return loss, d


def diff_time(x):
    _check_dev(x)
    x = x.contiguous()
    B, T, Fd = x.shape
    y = torch.empty(B, T - 1, Fd, device=x.device)
    N.check(N.lib.a2m_diff_time_f32(_p(x), B, T, Fd, _p(y), _stream()))
    return y


def diff_time_bwd(dy, dx=None, accumulate=False):
    _check_dev(dy, dx)
    dy = dy.contiguous()
    B, T1, Fd = dy.shape
    if dx is None:
        dx = torch.empty(B, T1 + 1, Fd, device=dy.device)
    N.check(N.lib.a2m_diff_time_bwd_f32(_p(dy), B, T1 + 1, Fd, _p(dx), int(accumulate), _stream()))
    return dx


def gather_segments_(dst, segments):
    """dst[off:off + t.numel()] = t.reshape(-1) for every (off, t) in segments (contiguous fp32
    device tensors), 48 segments per launch (a2m_gather_segments_f32)."""
    if not segments:
        return dst
    _check_dev(dst, *[t for _, t in segments])
    assert dst.is_contiguous() and all(t.is_contiguous() and t.dtype == torch.float32 for _, t in segments)
    k = len(segments)
    src = (ctypes.c_void_p * k)(*[t.data_ptr() for _, t in segments])
    off = (ctypes.c_int64 * k)(*[o for o, _ in segments])
    n = (ctypes.c_int64 * k)(*[t.numel() for _, t in segments])
    N.check(N.lib.a2m_gather_segments_f32(src, off, n, k, _p(dst), _stream()))
    return dst


def set_dropout_seed_offset(counter):
    """Register a device uint64 counter (int64 tensor of one element) whose value offsets every
    dropout seed of the launches issued while it is registered (a2m_set_dropout_seed_offset: a
    graph-replayed training step draws fresh masks); None restores the plain seeds."""
    if counter is not None:
        _check_dev_any(counter)
        assert counter.dtype == torch.int64 and counter.numel() == 1
    N.check(N.lib.a2m_set_dropout_seed_offset(_p(counter)))


def _check_dev_any(*ts):
    for t in ts:
        if not t.is_cuda:
            raise RuntimeError('a2m ops need device tensors (no CPU fallback); got a CPU tensor')


def adam_dev_(param, grad, exp_avg, exp_avg_sq, lr_dev, beta1, beta2, eps, weight_decay, step_dev):
    """Adam with the learning rate (device float32[1]) and step (device int32[1], advanced by one
    here) in device memory: the launch of a graph-captured step (a2m_adam_dev_f32)."""
    _check_dev(param, grad, exp_avg, exp_avg_sq, lr_dev)
    _check_dev_any(step_dev)
    assert step_dev.dtype == torch.int32
    N.check(N.lib.a2m_adam_dev_f32(_p(param), _p(grad), _p(exp_avg), _p(exp_avg_sq), param.numel(), _p(lr_dev),
                                   beta1, beta2, eps, weight_decay, _p(step_dev), _stream()))


def adam_(param, grad, exp_avg, exp_avg_sq, lr, beta1, beta2, eps, weight_decay, step):
    _check_dev(param, grad, exp_avg, exp_avg_sq)
    N.check(N.lib.a2m_adam_f32(_p(param), _p(grad), _p(exp_avg), _p(exp_avg_sq), param.numel(), lr, beta1,
                               beta2, eps, weight_decay, step, _stream()))


class gemm_timing:
    """Context manager: span-stamp timing of every implicit-GEMM launch issued inside it
    (a2m_gemm_timing_begin/_end).  After exit: .launches, .flops, .ms_tile, .ms_reduce,
    .reduces.  With keep=True the records outlive the block: launches captured into a HIP graph
    inside it keep their span stamps, and read() after each replay of that graph returns the
    latest replay's sums (and re-arms the stamps); release() forgets the records."""

    def __init__(self, keep=False):
        self.keep = keep

    def __enter__(self):
        N.check(N.lib.a2m_gemm_timing_begin())
        return self

    def _sums(self, fn):
        import ctypes
        n, r = ctypes.c_int64(), ctypes.c_int64()
        f, mt, mr = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        N.check(fn(ctypes.byref(n), ctypes.byref(f), ctypes.byref(mt), ctypes.byref(mr), ctypes.byref(r)))
        self.launches, self.flops, self.ms_tile = n.value, f.value, mt.value
        self.ms_reduce, self.reduces = mr.value, r.value
        return self

    def read(self):
        """The latest execution's sums (re-arms the stamps); also .ms_queued: the launches'
        times from their ready marks (their stream reaching them) to their last block end."""
        import ctypes
        q = ctypes.c_double()
        self._sums(lambda *a: N.lib.a2m_gemm_timing_read_ex(*a, ctypes.byref(q)))
        self.ms_queued = q.value
        return self

    def spans(self, cap=1024, ready=False):
        """[(start_us, end_us)] of every recorded launch's tile kernel in the latest execution
        ([(ready_us, start_us, end_us)] with ready=True; re-arms the stamps like read())."""
        import ctypes
        r, s, e, n = (ctypes.c_double * cap)(), (ctypes.c_double * cap)(), (ctypes.c_double * cap)(), ctypes.c_int64()
        N.check(N.lib.a2m_gemm_timing_read_spans_ex(cap, r, s, e, ctypes.byref(n)))
        if ready:
            return [(r[i], s[i], e[i]) for i in range(n.value)]
        return [(s[i], e[i]) for i in range(n.value)]

    def release(self):
        N.check(N.lib.a2m_gemm_timing_clear())

    def __exit__(self, *exc):
        if self.keep:
            N.check(N.lib.a2m_gemm_timing_stop())
        else:
            self._sums(N.lib.a2m_gemm_timing_end)
        return False


def timing_mark_to_launch_end(slot, rec):
    """ms from mark `slot` to the last block end of engine launch record `rec` (its tile kernel
    or split-K reduce) in the latest execution of the kept timing window (no re-arm)."""
    import ctypes
    ms = ctypes.c_float()
    N.check(N.lib.a2m_timing_mark_to_launch_end(int(slot), int(rec), ctypes.byref(ms)))
    return ms.value


def timing_mark(slot):
    """Store the GPU wall clock into mark `slot` from a one-thread kernel on the current stream
    (a node of the graph when capturing; needs gemm_timing to have been entered once)."""
    N.check(N.lib.a2m_timing_mark(int(slot), _stream()))


def timing_mark_elapsed(a, b):
    """ms from mark a to mark b (synchronises the device)."""
    import ctypes
    ms = ctypes.c_float()
    N.check(N.lib.a2m_timing_mark_elapsed(int(a), int(b), ctypes.byref(ms)))
    return ms.value
