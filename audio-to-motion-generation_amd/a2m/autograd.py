"""Training-mode path: torch.autograd.Functions whose forward and backward both run in
liba2m_hip.so.  PyTorch's autograd only records the graph and sums gradients of tensors
used twice; skip concatenations / transposes between ops are torch views and copies.

Semantics follow the reference modules in training mode:
  ConvNormRelu   conv -> Dropout(2d) -> BatchNorm(batch stats, running stats updated) -> act
  D blocks       conv -> BatchNorm -> LeakyReLU -> Dropout          (real_motion_model.py:504-551)
  GNN stack      proj_in -> 5 x {layer, LN, LeakyReLU, +res} -> Dropout -> proj_out -> LN
Dropout masks are a counter-based hash of (seed, element); every call draws a fresh seed
from a2m.autograd.next_seed() (seeded from torch.initial_seed(), or manual_seed()).
BatchNorm in eval mode with gradients enabled normalises with the running statistics (fixed in
the backward), as nn.BatchNorm*d.eval() does.
"""

import torch

from . import functional as F

_MASK64 = (1 << 64) - 1
_seed = {'base': None, 'n': 0}


def manual_seed(s):
    _seed['base'] = (s * 0x9E3779B97F4A7C15) & _MASK64
    _seed['n'] = 0


def next_seed():
    if _seed['base'] is None:
        manual_seed(torch.initial_seed())
    _seed['n'] += 1
    return (_seed['base'] + _seed['n'] * 0xD1B54A32D192ED03) & _MASK64


def _need(ctx, i):
    return ctx.needs_input_grad[i]


# ------------------------------------------------------------------------------ convolutions
class _ConvBNAct(torch.autograd.Function):
    """conv{1,2}d + training BatchNorm (+ dropout before / after) + activation."""

    @staticmethod
    def forward(ctx, x, w, b, gamma, beta, cfg):
        if cfg['two_d']:
            raw = F.conv2d(x.contiguous(), w, b, cfg['stride'], cfg['pad'])
        else:
            raw = F.conv1d(x, w, b, cfg['stride'], cfg['pad'])
        out, mean, rstd = _bn_fwd(raw, gamma, beta, cfg, cfg['p'], cfg['mode'], cfg['seed'], cfg['act'],
                                  cfg['slope'])
        ctx.save_for_backward(x, w, raw, gamma, beta, mean, rstd)
        ctx.cfg = cfg
        ctx.has_bias = b is not None
        return out

    @staticmethod
    def backward(ctx, dout):
        x, w, raw, gamma, beta, mean, rstd = ctx.saved_tensors
        c = ctx.cfg
        draw, dg, db, dbias = _bn_bwd(dout.contiguous(), raw, gamma, beta, mean, rstd, c, c['p'], c['mode'],
                                      c['seed'], c['act'], c['slope'], ctx.has_bias)
        dx = F.conv_dgrad(draw, w, x.shape, c['stride'], c['pad']) if _need(ctx, 0) else None
        dw = F.conv_wgrad(draw, x, w.shape, c['stride'], c['pad']) if _need(ctx, 1) else None
        return dx, dw, dbias, dg, db, None


# BatchNorm's num_batches_tracked += 1 is one tiny int64 kernel per layer per forward (~150 an
# iteration); inside a whole-model forward the increments are deferred and applied in one
# multi-tensor launch at its end (torch._foreach_add_).
_NBT = {'defer': 0, 'pending': []}


def _count_batch(norm):
    t = norm.num_batches_tracked
    if t is None:
        return
    if _NBT['defer']:
        _NBT['pending'].append(t)
    else:
        t.add_(1)


class _deferred_batch_counters:
    def __enter__(self):
        _NBT['defer'] += 1

    def __exit__(self, *exc):
        _NBT['defer'] -= 1
        if _NBT['defer'] == 0 and _NBT['pending']:
            with torch.no_grad():
                torch._foreach_add_(_NBT['pending'], 1)
            _NBT['pending'].clear()
        return False


def _bn_fwd(raw, gamma, beta, cfg, p, mode, seed, act, slope):
    """BatchNorm (+ dropout) + activation of a conv output: batch statistics in training mode,
    the running statistics (fixed, not updated) in eval mode; dropout follows its own module."""
    if cfg['eval']:
        return F.bn_eval(raw, gamma, beta, cfg['rm'], cfg['rv'], cfg['eps'], act, slope, p=p, mode=mode,
                         seed=seed)
    return F.bn_train(raw, gamma, beta, cfg['rm'], cfg['rv'], cfg['momentum'], cfg['eps'], p, mode, seed, act,
                      slope)


def _bn_bwd(dout, raw, gamma, beta, mean, rstd, cfg, p, mode, seed, act, slope, want_bias):
    if cfg['eval']:
        return F.bn_eval_bwd(dout, raw, gamma, beta, mean, rstd, act, slope, want_bias=want_bias, p=p, mode=mode,
                             seed=seed)
    return F.bn_train_bwd(dout, raw, gamma, beta, mean, rstd, p, mode, seed, act, slope, want_bias=want_bias)


def _bn_cfg(norm, two_d, stride, pad, p, mode, act):
    """Per-call BatchNorm settings.  A norm in eval mode with gradients (e.g. attribution or
    fine-tuning through a frozen G) normalises with its running statistics, as nn.BatchNorm*d
    does in eval mode: no statistics update, no batch counter.  Dropout (p, mode) is the
    caller's, chosen from the Dropout module's own training flag, so freezing only the norms
    (bn.eval(), dropout left in training mode) still drops, as in the reference."""
    seed = next_seed() if p > 0 else 0
    if not norm.training:
        return dict(two_d=two_d, stride=stride, pad=pad, rm=norm.running_mean, rv=norm.running_var,
                    momentum=0.0, eps=norm.eps, p=p, mode=mode if p > 0 else F.DROP_NONE, seed=seed,
                    act=act, slope=0.2, eval=True)
    _count_batch(norm)
    return dict(two_d=two_d, stride=stride, pad=pad, rm=norm.running_mean, rv=norm.running_var,
                momentum=norm.momentum if norm.momentum is not None else 0.1, eps=norm.eps, p=p,
                mode=mode, seed=seed, act=act, slope=0.2, eval=False)


def conv_norm_act(m, x, out=None):
    k, s, p = m.geometry()
    two_d = m.type == '2d'
    drop = m.dropout.p if m.dropout.training else 0.0
    mode = (F.DROP_BEFORE_CH if two_d else F.DROP_BEFORE) if drop > 0 else F.DROP_NONE
    cfg = _bn_cfg(m.norm, two_d, s, tuple(p) if two_d else p, drop, mode, m.act)
    y = _ConvBNAct.apply(x, m.conv.weight, m.conv.bias, m.norm.weight, m.norm.bias, cfg)
    if out is not None:
        out.copy_(y)
        return out
    return y


def d_block(conv, bn, drop, x):
    """Discriminator block: Conv1d -> BatchNorm1d -> LeakyReLU(0.2) -> Dropout."""
    p = drop.p if drop.training else 0.0
    cfg = _bn_cfg(bn, False, conv.stride[0], conv.padding[0], p, F.DROP_AFTER if p > 0 else F.DROP_NONE,
                  F.ACT_LRELU)
    return _ConvBNAct.apply(x, conv.weight, conv.bias, bn.weight, bn.bias, cfg)


class _ConvTBN(torch.autograd.Function):
    """ConvTranspose1d + training BatchNorm + ReLU (ConvTranspose1D, model_layers.py:193-215)."""

    @staticmethod
    def forward(ctx, x, w, b, gamma, beta, cfg):
        raw = F.convt1d(x.contiguous(), w, b, cfg['stride'], cfg['pad'], cfg['out_pad'])
        out, mean, rstd = _bn_fwd(raw, gamma, beta, cfg, 0.0, F.DROP_NONE, 0, F.ACT_RELU, 0.2)
        ctx.save_for_backward(x, w, raw, gamma, beta, mean, rstd)
        ctx.cfg = cfg
        ctx.has_bias = b is not None
        return out

    @staticmethod
    def backward(ctx, dout):
        x, w, raw, gamma, beta, mean, rstd = ctx.saved_tensors
        c = ctx.cfg
        draw, dg, db, dbias = _bn_bwd(dout.contiguous(), raw, gamma, beta, mean, rstd, c, 0.0, F.DROP_NONE, 0,
                                      F.ACT_RELU, 0.2, ctx.has_bias)
        # ConvTranspose1d's dgrad is a plain conv with its own [Ci][Co][k] weight; its wgrad is
        # the conv wgrad with the operand roles exchanged.
        dx = F.conv1d(draw, w, None, c['stride'], c['pad']) if _need(ctx, 0) else None
        dw = F.conv_wgrad(x.contiguous(), draw, w.shape, c['stride'], c['pad']) if _need(ctx, 1) else None
        return dx, dw, dbias, dg, db, None


def convt_bn_relu(m, x, out=None):
    c, n = m.conv_transpose, m.bn
    cfg = _bn_cfg(n, False, c.stride[0], c.padding[0], 0.0, F.DROP_NONE, F.ACT_RELU)
    cfg['out_pad'] = c.output_padding[0]
    y = _ConvTBN.apply(x, c.weight, c.bias, n.weight, n.bias, cfg)
    if out is not None:
        out.copy_(y)
        return out
    return y


class _Conv1d(torch.autograd.Function):
    """Plain Conv1d with bias (final 1x1 convs, logits)."""

    @staticmethod
    def forward(ctx, x, w, b, stride, pad):
        y = F.conv1d(x, w, b, stride, pad)
        ctx.save_for_backward(x, w)
        ctx.sp = (stride, pad)
        ctx.has_bias = b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        s, p = ctx.sp
        dy = dy.contiguous()
        dx = F.conv_dgrad(dy, w, x.shape, s, p) if _need(ctx, 0) else None
        dw = F.conv_wgrad(dy, x, w.shape, s, p) if _need(ctx, 1) else None
        db = F.sum_bt(dy) if ctx.has_bias and _need(ctx, 2) else None
        return dx, dw, db, None, None


def conv1d(x, w, b=None, stride=1, pad=0):
    return _Conv1d.apply(x, w, b, stride, pad)


class _Linear(torch.autograd.Function):
    """y = x W^T + b on contiguous rows [R, I]."""

    @staticmethod
    def forward(ctx, x, w, b):
        x = x.contiguous()
        y = F.linear(x, w, b)
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous()
        R, I = x.shape
        O = w.shape[0]
        dx = dw = db = None
        if _need(ctx, 0):
            dx = torch.empty(R, I, device=x.device)
            F.gemm(I, R, O, w, 1, I, dy, O, 1, dx, 1, I)
        if _need(ctx, 1):
            dw = torch.empty(O, I, device=x.device)
            F.gemm(O, I, R, dy, 1, O, x, 1, I, dw, I, 1)
        if ctx.has_bias and _need(ctx, 2):
            db = F.sum_bt(dy.t().unsqueeze(0))
        return dx, dw, db


def linear(x, w, b=None):
    return _Linear.apply(x, w, b)


class _ProjIn(torch.autograd.Function):
    """Linear over channels of x [B, C, T] -> rows [B*T, O] (decoder proj_in, fused permute)."""

    @staticmethod
    def forward(ctx, x, w, b):
        B, C, T = x.shape
        O = w.shape[0]
        h = torch.empty(B, T, O, device=x.device)
        F.conv1d(x, w, b, out=h.permute(0, 2, 1))
        ctx.save_for_backward(x, w)
        return h.view(B * T, O)

    @staticmethod
    def backward(ctx, dh):
        x, w = ctx.saved_tensors
        B, C, T = x.shape
        O = w.shape[0]
        dh = dh.contiguous()
        dx = torch.empty(B, C, T, device=x.device)
        # dx[b][c][t] = sum_o W[o][c] dh[(b,t)][o]
        F.gemm(C, B * T, O, w, 1, C, dh, (T * O, O), 1, dx, T, (C * T, 1), N1=T)
        dw = torch.empty(O, C, device=x.device)
        # dW[o][c] = sum_{b,t} dh[(b,t)][o] x[b][c][t]
        F.gemm(O, C, B * T, dh, 1, (T * O, O), x, x.stride(1), (x.stride(0), x.stride(2)), dw, C, 1, K1=T)
        db = F.sum_bt(dh.t().unsqueeze(0))
        return dx, dw, db


class _LayerNormBCT(torch.autograd.Function):
    """LayerNorm over rows [B*T, D] written as [B, D, T] (decoder norm + permute)."""

    @staticmethod
    def forward(ctx, rows, w, b, T):
        stats = {}
        out = F.layernorm_to_bct(rows.contiguous(), w, b, T, stats=stats)
        ctx.save_for_backward(rows, w, stats['mean'], stats['rstd'])
        ctx.T = T
        return out

    @staticmethod
    def backward(ctx, dout):
        rows, w, mean, rstd = ctx.saved_tensors
        dx, dw, db = F.layernorm_bwd(dout, rows.contiguous(), w, mean, rstd, ctx.T)
        return dx, dw, db, None




class _GraphLayer(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w0, w1, att_src, att_dst, bias, ln_w, ln_b, topo):
        J, kind, ptr, idx, norm_res, grads = topo
        x = x.contiguous()
        # the pre-LayerNorm copy only when a backward will read it (not under no_grad, nor when no
        # input needs a gradient: e.g. a validation forward in train mode)
        pre = torch.empty_like(x) if norm_res and grads else None
        y = F.graph_layer(x, J, kind, ptr, idx, w0, w1, att_src, att_dst, bias, ln_w, ln_b,
                          norm_res=norm_res, pre_ln=pre)
        ctx.save_for_backward(x, w0, w1, att_src, att_dst, bias, ln_w, ln_b, pre)
        ctx.topo = topo
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w0, w1, att_src, att_dst, bias, ln_w, ln_b, pre = ctx.saved_tensors
        J, kind, ptr, idx, norm_res, _ = ctx.topo
        dx, dw0, dw1, das, dad, dbias, dlw, dlb = F.graph_layer_bwd(
            x, dy, J, kind, ptr, idx, w0, w1, att_src, att_dst, bias, ln_w, ln_b,
            norm_res=norm_res, pre_ln=pre)
        return dx, dw0, dw1, das, dad, dbias, dlw, dlb, None


def _grads_wanted(*ts):
    return torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in ts)


def gat(g, x, J, ptr, idx, ln=None):
    lw, lb = (ln.weight, ln.bias) if ln is not None else (None, None)
    return _GraphLayer.apply(x, g.lin.weight, None, g.att_src, g.att_dst, g.bias, lw, lb,
                             (J, 0, ptr, idx, ln is not None,
                              _grads_wanted(x, g.lin.weight, g.att_src, g.att_dst, g.bias, lw, lb)))


def graph_conv(g, x, J, ptr, idx, ln):
    return _GraphLayer.apply(x, g.lin_rel.weight, g.lin_root.weight, None, None, g.lin_rel.bias,
                             ln.weight, ln.bias,
                             (J, 1, ptr, idx, True, _grads_wanted(x, g.lin_rel.weight, g.lin_root.weight,
                                                                  g.lin_rel.bias, ln.weight, ln.bias)))


class _Dropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, seed):
        ctx.ps = (p, seed)
        return F.dropout(x.contiguous(), p, seed)

    @staticmethod
    def backward(ctx, dy):
        p, seed = ctx.ps
        return F.dropout(dy.contiguous(), p, seed), None, None


def dropout(mod, x):
    if not mod.training or mod.p == 0:
        return x
    return _Dropout.apply(x, mod.p, next_seed())


# ------------------------------------------------------------------------------ attention
class _SelfAttn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, res, wq, bq, wk, bk, wv, bv, gamma):
        x = x.contiguous()
        save = {}
        y = F.self_attention(x, wq, bq, wk, bk, wv, bv, gamma,
                             res=res.contiguous() if res is not None else None, save=save)
        ctx.save_for_backward(x, save['qkv'], save['attn'], wq, bq, wk, bk, wv, bv, gamma)
        ctx.has_res = res is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, qkv, attn, wq, bq, wk, bk, wv, bv, gamma = ctx.saved_tensors
        dy = dy.contiguous()
        dx, (dwq, dbq, dwk, dbk, dwv, dbv, dg) = F.self_attention_bwd(dy, x, (wq, bq, wk, bk, wv, bv, gamma),
                                                                       qkv, attn)
        return dx, (dy if ctx.has_res else None), dwq, dbq, dwk, dbk, dwv, dbv, dg


def self_attention(m, x, res=None, out=None):
    y = _SelfAttn.apply(x, res, *m.weights())
    if out is not None:
        out.copy_(y)
        return out
    return y


class _ChanAttn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2):
        x = x.contiguous()
        ctx.save_for_backward(x, w1, b1, w2, b2)
        return F.channel_attention(x, w1, b1, w2, b2)

    @staticmethod
    def backward(ctx, dy):
        x, w1, b1, w2, b2 = ctx.saved_tensors
        dx, g = F.channel_attention_bwd(dy, x, w1, b1, w2, b2)
        return (dx, *g)


def channel_attention(m, x):
    return _ChanAttn.apply(x, *m.weights())


# ------------------------------------------------------------------------------ plumbing
class _InterpTime(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, T):
        ctx.hw = x.shape[2:]
        return F.interp_time(x.contiguous(), T)

    @staticmethod
    def backward(ctx, dy):
        H, W = ctx.hw
        return F.interp_time_bwd(dy, H, W), None


class _MeanTime(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.T = x.shape[2]
        return F.mean_time(x)

    @staticmethod
    def backward(ctx, dy):
        B, C = dy.shape
        dx = torch.empty(B, C, ctx.T, device=dy.device)
        return F.repeat_time(dy.contiguous(), dx, scale=1.0 / ctx.T)


class _RepeatTime(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, T):
        B, C = x.shape
        out = torch.empty(B, C, T, device=x.device)
        return F.repeat_time(x.contiguous(), out)

    @staticmethod
    def backward(ctx, dy):
        T = dy.shape[2]
        return F.mean_time(dy.contiguous(), scale=float(T)), None


class _Diff(torch.autograd.Function):
    """pos_to_motion: torch.diff(x, dim=1) (version5_model_train.py:208-213)."""

    @staticmethod
    def forward(ctx, x):
        return F.diff_time(x)

    @staticmethod
    def backward(ctx, dy):
        return F.diff_time_bwd(dy)


def pos_to_motion(x):
    return _Diff.apply(x)


class _PoseLosses(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gen, real, angle_w=F.ANGLE_W):
        gen = gen.contiguous()
        ctx.save_for_backward(gen, real)
        ctx.angle_w = angle_w
        return F.pose_losses(gen, real, angle_w)

    @staticmethod
    def backward(ctx, dl):
        gen, real = ctx.saved_tensors
        dgen = torch.zeros_like(gen)
        F.pose_losses_bwd(gen, real, dl.contiguous(), dgen, ctx.angle_w)
        return dgen, None, None


def _no_real_grad(real, what):
    """The backward kernels produce d/d(generated pose) only.  The reference's losses are also
    differentiable in the real pose, which its training loop never asks for (the real pose is
    data); asking for it here is an error rather than a silently missing gradient."""
    if torch.is_grad_enabled() and real is not None and real.requires_grad:
        raise NotImplementedError(f'{what}: gradient with respect to the real pose is not '
                                  f'implemented (detach it)')


def pose_losses(gen, real=None, angle_w=F.ANGLE_W):
    """[bone, angle] with autograd when an input needs it (the plain HIP op otherwise)."""
    _no_real_grad(real, 'pose_losses')
    if torch.is_grad_enabled() and gen.requires_grad:
        return _PoseLosses.apply(gen, real, angle_w)
    return F.pose_losses(gen.contiguous(), real.contiguous() if real is not None else None, angle_w)


class _MotionTerms(torch.autograd.Function):
    """[L1(real motion, fake motion), smoothness, jerk] of a fake pose sequence."""

    @staticmethod
    def forward(ctx, fake, real):
        fake = fake.contiguous()
        ctx.save_for_backward(fake, real)
        terms, _ = F.motion_losses(fake, real)
        return terms

    @staticmethod
    def backward(ctx, dterms):
        fake, real = ctx.saved_tensors
        _, dfake = F.motion_losses(fake, real, grad_terms=dterms)
        return dfake, None


def motion_terms(fake_pose, real_pose):
    _no_real_grad(real_pose, 'motion_terms')
    return _MotionTerms.apply(fake_pose, real_pose)


class _MSE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, target):
        ctx.save_for_backward(pred, target)
        loss, _ = F.mse_loss(pred, target)
        return loss

    @staticmethod
    def backward(ctx, dl):
        pred, target = ctx.saved_tensors
        _, d = F.mse_loss(pred, target, grad_loss=dl.reshape(1).contiguous())
        return d, None


def mse_loss(pred, target):
    return _MSE.apply(pred, target)


# ------------------------------------------------------------------------------ modules
def audio_encoder(enc, x, time_steps):
    h = x.contiguous().unsqueeze(1)
    for layer in enc.conv:
        h = conv_norm_act(layer, h)
    return _InterpTime.apply(h, time_steps)


def unet(u, x):
    d, up = u.downsample_layers, u.upsample_layers
    s1 = d[0](x)
    h = d[1](s1)
    s2 = d[2](h)
    h = d[3](s2)
    h = u.bottleneck_attention(u.bottleneck(h))
    h = up[1](u.up_attention(torch.cat([up[0](h), s2], 1)))
    h = up[3](torch.cat([up[2](h), s1], 1))
    return conv1d(h, u.final_conv.weight, u.final_conv.bias)


def graph_stack(g, part, x):
    B, C, T = x.shape
    nj = getattr(g, f'num_{part}_joints')
    pin, pout = getattr(g, f'{part}_proj_in'), getattr(g, f'{part}_proj_out')
    ptr, idx = g.topology(part)
    lns = getattr(g, f'{part}_layer_norms')
    h = _ProjIn.apply(x, pin.weight, pin.bias).view(B * T * nj, 64)
    for L in range(5):
        layer = getattr(g, f'{part}_gcn{L + 1}')
        h = gat(layer, h, nj, ptr, idx, lns[L]) if L % 2 == 0 else graph_conv(layer, h, nj, ptr, idx, lns[L])
    h = dropout(getattr(g, f'{part}_dropout'), h)
    rows = linear(h.view(B * T, nj * 64), pout.weight, pout.bias)
    nrm = getattr(g, f'{part}_norm')
    return _LayerNormBCT.apply(rows, nrm.weight, nrm.bias, T)


def generator_forward(g, audio, real_pose=None):
    with _deferred_batch_counters():
        return _generator_forward(g, audio, real_pose)


def _generator_forward(g, audio, real_pose=None):
    feats = g.unet(g.audio_encoder(audio))
    outs = []
    for part in ('body', 'hand'):
        x = getattr(g, f'{part}_decoder_pre')(feats)
        x = graph_stack(g, part, x)
        x = getattr(g, f'{part}_decoder_post')(x)
        lg = getattr(g, f'{part}_logits')
        outs.append(conv1d(x, lg.weight, lg.bias))
    out = torch.cat(outs, 1).transpose(1, 2).contiguous()
    losses = _PoseLosses.apply(out, real_pose, F.ANGLE_W)
    internal = [losses[0]] if real_pose is not None else []
    internal.append(losses[1])
    return out, internal


def discriminator_forward(d, x):
    with _deferred_batch_counters():
        return _discriminator_forward(d, x)


def _discriminator_forward(d, x):
    h = x.transpose(-1, -2)
    if h.shape[2] < 4:
        h = torch.nn.functional.pad(h, (0, 4 - h.shape[2] % 4))
    seqs = [d.conv1] + list(d.conv2) + [d.conv3]
    for sq in seqs:
        mods = list(sq)
        i = 0
        while i < len(mods):
            m = mods[i]
            if isinstance(m, torch.nn.Conv1d):
                h = d_block(m, mods[i + 1], mods[i + 3], h)
                i += 4
            else:  # SelfAttention
                h = m(h)
                i += 1
    B, C, T = h.shape
    gs = []
    for k, (part, nj) in enumerate((('body', 10), ('hand', 42))):
        pooled = _MeanTime.apply(h[:, k * C // 2:(k + 1) * C // 2])
        proj = getattr(d, f'{part}_proj')
        z = linear(pooled, proj.weight, proj.bias).view(B * nj, 64)
        ptr, idx = d.topology(part)
        z = gat(getattr(d, f'{part}_gat'), z, nj, ptr, idx, None)
        go = getattr(d, f'{part}_graph_out')
        gs.append(linear(z.view(B, nj * 64), go.weight, go.bias))
    grep = _RepeatTime.apply(torch.cat(gs, 1), T)
    lg = conv1d(torch.cat([h, grep], 1), d.logits.weight, d.logits.bias, 1, 1)
    return lg.transpose(-1, -2).squeeze(-1)
