"""Drop-in layer modules for model_layers.py (the subset on the generator / discriminator
path).  Module names, constructor signatures and state_dict keys follow the reference so
reference checkpoints load unchanged; compute runs in liba2m_hip.so.

  ConvNormRelu     model_layers.py:51-118
  SelfAttention    model_layers.py:121-146
  ChannelAttention model_layers.py:149-174
  ResBlock         model_layers.py:177-190
  ConvTranspose1D  model_layers.py:193-215
  AudioEncoder     model_layers.py:219-280
  UNet1D           model_layers.py:283-374

In eval mode (and under no_grad) every module runs the fused forward kernels (BatchNorm
folded into the GEMM epilogue, zero-copy skip concatenation, dead encoder columns
pruned).  In training mode they run through a2m.autograd, whose Functions pair the same
forward kernels with hand-written HIP backward kernels.
"""
import torch
import torch.nn as nn

from . import functional as F

ACT = {'relu': F.ACT_RELU, 'lrelu': F.ACT_LRELU}


def _grad_path(module, *tensors):
    return module.training or (torch.is_grad_enabled() and (
        any(p.requires_grad for p in module.parameters()) or
        any(t is not None and t.requires_grad for t in tensors)))


def _autograd():
    from . import autograd
    return autograd


_MOVED_WARNED = []


def stage_inputs(module, *tensors):
    """Host-tensor entry for the top-level modules (generate_motion_video.py:257 calls
    `generator(audio)` on CPU tensors with a CPU-constructed generator).  There is no CPU
    compute path: a module whose parameters are still on the host is moved to the current
    GPU once (in place, as `module.cuda()` would), and host inputs are copied to it.  Returns
    (device tensors, the device the caller's first input lives on) so results can be handed
    back there."""
    p = next(module.parameters())
    if not p.is_cuda:
        if not torch.cuda.is_available():
            raise RuntimeError('a2m modules compute on the GPU only (no CPU fallback) and no GPU is visible')
        if not _MOVED_WARNED:
            import warnings
            warnings.warn(f'{type(module).__name__} had its parameters on the host: moved to '
                          f'cuda:{torch.cuda.current_device()} (a2m computes on the GPU only)')
            _MOVED_WARNED.append(True)
        module.cuda()
        p = next(module.parameters())
    home = next((t.device for t in tensors if t is not None), p.device)
    out = tuple(None if t is None else (t if t.device == p.device else t.to(p.device, non_blocking=True))
                for t in tensors)
    return out, home


def to_home(home, *ts):
    """Hand results back on the caller's device (no-op when it is the compute device)."""
    return tuple(t if (t is None or t.device == home) else t.to(home) for t in ts)


class ConvNormRelu(nn.Module):
    def __init__(self, in_channels, out_channels, type='1d', leaky=False, downsample=False,
                 kernel_size=None, stride=None, padding=None, p=0, groups=1):
        super().__init__()
        if groups != 1:
            raise NotImplementedError('grouped ConvNormRelu is not on the hot path')
        if kernel_size is None and stride is None:
            kernel_size, stride = (4, 2) if downsample else (3, 1)
        if padding is None:  # model_layers.py:70-84
            if isinstance(kernel_size, int) and isinstance(stride, tuple):
                padding = tuple(int((kernel_size - s) / 2) for s in stride)
            elif isinstance(kernel_size, tuple) and isinstance(stride, int):
                padding = tuple(int((k - stride) / 2) for k in kernel_size)
            elif isinstance(kernel_size, tuple) and isinstance(stride, tuple):
                padding = tuple(int((k - s) / 2) for k, s in zip(kernel_size, kernel_size))
            else:
                padding = int((kernel_size - stride) / 2)
        self.type = type
        self.leaky = leaky
        self.p = p
        self._tap = {}   # tap-chunked weights for the eval path (functional.conv1d_tap_packed)
        self._nhwc = {}  # [Co][kh][kw][Ci] weights for the channels-last encoder chain
        if type == '1d':
            self.conv = nn.Conv1d(in_channels, out_channels, kernel_size, stride, padding)
            self.norm = nn.BatchNorm1d(out_channels)
            self.dropout = nn.Dropout(p=p)
        else:
            self.conv = nn.Conv2d(in_channels, out_channels, kernel_size, stride, padding)
            self.norm = nn.BatchNorm2d(out_channels)
            self.dropout = nn.Dropout2d(p=p)
        self.relu = nn.LeakyReLU(negative_slope=0.2) if leaky else nn.ReLU()

    @property
    def act(self):
        return F.ACT_LRELU if self.leaky else F.ACT_RELU

    def bn_eval(self):
        n = self.norm
        return (n.weight, n.bias, n.running_mean, n.running_var, n.eps)

    def geometry(self):
        c = self.conv
        k = c.kernel_size if self.type == '2d' else c.kernel_size[0]
        s = c.stride[0]
        p = c.padding if self.type == '2d' else c.padding[0]
        return k, s, p

    def forward(self, x, out=None, cols=None):
        if _grad_path(self, x):
            return _autograd().conv_norm_act(self, x, out=out)
        k, s, p = self.geometry()
        if self.type == '1d':
            return F.conv1d(x, self.conv.weight, self.conv.bias, s, p, bn=self.bn_eval(),
                            act=self.act, out=out, cache=self._tap)
        return F.conv2d(x, self.conv.weight, self.conv.bias, s, tuple(p), bn=self.bn_eval(),
                        act=self.act, cols=cols, out=out)


class SelfAttention(nn.Module):
    def __init__(self, in_channels):
        super().__init__()
        self.query_conv = nn.Conv1d(in_channels, in_channels // 8, kernel_size=1)
        self.key_conv = nn.Conv1d(in_channels, in_channels // 8, kernel_size=1)
        self.value_conv = nn.Conv1d(in_channels, in_channels, kernel_size=1)
        self.gamma = nn.Parameter(torch.zeros(1))
        self._pack = {}   # stacked QKV weights for the eval path (functional.stacked_qkv)
        self.register_load_state_dict_post_hook(F.bump_weights_epoch)

    def weights(self):
        return (self.query_conv.weight, self.query_conv.bias, self.key_conv.weight,
                self.key_conv.bias, self.value_conv.weight, self.value_conv.bias, self.gamma)

    def forward(self, x, res=None, out=None):
        """gamma * softmax-attention(x) + x (+ res): res fuses ResBlock's outer residual."""
        if _grad_path(self, x, res):
            return _autograd().self_attention(self, x, res=res, out=out)
        return F.self_attention(x, *self.weights(), res=res, out=out, cache=self._pack)


class ChannelAttention(nn.Module):
    def __init__(self, channel, reduction=8):
        super().__init__()
        self.avg_pool = nn.AdaptiveAvgPool1d(1)
        self.max_pool = nn.AdaptiveMaxPool1d(1)
        self.fc = nn.Sequential(nn.Linear(channel, channel // reduction), nn.ReLU(inplace=True),
                                nn.Linear(channel // reduction, channel), nn.Sigmoid())

    def weights(self):
        return self.fc[0].weight, self.fc[0].bias, self.fc[2].weight, self.fc[2].bias

    def forward(self, x):
        if _grad_path(self, x):
            return _autograd().channel_attention(self, x)
        return F.channel_attention(x.contiguous(), *self.weights())


class ResBlock(nn.Module):
    def __init__(self, channels, type='1d', p=0.1):
        super().__init__()
        self.conv1 = ConvNormRelu(channels, channels, type=type, leaky=True, p=p)
        self.conv2 = ConvNormRelu(channels, channels, type=type, leaky=True, p=p)
        self.attention = SelfAttention(channels)

    def forward(self, x):
        y = self.conv2(self.conv1(x))
        return self.attention(y, res=x)


class ConvTranspose1D(nn.Module):
    def __init__(self, in_channels, out_channels, kernel_size=3, stride=2, padding=1, output_padding=1):
        super().__init__()
        self.conv_transpose = nn.ConvTranspose1d(in_channels, out_channels, kernel_size, stride,
                                                 padding, output_padding)
        self.bn = nn.BatchNorm1d(out_channels)
        self.relu = nn.ReLU(inplace=True)
        self._pack = {}   # phase-packed weights for the eval path (functional.convt_packed)
        self.register_load_state_dict_post_hook(F.bump_weights_epoch)

    def forward(self, x, out=None):
        if _grad_path(self, x):
            return _autograd().convt_bn_relu(self, x, out=out)
        c, n = self.conv_transpose, self.bn
        return F.convt1d(x, c.weight, c.bias, c.stride[0], c.padding[0], c.output_padding[0],
                         bn=(n.weight, n.bias, n.running_mean, n.running_var, n.eps),
                         act=F.ACT_RELU, out=out, cache=self._pack)


# module flags (measured-slower alternatives stay reachable from tests by flipping them)
_ENC_NHWC = True       # channels-last encoder chain
_ENC_NHWC_ALL = True   # ... for every layer whose Ci is 1 or a multiple of 64
# the last conv + time resample as one GEMM whose reduce writes the resampled output
# (a2m_conv2d_nhwc_interp_fwd_f32); False restores conv + interp_time
_ENC_FUSED_INTERP = True


class AudioEncoder(nn.Module):
    def __init__(self, output_feats=64, input_channels=1, kernel_size=None, stride=None, p=0, groups=1):
        super().__init__()
        self.conv = nn.ModuleList([
            ConvNormRelu(input_channels, 64, type='2d', leaky=True, downsample=True, kernel_size=kernel_size, stride=stride, p=p, groups=groups),
            ConvNormRelu(64, 128, type='2d', leaky=True, downsample=True, kernel_size=kernel_size, stride=stride, p=p, groups=groups),
            ConvNormRelu(128, 256, type='2d', leaky=True, downsample=True, kernel_size=kernel_size, stride=stride, p=p, groups=groups),
            ConvNormRelu(256, 512, type='2d', leaky=True, downsample=False, kernel_size=kernel_size, stride=stride, p=p, groups=groups),
            ConvNormRelu(512, 256, type='2d', leaky=True, downsample=False, kernel_size=(3, 8), stride=1, p=p, groups=groups),
        ])
        self._cols = {}

    def live_columns(self, F_in):
        """Per layer, the output columns [lo, hi) that reach the encoder output.
        interpolate(size=(T,1), align_corners=False) over the last layer's W_out columns samples
        source column W_out/2 - 1/2 (model_layers.py:277); when that is an integer only that one
        column carries weight, and its receptive field is propagated back through every layer
        (71% of the dense encoder work is dead)."""
        if F_in in self._cols:
            return self._cols[F_in]
        widths = [F_in]
        for layer in self.conv:
            k, s, p = layer.geometry()
            widths.append((widths[-1] + 2 * p[1] - k[1]) // s + 1)
        Wl = widths[-1]
        src = max(Wl * 0.5 - 0.5, 0.0)
        lo = int(src)
        hi = lo + 1 if src == lo or lo == Wl - 1 else lo + 2
        cols = [None] * len(self.conv)
        for i in range(len(self.conv) - 1, -1, -1):
            cols[i] = (lo, hi)
            k, s, p = self.conv[i].geometry()
            lo, hi = max(lo * s - p[1], 0), min((hi - 1) * s - p[1] + k[1], widths[i])
        self._cols[F_in] = cols
        return cols

    def forward(self, x, time_steps=None):
        if time_steps is None:
            time_steps = x.shape[-2]
        if _grad_path(self, x):
            return _autograd().audio_encoder(self, x, time_steps)
        return self._eval_chain(x.contiguous(), time_steps)

    def _eval_chain(self, x, time_steps, out=None):
        cols = self.live_columns(x.shape[-1])
        nhwc = [_ENC_NHWC and self._nhwc_layer(i) for i in range(len(self.conv))]
        # the mel [B, T, F] is NHWC with C = 1 and NCHW with the channel unsqueezed, for free
        h = x.unsqueeze(-1 if nhwc[0] else 1)
        for i, (layer, c) in enumerate(zip(self.conv, cols)):
            if nhwc[i] and i + 1 == len(self.conv) and _ENC_FUSED_INTERP and self._single_live_column(h, c):
                # the last conv's one live column straight into the resampled [B, C, T] output
                k, s, p = layer.geometry()
                return F.conv2d_nhwc_interp(h, layer.conv.weight, layer.conv.bias, s, tuple(p), time_steps,
                                            c[0], bn=layer.bn_eval(), act=layer.act, cache=layer._nhwc,
                                            out=out)
            if nhwc[i]:
                k, s, p = layer.geometry()
                out_nhwc = i + 1 < len(self.conv) and nhwc[i + 1]
                h = F.conv2d_nhwc(h, layer.conv.weight, layer.conv.bias, s, tuple(p),
                                  bn=layer.bn_eval(), act=layer.act, cols=c, out_nhwc=out_nhwc,
                                  cache=layer._nhwc)
            else:
                h = layer(h, cols=c)
        return F.interp_time(h, time_steps, out=out)

    def _single_live_column(self, h, c):
        """The last layer's live columns c are one column the resample reads with weight 1
        (its source position Wout/2 - 1/2 is that integer column): the fused path's condition."""
        k, s, p = self.conv[-1].geometry()
        Wo = (h.shape[2] + 2 * p[1] - k[1]) // s + 1
        src = max(Wo * 0.5 - 0.5, 0.0)
        return c[1] - c[0] == 1 and src == c[0]

    def _nhwc_layer(self, i):
        """Channels-last for every layer the GEMM engine can read as contiguous channel runs:
        conv0 (Ci = 1, its direct kernel) and every layer with Ci a multiple of the k-tile
        (loader mode 6: each k-tile is one tap's channel slice), so no layer needs an im2col
        matrix (_ENC_NHWC_ALL = False restores the round-2 split: channels-last only below K =
        2048, im2col + dense GEMM above)."""
        w = self.conv[i].conv.weight
        Ci, kw = w.shape[1], w.shape[3]
        if (Ci * kw) % 4 != 0:
            return False
        if _ENC_NHWC_ALL and (Ci == 1 or Ci % 64 == 0):
            return True
        return Ci * w.shape[2] * kw < 2048


class UNet1D(nn.Module):
    """UNet1D with the one shape fix the reference needs to run: up_attention is built over
    the 8C channels of the concatenated tensor it is applied to (model_layers.py:339 builds
    SelfAttention(4C) but :364-365 feeds it 8C channels and crashes).  The skip
    concatenations are zero-copy: the skip producers write straight into the halves of the
    buffers the up path reads."""

    def __init__(self, input_channels, output_channels, max_depth=5, kernel_size=None, stride=None, p=0, groups=1):
        super().__init__()
        C = input_channels
        kw = dict(type='1d', leaky=True, downsample=False, kernel_size=kernel_size, stride=stride, p=p, groups=groups)
        kd = dict(kw, downsample=True)
        self.max_depth = max_depth
        self.downsample_layers = nn.ModuleList([
            ConvNormRelu(C, C * 2, **kw), ConvNormRelu(C * 2, C * 2, **kd),
            ConvNormRelu(C * 2, C * 4, **kw), ConvNormRelu(C * 4, C * 4, **kd)])
        self.bottleneck = ConvNormRelu(C * 4, C * 8, type='1d', leaky=True, downsample=False, p=p, groups=groups)
        self.upsample_layers = nn.ModuleList([
            ConvTranspose1D(C * 8, C * 4, stride=2, output_padding=1), ConvNormRelu(C * 8, C * 4, **kw),
            ConvTranspose1D(C * 4, C * 2, stride=2, output_padding=1), ConvNormRelu(C * 4, C * 2, **kw)])
        self.final_conv = nn.Conv1d(C * 2, output_channels, kernel_size=1)
        self.bottleneck_attention = SelfAttention(C * 8)
        self.up_attention = SelfAttention(C * 8)

    def forward(self, x):
        if _grad_path(self, x):
            return _autograd().unet(self, x)
        B, C, T = x.shape
        dev = x.device
        cat1 = torch.empty(B, 4 * C, T, device=dev)
        cat2 = torch.empty(B, 8 * C, T // 2, device=dev)
        d, u = self.downsample_layers, self.upsample_layers
        s1 = d[0](x, out=cat1[:, 2 * C:])
        h = d[1](s1)
        s2 = d[2](h, out=cat2[:, 4 * C:])
        h = d[3](s2)
        h = self.bottleneck_attention(self.bottleneck(h))
        u[0](h, out=cat2[:, :4 * C])
        h = u[1](self.up_attention(cat2))
        u[2](h, out=cat1[:, :2 * C])
        h = u[3](cat1)
        return F.conv1d(h, self.final_conv.weight, self.final_conv.bias)
