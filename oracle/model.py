"""Functional torch-CPU fp32 restatement of the generator / discriminator.  TEST ORACLE ONLY.

Operates on a plain state_dict (names identical to the reference's), so the same weights
drive the reference harness, this oracle and the HIP product.  Follows:
  ConvNormRelu        model_layers.py:51-118   conv -> dropout -> BN -> (Leaky)ReLU
  SelfAttention       model_layers.py:121-146  softmax(Q^T K) without 1/sqrt(d), gamma*out + x
  ChannelAttention    model_layers.py:149-174
  ResBlock            model_layers.py:177-190
  ConvTranspose1D     model_layers.py:193-215
  AudioEncoder        model_layers.py:219-280  (bilinear interp (T,1), align_corners=False)
  UNet1D              model_layers.py:283-374  (up_attention over 8C channels: see DESIGN.md)
  SelfAttention_G     real_motion_model.py:154-278
  losses              real_motion_model.py:307-461
  SelfAttention_D     real_motion_model.py:580-642
  train-step losses   version5_model_train.py:208-248, 350-405
GNN layers come from oracle/pyg_restatement.py semantics (see its header).
Dropout is not modelled (oracle runs with p=0).
"""
import math

import torch
import torch.nn.functional as F

from oracle import pyg_restatement as pyg

PARENTS = [-1, 0, 1, 2, 0, 4, 5, 0, 7, 7, 6,
           10, 11, 12, 13, 10, 15, 16, 17, 10, 19, 20, 21, 10, 23, 24, 25, 10, 27, 28, 29,
           3, 31, 32, 33, 34, 31, 36, 37, 38, 31, 40, 41, 42, 31, 44, 45, 46, 31, 48, 49, 50]


def _edges(lo, n):
    src, dst = [], []
    for i in range(n):
        par = PARENTS[lo + i]
        if par >= lo and par < lo + n:
            src += [par - lo, i]
            dst += [i, par - lo]
    return torch.tensor([src, dst], dtype=torch.long)


BODY_EDGES = _edges(0, 10)
HAND_EDGES = _edges(10, 42)


def _triples(lo, n):
    out = []
    for i in range(n):
        par = PARENTS[lo + i]
        if not (lo <= par < lo + n):
            continue
        kids = [j for j in range(i + 1, n) if PARENTS[lo + j] == lo + i]
        if kids:
            out.append((par - lo, i, kids[0]))
    return out


HAND_TRIPLES = _triples(10, 42)
BODY_TRIPLES = _triples(0, 10)


class Ctx:
    def __init__(self, sd, train=False):
        self.sd, self.train = sd, train

    def __getitem__(self, k):
        return self.sd[k]

    def bn(self, x, pfx):
        return F.batch_norm(x, self.sd[pfx + '.running_mean'], self.sd[pfx + '.running_var'],
                            self.sd[pfx + '.weight'], self.sd[pfx + '.bias'],
                            training=self.train, momentum=0.1, eps=1e-5)


def conv_norm_act(c, pfx, x, stride=1, pad=1, two_d=False, leaky=True):
    conv = F.conv2d if two_d else F.conv1d
    y = conv(x, c[pfx + '.conv.weight'], c[pfx + '.conv.bias'], stride=stride, padding=pad)
    y = c.bn(y, pfx + '.norm')
    return F.leaky_relu(y, 0.2) if leaky else F.relu(y)


def self_attention(c, pfx, x):
    q = F.conv1d(x, c[pfx + '.query_conv.weight'], c[pfx + '.query_conv.bias'])
    k = F.conv1d(x, c[pfx + '.key_conv.weight'], c[pfx + '.key_conv.bias'])
    v = F.conv1d(x, c[pfx + '.value_conv.weight'], c[pfx + '.value_conv.bias'])
    a = torch.softmax(torch.bmm(q.transpose(1, 2), k), dim=-1)          # [B,T,T]
    o = torch.bmm(v, a.transpose(1, 2))                                  # [B,C,T]
    return c[pfx + '.gamma'] * o + x


def channel_attention(c, pfx, x):
    def mlp(z):
        z = F.relu(F.linear(z, c[pfx + '.fc.0.weight'], c[pfx + '.fc.0.bias']))
        return torch.sigmoid(F.linear(z, c[pfx + '.fc.2.weight'], c[pfx + '.fc.2.bias']))
    return x * (mlp(x.mean(-1)) + mlp(x.amax(-1))).unsqueeze(-1)


def res_block(c, pfx, x):
    y = conv_norm_act(c, pfx + '.conv1', x)
    y = conv_norm_act(c, pfx + '.conv2', y)
    return self_attention(c, pfx + '.attention', y) + x


def conv_t_bn_relu(c, pfx, x):
    y = F.conv_transpose1d(x, c[pfx + '.conv_transpose.weight'], c[pfx + '.conv_transpose.bias'],
                           stride=2, padding=1, output_padding=1)
    return F.relu(c.bn(y, pfx + '.bn'))


def audio_encoder(c, audio):
    x = audio.unsqueeze(1)
    for i in range(3):
        x = conv_norm_act(c, f'audio_encoder.conv.{i}', x, stride=2, pad=1, two_d=True)
    x = conv_norm_act(c, 'audio_encoder.conv.3', x, stride=1, pad=1, two_d=True)
    x = conv_norm_act(c, 'audio_encoder.conv.4', x, stride=1, pad=(1, 3), two_d=True)
    x = F.interpolate(x, size=(audio.shape[1], 1), mode='bilinear', align_corners=False)
    return x.squeeze(-1)


def unet(c, x):
    p = 'unet.'
    x = conv_norm_act(c, p + 'downsample_layers.0', x)
    s1 = x
    x = conv_norm_act(c, p + 'downsample_layers.1', x, stride=2)
    x = conv_norm_act(c, p + 'downsample_layers.2', x)
    s2 = x
    x = conv_norm_act(c, p + 'downsample_layers.3', x, stride=2)
    x = conv_norm_act(c, p + 'bottleneck', x)
    x = self_attention(c, p + 'bottleneck_attention', x)
    x = torch.cat([conv_t_bn_relu(c, p + 'upsample_layers.0', x), s2], 1)
    x = self_attention(c, p + 'up_attention', x)
    x = conv_norm_act(c, p + 'upsample_layers.1', x)
    x = torch.cat([conv_t_bn_relu(c, p + 'upsample_layers.2', x), s1], 1)
    x = conv_norm_act(c, p + 'upsample_layers.3', x)
    return F.conv1d(x, c[p + 'final_conv.weight'], c[p + 'final_conv.bias'])


def gat(c, pfx, x, edges, heads=4):
    lw = c.sd.get(pfx + '.lin.weight', c.sd.get(pfx + '.lin_src.weight'))
    return _gat_fn(x, edges, lw, c[pfx + '.att_src'], c[pfx + '.att_dst'], c[pfx + '.bias'], heads)


def _gat_fn(x, edges, lw, a_s, a_d, bias, heads):
    N = x.shape[0]
    xp = F.linear(x, lw).view(N, heads, -1)
    asrc, adst = (xp * a_s).sum(-1), (xp * a_d).sum(-1)
    ei = pyg._add_self_loops(edges, N)
    e = F.leaky_relu(asrc[ei[0]] + adst[ei[1]], 0.2)
    alpha = pyg._segment_softmax(e, ei[1], N)
    msg = xp[ei[0]] * alpha.unsqueeze(-1)   # (under autocast: bf16 rows x fp32 weights -> fp32)
    out = torch.zeros(xp.shape, dtype=msg.dtype, device=xp.device).index_add(0, ei[1], msg)
    return out.mean(1) + bias


def graph_conv(c, pfx, x, edges):
    agg = torch.zeros_like(x).index_add(0, edges[1], x[edges[0]])
    return F.linear(agg, c[pfx + '.lin_rel.weight'], c[pfx + '.lin_rel.bias']) + \
        F.linear(x, c[pfx + '.lin_root.weight'])


def expand_edges(tmpl, nodes, graphs):
    off = (torch.arange(graphs) * nodes).view(-1, 1, 1)
    return (tmpl.unsqueeze(0) + off).permute(1, 0, 2).reshape(2, -1)


def graph_stack(c, part, x, J, tmpl):
    """[B,C,T] -> proj_in -> 5 x {GNN, LN64, LReLU, +res} -> proj_out -> LN256 -> [B,C,T]."""
    B, C, T = x.shape
    h = F.linear(x.permute(0, 2, 1), c[f'{part}_proj_in.weight'], c[f'{part}_proj_in.bias'])
    h = h.reshape(B * T * J, 64)
    edges = expand_edges(tmpl, J, B * T)
    for L in range(5):
        pfx = f'{part}_gcn{L + 1}'
        y = gat(c, pfx, h, edges) if L % 2 == 0 else graph_conv(c, pfx, h, edges)
        y = F.layer_norm(y, (64,), c[f'{part}_layer_norms.{L}.weight'],
                         c[f'{part}_layer_norms.{L}.bias'], eps=1e-5)
        h = F.leaky_relu(y, 0.2) + h
    h = F.linear(h.view(B, T, J * 64), c[f'{part}_proj_out.weight'], c[f'{part}_proj_out.bias'])
    h = F.layer_norm(h, (C,), c[f'{part}_norm.weight'], c[f'{part}_norm.bias'], eps=1e-5)
    return h.permute(0, 2, 1)


def generator(sd, audio, real_pose=None, train=False):
    """SelfAttention_G.forward (real_motion_model.py:154-278). Returns (pose [B,T,104], losses)."""
    c = Ctx(sd, train)
    feats = unet(c, audio_encoder(c, audio))
    # body branch
    b = res_block(c, 'body_decoder_pre.0', feats)
    b = conv_norm_act(c, 'body_decoder_pre.1', b)
    b = channel_attention(c, 'body_decoder_pre.2', b)
    b = self_attention(c, 'body_decoder_pre.3', b)
    b = graph_stack(c, 'body', b, 10, BODY_EDGES)
    b = res_block(c, 'body_decoder_post.0', b)
    b = conv_norm_act(c, 'body_decoder_post.1', b)
    b = self_attention(c, 'body_decoder_post.2', b)
    b = F.conv1d(b, c['body_logits.weight'], c['body_logits.bias'])
    # hand branch
    h = res_block(c, 'hand_decoder_pre.0', feats)
    h = conv_norm_act(c, 'hand_decoder_pre.1', h)
    h = self_attention(c, 'hand_decoder_pre.2', h)
    h = channel_attention(c, 'hand_decoder_pre.3', h)
    h = graph_stack(c, 'hand', h, 42, HAND_EDGES)
    h = res_block(c, 'hand_decoder_post.0', h)
    h = conv_norm_act(c, 'hand_decoder_post.1', h)
    h = self_attention(c, 'hand_decoder_post.2', h)
    h = channel_attention(c, 'hand_decoder_post.3', h)
    h = F.conv1d(h, c['hand_logits.weight'], c['hand_logits.bias'])
    out = torch.cat([b, h], 1).transpose(1, 2)
    losses = []
    if real_pose is not None:
        losses.append(bone_length_loss(real_pose, out))
    losses.append(angle_loss(out))
    return out, losses


# ---------------------------------------------------------------- losses
def bone_length_loss(real, gen):
    B, T, _ = real.shape
    child = torch.tensor([i for i in range(52) if PARENTS[i] != -1])
    par = torch.tensor([PARENTS[i] for i in range(52) if PARENTS[i] != -1])

    def lens(p):
        p = p.reshape(B, T, 52, 2)
        return torch.linalg.vector_norm(p[:, :, child] - p[:, :, par], dim=-1).mean(1)
    return F.mse_loss(lens(gen), lens(real))


def _signed_angles(p, triples):
    t = torch.tensor(triples)
    a, j, k = p[:, :, t[:, 0]], p[:, :, t[:, 1]], p[:, :, t[:, 2]]
    u, v = j - a, k - j
    dot = (u * v).sum(-1)
    cross = u[..., 0] * v[..., 1] - u[..., 1] * v[..., 0]
    return torch.atan2(cross, dot)


def hand_angle_loss(gen):
    B, T, _ = gen.shape
    ang = _signed_angles(gen.reshape(B, T, 52, 2)[:, :, 10:52], HAND_TRIPLES)
    return (F.relu(0.0 - ang) + F.relu(ang - math.pi)).mean()


def body_angle_loss(gen):
    B, T, _ = gen.shape
    ang = _signed_angles(gen.reshape(B, T, 52, 2)[:, :, :10], BODY_TRIPLES)
    return (F.relu(-math.pi / 2 - ang) + F.relu(ang - math.pi)).mean()


def angle_loss(gen):
    return 0.7 * hand_angle_loss(gen) + 0.3 * body_angle_loss(gen)


def motion_terms(real_pose, fake_pose):
    """version5_model_train.py:208-248: L1 on motion, smoothness (accel), jerk."""
    rm, fm = torch.diff(real_pose, dim=1), torch.diff(fake_pose, dim=1)
    acc = fm[:, 1:] - fm[:, :-1]
    jerk = acc[:, 1:] - acc[:, :-1]
    return (F.l1_loss(fm, rm), torch.linalg.vector_norm(acc, dim=-1).mean(),
            torch.linalg.vector_norm(jerk, dim=-1).mean())


# ---------------------------------------------------------------- discriminator
def _d_block(c, pfx, x, idx, stride, pad=1):
    x = F.conv1d(x, c[f'{pfx}.{idx}.weight'], c[f'{pfx}.{idx}.bias'], stride=stride, padding=pad)
    return F.leaky_relu(c.bn(x, f'{pfx}.{idx + 1}'), 0.2)


def discriminator(sd, x, train=False):
    """SelfAttention_D.forward (real_motion_model.py:580-642), audio=None, aux_labels=None."""
    c = Ctx(sd, train)
    x = x.transpose(1, 2)
    if x.shape[2] < 4:
        x = F.pad(x, (0, 4 - x.shape[2] % 4))
    x = _d_block(c, 'conv1', x, 0, 2)
    x = _d_block(c, 'conv1', x, 4, 1)
    for n in range(2):
        x = _d_block(c, f'conv2.{n}', x, 0, 2)
        x = _d_block(c, f'conv2.{n}', x, 4, 1)
    x = _d_block(c, 'conv3', x, 0, 1)
    x = _d_block(c, 'conv3', x, 4, 1)
    x = self_attention(c, 'conv3.8', x)
    x = _d_block(c, 'conv3', x, 9, 1)
    B, C, T = x.shape
    outs = []
    for part, J, tmpl, half in (('body', 10, BODY_EDGES, x[:, :C // 2]), ('hand', 42, HAND_EDGES, x[:, C // 2:])):
        z = F.linear(half.mean(2), c[f'{part}_proj.weight'], c[f'{part}_proj.bias']).reshape(B * J, 64)
        z = _gat_fn(z, expand_edges(tmpl, J, B), c.sd.get(f'{part}_gat.lin.weight', c.sd.get(f'{part}_gat.lin_src.weight')),
                    c[f'{part}_gat.att_src'], c[f'{part}_gat.att_dst'], c[f'{part}_gat.bias'], 4)
        outs.append(F.linear(z.reshape(B, -1), c[f'{part}_graph_out.weight'], c[f'{part}_graph_out.bias']))
    g = torch.cat(outs, 1).unsqueeze(2).repeat(1, 1, T)
    x = torch.cat([x, g], 1)
    x = F.conv1d(x, c['logits.weight'], c['logits.bias'], padding=1)
    return x.transpose(-1, -2).squeeze(-1)
