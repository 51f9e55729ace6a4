"""Drop-in SelfAttention_G / SelfAttention_D (real_motion_model.py) on the MI355X HIP path.

Same constructors, forward signatures, return values and state_dict keys as the reference:
  SelfAttention_G(time_steps=64, in_channels=256, out_channels=256, out_feats=104, p=0.2)
      .forward(audio [B,T,128], real_pose=None) -> (pose [B,T,104], [bone?, angle])
  SelfAttention_D(in_channels=104, out_channels=64, n_downsampling=2, p=0.3, groups=1, aux_classes=10)
      .forward(motion [B,T-1,104], audio=None, aux_labels=None) -> ([B,4], [aux?])
"""
import os

import torch
import torch.nn as nn

from . import functional as F
from . import skeleton as S
from .graph_layers import GATConv, GraphConv
from .model_layers import (AudioEncoder, ChannelAttention, ConvNormRelu, ResBlock, SelfAttention,
                           UNet1D, _autograd, _grad_path, stage_inputs, to_home)


class _GraphTopology(nn.Module):
    """Edge-index templates (persistent buffers, reference keys) + the in-neighbour CSR the
    fused HIP kernel reads (non-persistent)."""

    def _register_topology(self):
        self.register_buffer('body_edge_index_template', S.edge_index(0, S.NUM_BODY))
        self.register_buffer('hand_edge_index_template', S.edge_index(10, S.NUM_HAND))
        for part, n in (('body', S.NUM_BODY), ('hand', S.NUM_HAND)):
            ptr, idx = S.in_neighbour_csr(getattr(self, f'{part}_edge_index_template'), n)
            self.register_buffer(f'_{part}_nbr_ptr', ptr, persistent=False)
            self.register_buffer(f'_{part}_nbr_idx', idx, persistent=False)

    def topology(self, part):
        return getattr(self, f'_{part}_nbr_ptr'), getattr(self, f'_{part}_nbr_idx')

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys,
                              unexpected_keys, error_msgs):
        # A checkpoint's template must hold the skeleton's edges (real_motion_model.py:43-60, any
        # order): the kernels' neighbour CSR is derived from them once, at construction.
        for part in ('body', 'hand'):
            key = f'{prefix}{part}_edge_index_template'
            if key in state_dict:
                mine = getattr(self, f'{part}_edge_index_template')
                theirs = state_dict[key]
                same = tuple(theirs.shape) == tuple(mine.shape) and \
                    sorted(map(tuple, theirs.cpu().long().t().tolist())) == sorted(map(tuple, mine.cpu().t().tolist()))
                if not same:
                    error_msgs.append(f'{key}: checkpoint edge template differs from the Skeleton2D topology')
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys,
                                      unexpected_keys, error_msgs)


class SelfAttention_G(_GraphTopology):
    def __init__(self, time_steps=64, in_channels=256, out_channels=256, out_feats=104, p=0.2):
        super().__init__()
        self.audio_encoder = AudioEncoder(output_feats=time_steps, p=p)
        self.unet = UNet1D(input_channels=in_channels, output_channels=out_channels, p=p)
        self.body_feats = 20
        self.hand_feats = out_feats - self.body_feats
        self.num_body_joints, self.num_hand_joints, self.joint_feat_dim = S.NUM_BODY, S.NUM_HAND, S.FEAT
        self.skeleton = S.Skeleton2D()
        self.parents = S.PARENTS
        self.joint_names = S.JOINT_NAMES
        self.joint_subset = list(range(out_feats // 2))
        self.hand_triples = S.triples(10, S.NUM_HAND)
        self.body_triples = S.triples(0, S.NUM_BODY)
        self.body_edge_index = S.edge_index(0, S.NUM_BODY)
        self.hand_edge_index = S.edge_index(10, S.NUM_HAND)
        self._register_topology()
        self._grouped = {}   # stacked per-branch parameters of the grouped eval launches
        C, J = out_channels, self.joint_feat_dim
        for part, nj in (('body', S.NUM_BODY), ('hand', S.NUM_HAND)):
            if part == 'body':
                pre = [ResBlock(C, type='1d', p=p), ConvNormRelu(C, C, type='1d', leaky=True, p=p),
                       ChannelAttention(C), SelfAttention(C)]
                post = [ResBlock(C, type='1d', p=p), ConvNormRelu(C, C, type='1d', leaky=True, p=p),
                        SelfAttention(C)]
            else:
                pre = [ResBlock(C, type='1d', p=p), ConvNormRelu(C, C, type='1d', leaky=True, p=p),
                       SelfAttention(C), ChannelAttention(C)]
                post = [ResBlock(C, type='1d', p=p), ConvNormRelu(C, C, type='1d', leaky=True, p=p),
                        SelfAttention(C), ChannelAttention(C)]
            setattr(self, f'{part}_decoder_pre', nn.Sequential(*pre))
            setattr(self, f'{part}_proj_in', nn.Linear(C, nj * J))
            for L in range(1, 6):
                layer = GATConv(J, J, heads=4, concat=False) if L % 2 == 1 else GraphConv(J, J)
                setattr(self, f'{part}_gcn{L}', layer)
            setattr(self, f'{part}_layer_norms', nn.ModuleList([nn.LayerNorm(J) for _ in range(5)]))
            setattr(self, f'{part}_relu', nn.LeakyReLU(0.2))
            setattr(self, f'{part}_dropout', nn.Dropout(p=p))
            setattr(self, f'{part}_proj_out', nn.Linear(nj * J, C))
            setattr(self, f'{part}_norm', nn.LayerNorm(C))
            setattr(self, f'{part}_decoder_post', nn.Sequential(*post))
            setattr(self, f'{part}_logits', nn.Conv1d(C, self.body_feats if part == 'body' else self.hand_feats, 1))

    # ------------------------------------------------------------------ eval-mode fused path
    def _graph_stack(self, part, x, out_bct):
        """proj_in -> 5 x fused {GNN, LN64, LeakyReLU, +res} -> proj_out -> LN -> [B,C,T]."""
        B, C, T = x.shape
        nj = getattr(self, f'num_{part}_joints')
        pin, pout = getattr(self, f'{part}_proj_in'), getattr(self, f'{part}_proj_out')
        h = torch.empty(B, T, nj * 64, device=x.device)
        F.conv1d(x, pin.weight, pin.bias, out=h.permute(0, 2, 1))
        a, b = h.view(B * T * nj, 64), torch.empty(B * T * nj, 64, device=x.device)
        ptr, idx = self.topology(part)
        lns = getattr(self, f'{part}_layer_norms')
        if _FUSED_STACK:
            layers, wh = [], []
            bf16 = F.N.lib.a2m_get_gemm_precision() == 1
            for L in range(5):
                g = getattr(self, f'{part}_gcn{L + 1}')
                if L % 2 == 0:
                    U = F.graph_att_proj(g.lin.weight, g.att_src, g.att_dst, cache=g._U)
                    layers.append((0, g.lin.weight, None, U, g.bias, lns[L].weight, lns[L].bias))
                else:
                    layers.append((1, g.lin_rel.weight, g.lin_root.weight, None, g.lin_rel.bias,
                                   lns[L].weight, lns[L].bias))
                if bf16 and _STACK_BF16_WEIGHTS:
                    wh.append(F.graph_weights_bf16(layers[-1][1], layers[-1][2], g._Wh))
            a = F.graph_stack(a, nj, ptr, idx, layers, out=b, wh=wh or None)
        else:
            for L in range(5):
                g = getattr(self, f'{part}_gcn{L + 1}')
                if L % 2 == 0:
                    F.graph_layer(a, nj, 0, ptr, idx, g.lin.weight, None, g.att_src, g.att_dst, g.bias,
                                  lns[L].weight, lns[L].bias, out=b)
                else:
                    F.graph_layer(a, nj, 1, ptr, idx, g.lin_rel.weight, g.lin_root.weight, None, None,
                                  g.lin_rel.bias, lns[L].weight, lns[L].bias, out=b)
                a, b = b, a
        rows = torch.empty(B, T, C, device=x.device)
        F.conv1d(a.view(B, T, nj * 64).permute(0, 2, 1), pout.weight, pout.bias, out=rows.permute(0, 2, 1))
        nrm = getattr(self, f'{part}_norm')
        return F.layernorm_to_bct(rows.view(B * T, C), nrm.weight, nrm.bias, T, eps=nrm.eps, out=out_bct)

    def _branch(self, part, feats, pose_out, f0):
        self._branch_tail(part, getattr(self, f'{part}_decoder_pre')(feats), pose_out, f0)

    def _branch_tail(self, part, x, pose_out, f0):
        x = self._graph_stack(part, x, None)
        x = getattr(self, f'{part}_decoder_post')(x)
        lg = getattr(self, f'{part}_logits')
        nf = lg.weight.shape[0]
        F.conv1d(x, lg.weight, lg.bias, out=pose_out[:, :, f0:f0 + nf].permute(0, 2, 1))

    # ------------------------------------------------------------------ grouped decoders
    # The body and hand decoders share their layer shapes up to the graph stacks' joint counts:
    # decoder_pre = ResBlock + ConvNormRelu (+ ChannelAttention / SelfAttention in either
    # order), decoder_post = ResBlock + ConvNormRelu + SelfAttention (+ hand's ChannelAttention).
    # Eval can run each shared layer for both branches as ONE grouped launch (batch = 2
    # problems with their own weights): twice the workgroups per launch, half the launches.
    # Per launch that is faster (two 256->256 k3 convs 62 -> 48 us, two attentions 40 -> 33 us),
    # but the step measured slower than two concurrent branch streams (_GROUPED 0 / 1 /
    # 2: 2.787 / 2.824 / 2.851 ms, three interleaved 200-step runs each): the chip is already
    # full at B = 64, and the grouped schedule leaves the latency-bound hand graph stack with
    # less concurrent work beside it.  Off by default; tests/test_gpu_grouped.py keeps it exact.
    def _group(self, key, mods, build):
        """Per-problem stacked parameters of `mods` (one per branch), rebuilt when any source
        parameter changes (functional._wkey: weight epoch, pointer, version)."""
        srcs = tuple(t for m in mods for t in _group_sources(m))
        k = F._wkey(srcs)
        c = self._grouped.get(key)
        if c is None or c[0] != k:
            c = self._grouped[key] = (k, build(mods))
        return c[1]

    def _cnr_group(self, key, mods, xs, outs):
        def build(ms):
            chunk = N_tap_chunk()
            packed = torch.stack([F.conv1d_tap_packed(m.conv.weight, m._tap)[0] for m in ms])
            st = lambda f: torch.stack([f(m) for m in ms]).contiguous()
            bn = (st(lambda m: m.norm.weight), st(lambda m: m.norm.bias),
                  st(lambda m: m.norm.running_mean), st(lambda m: m.norm.running_var), ms[0].norm.eps)
            return packed, chunk, st(lambda m: m.conv.bias), bn
        packed, chunk, bias, bn = self._group(key, mods, build)
        m0 = mods[0]
        k, s, p = m0.geometry()
        F.conv1d_tap_group(xs, packed, chunk, bias, m0.conv.out_channels, k, p, bn, m0.act, 0.2, outs)
        return outs

    def _sa_group(self, key, mods, xs, outs, res=None):
        def build(ms):
            qkv = [F.stacked_qkv(*m.weights()[:6], cache=m._pack) for m in ms]
            return (torch.stack([w for w, _ in qkv]), torch.stack([b for _, b in qkv]),
                    torch.cat([m.gamma.reshape(1) for m in ms]))
        wqkv, bqkv, gamma = self._group(key, mods, build)
        return F.self_attention_group(xs, wqkv, bqkv, gamma, outs, res=res)

    def _resblock_group(self, key, mods, xs, outs):
        B, C, T = xs[0].shape
        t1 = torch.empty(2, B, C, T, device=xs[0].device)
        t2 = torch.empty(2, B, C, T, device=xs[0].device)
        self._cnr_group(key + '.c1', [m.conv1 for m in mods], xs, list(t1))
        self._cnr_group(key + '.c2', [m.conv2 for m in mods], list(t1), list(t2))
        return self._sa_group(key + '.sa', [m.attention for m in mods], list(t2), outs, res=xs)

    def _groupable(self, feats):
        B, C, T = feats.shape
        return (_GROUPED and F.N.lib.a2m_get_gemm_precision() == 0 and
                F.N.lib.a2m_self_attention_eval_fits(C, T) and
                F._tap_eligible(feats, 3, 1, 1, C) and C % N_tap_chunk() == 0)

    def _decoders_grouped(self, feats, out):
        B, C, T = feats.shape
        dev = feats.device
        bp, hp = self.body_decoder_pre, self.hand_decoder_pre
        bq, hq = self.body_decoder_post, self.hand_decoder_post
        buf = lambda: torch.empty(2, B, C, T, device=dev)
        # pre: ResBlock, ConvNormRelu grouped; body CA -> SA | hand SA -> CA
        a, b = buf(), buf()
        self._resblock_group('pre.rb', [bp[0], hp[0]], [feats, feats], list(a))
        self._cnr_group('pre.cnr', [bp[1], hp[1]], list(a), list(b))
        body_ca = F.channel_attention(b[0], *bp[2].weights())
        self._sa_group('pre.sa', [bp[3], hp[2]], [body_ca, b[1]], list(a))
        hand_x = F.channel_attention(a[1], *hp[3].weights())
        if _GROUPED == 1:
            # the rest per branch: the hand's graph stack (the longest launch, latency-bound)
            # runs beside the body's stack and decoder_post instead of alone
            if _BRANCH_STREAMS:
                main = torch.cuda.current_stream(dev)
                side = _side_stream(dev)
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    self._branch_tail('hand', hand_x, out, self.body_feats)
                self._branch_tail('body', a[0], out, 0)
                main.wait_stream(side)
            else:
                self._branch_tail('body', a[0], out, 0)
                self._branch_tail('hand', hand_x, out, self.body_feats)
            return
        # graph stacks (10 / 42 joints): body on the side stream, hand on the caller's
        g = buf()
        if _BRANCH_STREAMS:
            main = torch.cuda.current_stream(dev)
            side = _side_stream(dev)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                self._graph_stack('body', a[0], g[0])
            self._graph_stack('hand', hand_x, g[1])
            main.wait_stream(side)
        else:
            self._graph_stack('body', a[0], g[0])
            self._graph_stack('hand', hand_x, g[1])
        # post: ResBlock, ConvNormRelu, SelfAttention grouped; hand's ChannelAttention
        self._resblock_group('post.rb', [bq[0], hq[0]], list(g), list(a))
        self._cnr_group('post.cnr', [bq[1], hq[1]], list(a), list(b))
        self._sa_group('post.sa', [bq[2], hq[2]], list(b), list(a))
        hand_y = F.channel_attention(a[1], *hq[3].weights())
        for part, x, f0 in (('body', a[0], 0), ('hand', hand_y, self.body_feats)):
            lg = getattr(self, f'{part}_logits')
            nf = lg.weight.shape[0]
            F.conv1d(x, lg.weight, lg.bias, out=out[:, :, f0:f0 + nf].permute(0, 2, 1))

    def forward(self, audio, real_pose=None):
        (audio, real_pose), home = stage_inputs(self, audio, real_pose)
        out, losses = self._forward(audio, real_pose)
        if home != out.device:
            out, *losses = to_home(home, out, *losses)
        return out, list(losses)

    def _forward(self, audio, real_pose=None):
        if _grad_path(self, audio):
            return _autograd().generator_forward(self, audio, real_pose)
        B, T, _ = audio.shape
        feats = self.unet(self.audio_encoder(audio))
        out = torch.empty(B, T, self.body_feats + self.hand_feats, device=audio.device)
        if self._groupable(feats):
            self._decoders_grouped(feats, out)
        elif _BRANCH_STREAMS:
            # the body and hand decoders are independent after the UNet: the body branch runs
            # on a side stream (forked from / joined to the caller's, so graph capture records
            # both), overlapping its latency-bound small launches with the hand branch's
            # the hand branch (42-joint graph stack) is the longer one; forked first, on the side
            # stream (measured 2.96 vs 3.00 ms a step; a high-priority side stream measured 4.8 ms,
            # each branch on its own side stream or the branches captured layer by layer in
            # alternation measured neutral or slower: DESIGN.md 6 / 9)
            main = torch.cuda.current_stream(audio.device)
            side = _side_stream(audio.device)
            side.wait_stream(main)
            first, second = (('hand', self.body_feats), ('body', 0)) if _HAND_ON_SIDE else \
                (('body', 0), ('hand', self.body_feats))
            with torch.cuda.stream(side):
                self._branch(first[0], feats, out, first[1])
            self._branch(second[0], feats, out, second[1])
            main.wait_stream(side)
        else:
            self._branch('body', feats, out, 0)
            self._branch('hand', feats, out, self.body_feats)
        losses = F.pose_losses(out, real_pose)
        internal = [losses[0]] if real_pose is not None else []
        internal.append(losses[1])
        return out, internal

    # ------------------------------------------------------------------ reference loss API
    # real_motion_model.py:307-461; differentiable in gen_pose, host tensors staged like forward
    def _pose_loss(self, gen_pose, real_pose, angle_w, which):
        (gen_pose, real_pose), home = stage_inputs(self, gen_pose, real_pose)
        assert gen_pose.shape[-1] == len(self.parents) * 2, 'Pose dimension mismatch'
        loss = _autograd().pose_losses(gen_pose, real_pose, angle_w)[which]
        return to_home(home, loss)[0]

    def compute_bone_length_loss(self, real_pose, gen_pose):
        assert real_pose.shape[-1] == len(self.parents) * 2, 'Pose dimension mismatch'
        return self._pose_loss(gen_pose, real_pose, F.ANGLE_W, 0)

    def compute_hand_joint_angle_loss(self, gen_pose):
        return self._pose_loss(gen_pose, None, (1.0, 0.0), 1)

    def compute_body_joint_angle_loss(self, gen_pose):
        if gen_pose.shape[-1] != len(self.parents) * 2:   # :403-404
            return torch.tensor(0.0, device=gen_pose.device)
        return self._pose_loss(gen_pose, None, (0.0, 1.0), 1)

    def compute_comprehensive_angle_loss(self, gen_pose):
        return self._pose_loss(gen_pose, None, F.ANGLE_W, 1)


_BRANCH_STREAMS = os.environ.get('A2M_BRANCH_STREAMS', '1') != '0'
# the hand branch (the longer one) forked onto the side stream and issued first; False: the body
_HAND_ON_SIDE = True
# body + hand decoder layers as grouped launches: 0 off, 1 decoder_pre grouped (the rest per
# branch on two streams), 2 decoder_pre and decoder_post grouped
_GROUPED = 0


def N_tap_chunk():
    return F.N.lib.a2m_conv1d_tap_chunk()


def _group_sources(m):
    """The parameters / buffers a grouped launch stacks for module m."""
    if isinstance(m, ConvNormRelu):
        n = m.norm
        return (m.conv.weight, m.conv.bias, n.weight, n.bias, n.running_mean, n.running_var)
    return m.weights()   # SelfAttention
_FUSED_STACK = True   # one launch for the 5 graph layers
# bf16 operand mode: the stack's layer weights as cached bf16 copies (bitwise the same result)
_STACK_BF16_WEIGHTS = True
_SIDE_STREAMS = {}


def _side_stream(device):
    key = device.index or 0
    s = _SIDE_STREAMS.get(key)
    if s is None:
        s = _SIDE_STREAMS[key] = torch.cuda.Stream(device=device)
    return s


class SelfAttention_D(_GraphTopology):
    def __init__(self, in_channels=104, out_channels=64, n_downsampling=2, p=0.3, groups=1, aux_classes=10, **kwargs):
        super().__init__()
        assert groups == 1
        self.n_downsampling, self.groups, self.p = n_downsampling, groups, p
        self.skeleton = S.Skeleton2D()
        self.num_body_joints, self.num_hand_joints, self.joint_feat_dim = S.NUM_BODY, S.NUM_HAND, S.FEAT
        self.body_edge_index = S.edge_index(0, S.NUM_BODY)
        self.hand_edge_index = S.edge_index(10, S.NUM_HAND)
        self._register_topology()

        def block(ci, co, k, s, pad=1):
            return [nn.Conv1d(ci, co, k, s, pad), nn.BatchNorm1d(co), nn.LeakyReLU(0.2), nn.Dropout(p)]

        oc = out_channels
        self.conv1 = nn.Sequential(*block(in_channels, oc, 4, 2), *block(oc, oc, 4, 1))
        self.conv2 = nn.ModuleList()
        cur = oc
        for n in range(1, n_downsampling + 1):
            mul = min(2 ** n, 16)
            self.conv2.append(nn.Sequential(*block(cur, cur * mul, 4, 2), *block(cur * mul, cur * mul, 4, 1)))
            cur *= mul
        self.conv3 = nn.Sequential(*block(cur, cur * 2, 4, 1), *block(cur * 2, cur * 4, 4, 1),
                                   SelfAttention(cur * 4), *block(cur * 4, cur * 4, 3, 1))
        J = self.joint_feat_dim
        self.body_proj = nn.Linear(cur * 4 // 2, S.NUM_BODY * J)
        self.hand_proj = nn.Linear(cur * 4 // 2, S.NUM_HAND * J)
        self.body_gat = GATConv(J, J, heads=4, concat=False)
        self.hand_gat = GATConv(J, J, heads=4, concat=False)
        self.body_graph_out = nn.Linear(S.NUM_BODY * J, cur * 2)
        self.hand_graph_out = nn.Linear(S.NUM_HAND * J, cur * 2)
        self.audio_fusion = nn.Conv1d(256, cur * 4, kernel_size=1)
        out_shape = kwargs.get('out_shape', 1)
        self.logits = nn.Conv1d(cur * 4 * 2, out_shape, kernel_size=3, stride=1, padding=1)
        self.aux_classifier = nn.Sequential(nn.Linear(cur * 4, 512), nn.LeakyReLU(0.2), nn.Dropout(p),
                                            nn.Linear(512, aux_classes))
        self.aux_loss_fn = nn.CrossEntropyLoss()
        self.cur = cur

    def conv_blocks(self):
        """(conv, bn) pairs of the trunk in order, with the SelfAttention position marked."""
        seqs = [self.conv1] + list(self.conv2) + [self.conv3]
        out = []
        for sq in seqs:
            mods = list(sq)
            for i, m in enumerate(mods):
                if isinstance(m, nn.Conv1d):
                    out.append((m, mods[i + 1]))
                elif isinstance(m, SelfAttention):
                    out.append(m)
        return out

    def forward(self, x, audio=None, aux_labels=None):
        if audio is not None or aux_labels is not None:
            raise NotImplementedError('audio fusion / aux classifier are off the training path '
                                      '(version5_model_train.py never passes them)')
        (x,), home = stage_inputs(self, x)
        out, aux = self._forward(x)
        return to_home(home, out)[0], aux

    def _forward(self, x):
        if _grad_path(self, x):
            return _autograd().discriminator_forward(self, x), []
        h = x.transpose(-1, -2)
        if h.shape[2] < 4:
            h = torch.nn.functional.pad(h, (0, 4 - h.shape[2] % 4)).contiguous()
        blocks = self.conv_blocks()
        B = x.shape[0]
        for i, blk in enumerate(blocks):
            if isinstance(blk, SelfAttention):
                h = blk(h)
                continue
            conv, bn = blk
            last = i == len(blocks) - 1
            Tin = h.shape[2]
            Tout = (Tin + 2 * conv.padding[0] - conv.kernel_size[0]) // conv.stride[0] + 1
            out = None
            if last:  # write straight into the first half of the logits' concat buffer
                cat = torch.empty(B, 2 * conv.out_channels, Tout, device=x.device)
                out = cat[:, :conv.out_channels]
            h = F.conv1d(h, conv.weight, conv.bias, conv.stride[0], conv.padding[0],
                         bn=(bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.eps),
                         act=F.ACT_LRELU, out=out)
        C, T = h.shape[1], h.shape[2]
        g = torch.empty(B, 2 * self.cur * 2, device=x.device)
        for k, (part, nj) in enumerate((('body', S.NUM_BODY), ('hand', S.NUM_HAND))):
            half = h[:, k * C // 2:(k + 1) * C // 2]
            pooled = F.mean_time(half)
            proj = getattr(self, f'{part}_proj')
            z = F.linear(pooled, proj.weight, proj.bias).view(B * nj, 64)
            gat = getattr(self, f'{part}_gat')
            ptr, idx = self.topology(part)
            z2 = F.graph_layer(z, nj, 0, ptr, idx, gat.lin.weight, None, gat.att_src, gat.att_dst,
                               gat.bias, None, None, norm_res=False)
            go = getattr(self, f'{part}_graph_out')
            F.linear(z2.view(B, nj * 64), go.weight, go.bias, out=g[:, k * self.cur * 2:(k + 1) * self.cur * 2])
        F.repeat_time(g, cat[:, C:])
        lg = F.conv1d(cat, self.logits.weight, self.logits.bias, 1, 1)
        return lg.transpose(-1, -2).squeeze(-1), []


# generate_motion_video.py:18 imports `Speech2Gesture_G` from a module absent from the reference;
# the generator it loads (MODEL_PATH_G, saved by version5_model_train.py:510-516) is this one.
Speech2Gesture_G = SelfAttention_G
