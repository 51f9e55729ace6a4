"""GPU parity of the training path: every autograd Function (HIP forward + HIP backward)
against torch-CPU fp32 autograd of the same op, then one full G-step + D-step against the
reference's own gradients (tests/golden/train_step_b2t64.npz, produced by running
version5_model_train.py's step math on the reference modules)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as TF

from conftest import golden, rel_err

pytestmark = pytest.mark.gpu
DEV = 'cuda'
TOL = 1e-4
GTOL = 2e-4   # gradients: deeper fp32 chains, relative to max |ref|


def _r(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).float()


def _leaf(t):
    return t.clone().to(DEV).requires_grad_(True), t.clone().requires_grad_(True)


def _check_grads(pairs, tol=GTOL):
    for name, (gd, gc) in pairs.items():
        assert gd is not None and gc is not None, name
        assert rel_err(gd.detach().cpu(), gc.detach()) < tol, (name, rel_err(gd.detach().cpu(), gc.detach()))


@pytest.mark.parametrize('two_d', [False, True])
def test_conv_norm_act_train(two_d):
    from a2m.model_layers import ConvNormRelu
    torch.manual_seed(0)
    if two_d:
        m = ConvNormRelu(3, 8, type='2d', leaky=True, downsample=True)
        x = _r(4, 3, 12, 20, seed=1)
    else:
        m = ConvNormRelu(6, 10, type='1d', leaky=True, downsample=True)
        x = _r(3, 6, 17, seed=1)
    ref = ConvNormRelu(*(3, 8) if two_d else (6, 10), type='2d' if two_d else '1d', leaky=True, downsample=True)
    ref.load_state_dict(m.state_dict())
    with torch.no_grad():
        m.norm.running_var.fill_(1.3)
        ref.norm.running_var.fill_(1.3)
    m.to(DEV).train()
    ref.train()
    xd, xc = _leaf(x)
    yd = m(xd)
    conv = TF.conv2d if two_d else TF.conv1d
    yc = TF.leaky_relu(TF.batch_norm(conv(xc, ref.conv.weight, ref.conv.bias, stride=2, padding=1),
                                     ref.norm.running_mean, ref.norm.running_var, ref.norm.weight,
                                     ref.norm.bias, True, 0.1, 1e-5), 0.2)
    assert rel_err(yd.detach().cpu(), yc.detach()) < TOL
    assert rel_err(m.norm.running_mean.cpu(), ref.norm.running_mean) < TOL
    assert rel_err(m.norm.running_var.cpu(), ref.norm.running_var) < TOL
    gy = _r(*yc.shape, seed=2)
    yd.backward(gy.to(DEV))
    yc.backward(gy)
    _check_grads({'x': (xd.grad, xc.grad), 'w': (m.conv.weight.grad, ref.conv.weight.grad),
                  'gamma': (m.norm.weight.grad, ref.norm.weight.grad),
                  'beta': (m.norm.bias.grad, ref.norm.bias.grad)})


@pytest.mark.parametrize('two_d', [False, True])
def test_conv_norm_act_eval_mode_gradients(two_d):
    """nn.BatchNorm in eval mode with gradients (model_layers.py:51-118 after .eval(); e.g. input
    attribution through a frozen G): running statistics normalise and stay unchanged, and the
    backward holds them fixed -- against torch-CPU autograd of the same eval-mode layer."""
    from a2m.model_layers import ConvNormRelu
    torch.manual_seed(0)
    args = (3, 8) if two_d else (6, 10)
    kind = '2d' if two_d else '1d'
    m = ConvNormRelu(*args, type=kind, leaky=True, downsample=True)
    ref = ConvNormRelu(*args, type=kind, leaky=True, downsample=True)
    ref.load_state_dict(m.state_dict())
    with torch.no_grad():
        for mod in (m, ref):
            mod.norm.running_mean.copy_(_r(args[1], seed=5, scale=0.3))
            mod.norm.running_var.copy_(_r(args[1], seed=6).abs() + 0.5)
            mod.norm.weight.copy_(_r(args[1], seed=7).abs() + 0.5)
            mod.norm.bias.copy_(_r(args[1], seed=8, scale=0.2))
    m.to(DEV).eval()
    ref.eval()
    rm0 = m.norm.running_mean.clone()
    x = _r(4, 3, 12, 20, seed=1) if two_d else _r(3, 6, 17, seed=1)
    xd, xc = _leaf(x)
    yd = m(xd)
    conv = TF.conv2d if two_d else TF.conv1d
    yc = TF.leaky_relu(TF.batch_norm(conv(xc, ref.conv.weight, ref.conv.bias, stride=2, padding=1),
                                     ref.norm.running_mean, ref.norm.running_var, ref.norm.weight,
                                     ref.norm.bias, False, 0.1, 1e-5), 0.2)
    assert rel_err(yd.detach().cpu(), yc.detach()) < TOL
    assert torch.equal(m.norm.running_mean, rm0)
    gy = _r(*yc.shape, seed=2)
    yd.backward(gy.to(DEV))
    yc.backward(gy)
    _check_grads({'x': (xd.grad, xc.grad), 'w': (m.conv.weight.grad, ref.conv.weight.grad),
                  'bias': (m.conv.bias.grad, ref.conv.bias.grad),
                  'gamma': (m.norm.weight.grad, ref.norm.weight.grad),
                  'beta': (m.norm.bias.grad, ref.norm.bias.grad)})


@pytest.mark.parametrize('two_d', [False, True])
def test_frozen_norm_with_dropout_in_training(two_d):
    """Only the norm frozen (m.norm.eval(), the Dropout module left in training mode, a common
    fine-tuning pattern): the reference still drops (model_layers.py:118 runs self.dropout before
    the eval-mode norm).  The hash mask cannot be torch's, so it is read back from the HIP output
    (each element is either the kept raw / (1 - p) or the dropped 0 through the fixed norm) and the
    layer is checked against torch-CPU autograd of conv -> mask -> eval BN -> LeakyReLU with that
    mask; the dropped fraction must be ~p and the mask must differ from none."""
    from a2m.model_layers import ConvNormRelu
    torch.manual_seed(0)
    args = (3, 16) if two_d else (6, 16)
    kind = '2d' if two_d else '1d'
    p = 0.4
    m = ConvNormRelu(*args, type=kind, leaky=True, downsample=True, p=p)
    ref = ConvNormRelu(*args, type=kind, leaky=True, downsample=True, p=p)
    ref.load_state_dict(m.state_dict())
    with torch.no_grad():
        for mod in (m, ref):
            mod.norm.running_mean.copy_(_r(args[1], seed=5, scale=0.3))
            mod.norm.running_var.copy_(_r(args[1], seed=6).abs() + 0.5)
            mod.norm.weight.copy_(_r(args[1], seed=7).abs() + 0.5)
            mod.norm.bias.copy_(_r(args[1], seed=8, scale=0.2))
    m.to(DEV).train()
    m.norm.eval()
    assert m.dropout.training
    rm0 = m.norm.running_mean.clone()
    x = _r(8, 3, 12, 20, seed=1) if two_d else _r(8, 6, 40, seed=1)
    xd, xc = _leaf(x)
    yd = m(xd)
    assert torch.equal(m.norm.running_mean, rm0)
    conv = TF.conv2d if two_d else TF.conv1d
    n = ref.norm

    def head(z):
        return TF.leaky_relu(TF.batch_norm(z, n.running_mean, n.running_var, n.weight, n.bias, False, 0.1,
                                           1e-5), 0.2)
    with torch.no_grad():
        raw = conv(xc, ref.conv.weight, ref.conv.bias, stride=2, padding=1)
        y_keep, y_drop = head(raw / (1 - p)), head(raw * 0)
        y = yd.detach().cpu()
        keep = ((y - y_keep).abs() <= (y - y_drop).abs()).float()
        if two_d:   # Dropout2d: one decision per (clip, channel)
            frac = keep.mean(dim=(2, 3), keepdim=True)
            assert torch.all((frac == 0) | (frac == 1)), 'channel mask not uniform over the map'
            keep = frac.expand_as(keep).contiguous()
    dropped = 1 - keep.mean().item()
    assert 0.2 < dropped < 0.6, dropped
    yc = head(conv(xc, ref.conv.weight, ref.conv.bias, stride=2, padding=1) * keep / (1 - p))
    assert rel_err(y, yc.detach()) < TOL
    gy = _r(*yc.shape, seed=2)
    yd.backward(gy.to(DEV))
    yc.backward(gy)
    _check_grads({'x': (xd.grad, xc.grad), 'w': (m.conv.weight.grad, ref.conv.weight.grad),
                  'bias': (m.conv.bias.grad, ref.conv.bias.grad),
                  'gamma': (m.norm.weight.grad, ref.norm.weight.grad),
                  'beta': (m.norm.bias.grad, ref.norm.bias.grad)})


def test_generator_eval_mode_input_gradient():
    """SelfAttention_G in eval mode with gradients enabled (every BatchNorm on its running
    statistics): the forward equals the no-grad eval forward, and d(pose)/d(mel) matches the
    fp32 CPU oracle's autograd in eval mode."""
    from a2m.real_motion_model import SelfAttention_G
    from oracle import model as OM
    torch.manual_seed(3)
    g = SelfAttention_G(time_steps=64, p=0.2)
    for mod in g.modules():
        if isinstance(mod, torch.nn.modules.batchnorm._BatchNorm):
            with torch.no_grad():
                mod.running_mean.copy_(torch.randn(mod.num_features) * 0.1)
                mod.running_var.copy_(torch.rand(mod.num_features) + 0.5)
        if hasattr(mod, 'gamma'):
            torch.nn.init.constant_(mod.gamma, 0.3)
    sd = {k: v.clone() for k, v in g.state_dict().items()}
    g = g.to(DEV).eval()
    mel = _r(2, 64, 128, seed=4) * 2.0 - 3.0
    with torch.no_grad():
        ref_pose = g(mel.to(DEV))[0].cpu()
    md = mel.clone().to(DEV).requires_grad_(True)
    pose = g(md)[0]
    assert rel_err(pose.detach().cpu(), ref_pose) < TOL
    gy = _r(*pose.shape, seed=5)
    pose.backward(gy.to(DEV))
    mc = mel.clone().requires_grad_(True)
    pc, _ = OM.generator(sd, mc, train=False)
    assert rel_err(pose.detach().cpu(), pc.detach()) < TOL
    pc.backward(gy)
    assert rel_err(md.grad.cpu(), mc.grad) < 1e-3, rel_err(md.grad.cpu(), mc.grad)


def test_convt_bn_relu_train():
    from a2m.model_layers import ConvTranspose1D
    torch.manual_seed(0)
    m = ConvTranspose1D(12, 7)
    ref = torch.nn.Sequential(torch.nn.ConvTranspose1d(12, 7, 3, 2, 1, 1), torch.nn.BatchNorm1d(7), torch.nn.ReLU())
    ref[0].load_state_dict(m.conv_transpose.state_dict())
    ref[1].load_state_dict(m.bn.state_dict())
    m.to(DEV).train()
    ref.train()
    xd, xc = _leaf(_r(3, 12, 9, seed=3))
    yd, yc = m(xd), ref(xc)
    assert rel_err(yd.detach().cpu(), yc.detach()) < TOL
    gy = _r(*yc.shape, seed=4)
    yd.backward(gy.to(DEV))
    yc.backward(gy)
    _check_grads({'x': (xd.grad, xc.grad), 'w': (m.conv_transpose.weight.grad, ref[0].weight.grad),
                  'b': (m.bn.weight.grad, ref[1].weight.grad)})


@pytest.mark.parametrize('C,T,res', [(64, 16, False), (256, 64, True), (256, 64, False), (16, 5, True), (2048, 16, True), (2048, 4, False)])
def test_self_attention_train(C, T, res):
    from a2m.model_layers import SelfAttention
    from oracle import model as OM
    torch.manual_seed(1)
    m = SelfAttention(C)
    with torch.no_grad():
        m.gamma.fill_(0.4)
    sd = {'a.' + k: v.clone().requires_grad_(True) for k, v in m.state_dict().items()}
    m.to(DEV).train()
    xd, xc = _leaf(_r(2, C, T, seed=5))
    rd, rc = _leaf(_r(2, C, T, seed=6)) if res else (None, None)
    yd = m(xd, res=rd)
    yc = OM.self_attention(OM.Ctx(sd), 'a', xc) + (rc if res else 0)
    assert rel_err(yd.detach().cpu(), yc.detach()) < TOL
    gy = _r(2, C, T, seed=7)
    yd.backward(gy.to(DEV))
    yc.backward(gy)
    pairs = {'x': (xd.grad, xc.grad), 'gamma': (m.gamma.grad, sd['a.gamma'].grad)}
    for k in ('query_conv', 'key_conv', 'value_conv'):
        pairs[k + '.w'] = (getattr(m, k).weight.grad, sd[f'a.{k}.weight'].grad)
    pairs['value_conv.b'] = (m.value_conv.bias.grad, sd['a.value_conv.bias'].grad)
    pairs['query_conv.b'] = (m.query_conv.bias.grad, sd['a.query_conv.bias'].grad)
    if res:
        pairs['res'] = (rd.grad, rc.grad)
    _check_grads(pairs)


@pytest.mark.parametrize('B,C,T', [(3, 64, 20), (3, 256, 64), (2, 128, 33)])
def test_channel_attention_train(B, C, T):
    """T = 64: the backward's float4 path; T = 20 / 33: its element path."""
    from a2m.model_layers import ChannelAttention
    from oracle import model as OM
    torch.manual_seed(2)
    m = ChannelAttention(C)
    sd = {'c.' + k: v.clone().requires_grad_(True) for k, v in m.state_dict().items()}
    m.to(DEV).train()
    xd, xc = _leaf(_r(B, C, T, seed=8))
    yd, yc = m(xd), OM.channel_attention(OM.Ctx(sd), 'c', xc)
    assert rel_err(yd.detach().cpu(), yc.detach()) < TOL
    gy = _r(B, C, T, seed=9)
    yd.backward(gy.to(DEV))
    yc.backward(gy)
    _check_grads({'x': (xd.grad, xc.grad), 'w1': (m.fc[0].weight.grad, sd['c.fc.0.weight'].grad),
                  'b1': (m.fc[0].bias.grad, sd['c.fc.0.bias'].grad),
                  'w2': (m.fc[2].weight.grad, sd['c.fc.2.weight'].grad),
                  'b2': (m.fc[2].bias.grad, sd['c.fc.2.bias'].grad)})


@pytest.mark.parametrize('save_pre', [True, False], ids=['saved', 'recompute'])
@pytest.mark.parametrize('kind,J,lo,norm_res,Fr', [(0, 10, 0, True, 7), (0, 42, 10, True, 7), (1, 42, 10, True, 7),
                                                   (1, 10, 0, True, 7), (0, 42, 10, False, 7),
                                                   (0, 42, 10, True, 29), (1, 10, 0, True, 29)])
def test_graph_layer_train(kind, J, lo, norm_res, Fr, save_pre):
    """Both backward paths: the forward's saved pre-LayerNorm output (the weight gradients as
    Z (x) x, Z the aggregation adjoint of dout) and the in-kernel recompute (dout (x) Y)."""
    from a2m import autograd as AG
    from a2m import skeleton as S
    from oracle import model as OM
    ei = S.edge_index(lo, J)
    ptr, idx = [t.to(DEV) for t in S.in_neighbour_csr(ei, J)]
    edges = OM.expand_edges(ei, J, Fr)
    x = _r(Fr * J, 64, seed=10)
    if kind == 0:
        params = [_r(256, 64, seed=11, scale=0.15), None, _r(1, 4, 64, seed=12, scale=0.3),
                  _r(1, 4, 64, seed=13, scale=0.3), _r(64, seed=14, scale=0.1)]
    else:
        params = [_r(64, 64, seed=15, scale=0.12), _r(64, 64, seed=16, scale=0.12), None, None,
                  _r(64, seed=17, scale=0.1)]
    lnw, lnb = (_r(64, seed=18).abs() + 0.5, _r(64, seed=19, scale=0.1)) if norm_res else (None, None)
    allp = params + [lnw, lnb]
    dev_p = [p.clone().to(DEV).requires_grad_(True) if p is not None else None for p in allp]
    cpu_p = [p.clone().requires_grad_(True) if p is not None else None for p in allp]
    xd, xc = _leaf(x)
    # the topology's last entry: keep the pre-LayerNorm copy for the backward (False: recompute)
    yd = AG._GraphLayer.apply(xd, *dev_p, (J, kind, ptr, idx, norm_res, save_pre))
    w0, w1, a_s, a_d, b, lw, lb = cpu_p
    if kind == 0:
        g = OM._gat_fn(xc, edges, w0, a_s, a_d, b, 4)
    else:
        g = OM.graph_conv(OM.Ctx({'g.lin_rel.weight': w0, 'g.lin_rel.bias': b, 'g.lin_root.weight': w1}), 'g',
                          xc, edges)
    yc = TF.leaky_relu(TF.layer_norm(g, (64,), lw, lb), 0.2) + xc if norm_res else g
    assert rel_err(yd.detach().cpu(), yc.detach()) < TOL
    gy = _r(*yc.shape, seed=20)
    yd.backward(gy.to(DEV))
    yc.backward(gy)
    pairs = {'x': (xd.grad, xc.grad)}
    for i, name in enumerate(['w0', 'w1', 'att_src', 'att_dst', 'bias', 'ln_w', 'ln_b']):
        if cpu_p[i] is not None:
            pairs[name] = (dev_p[i].grad, cpu_p[i].grad)
    _check_grads(pairs)


def test_linear_projin_layernorm_train():
    from a2m import autograd as AG
    x = _r(3, 32, 10, seed=21)
    w, b = _r(40, 32, seed=22, scale=0.2), _r(40, seed=23)
    xd, xc = _leaf(x)
    wd, wc = _leaf(w)
    bd, bc = _leaf(b)
    yd = AG._ProjIn.apply(xd, wd, bd)
    yc = TF.linear(xc.permute(0, 2, 1), wc, bc).reshape(30, 40)
    assert rel_err(yd.detach().cpu(), yc.detach()) < TOL
    lw, lb = _r(40, seed=24).abs() + .5, _r(40, seed=25)
    lwd, lwc = _leaf(lw)
    lbd, lbc = _leaf(lb)
    w2, b2 = _r(40, 40, seed=26, scale=0.2), _r(40, seed=27)
    w2d, w2c = _leaf(w2)
    b2d, b2c = _leaf(b2)
    zd = AG._LayerNormBCT.apply(AG.linear(yd, w2d, b2d), lwd, lbd, 10)
    zc = TF.layer_norm(TF.linear(yc, w2c, b2c), (40,), lwc, lbc).view(3, 10, 40).permute(0, 2, 1)
    assert rel_err(zd.detach().cpu(), zc.detach()) < TOL
    gz = _r(3, 40, 10, seed=28)
    zd.backward(gz.to(DEV))
    zc.backward(gz)
    _check_grads({'x': (xd.grad, xc.grad), 'w': (wd.grad, wc.grad), 'b': (bd.grad, bc.grad),
                  'w2': (w2d.grad, w2c.grad), 'b2': (b2d.grad, b2c.grad), 'lw': (lwd.grad, lwc.grad),
                  'lb': (lbd.grad, lbc.grad)})


def test_losses_and_plumbing_train():
    from a2m import autograd as AG
    from oracle import model as OM
    z = golden('losses.npz')
    gd, gc = _leaf(torch.from_numpy(z['gen']))
    real = torch.from_numpy(z['real'])
    ld = AG._PoseLosses.apply(gd, real.to(DEV), (0.7, 0.3))
    lc = torch.stack([OM.bone_length_loss(real, gc), OM.angle_loss(gc)])
    assert rel_err(ld.detach().cpu(), lc.detach()) < TOL
    w = torch.tensor([0.7, 1.3])
    (ld * w.to(DEV)).sum().backward()
    (lc * w).sum().backward()
    _check_grads({'gen': (gd.grad, gc.grad)})
    # motion terms + MSE + diff
    fd, fc = _leaf(_r(3, 9, 104, seed=30))
    rp = _r(3, 9, 104, seed=31)
    td = AG.motion_terms(fd, rp.to(DEV))
    tc = torch.stack(OM.motion_terms(rp, fc))
    assert rel_err(td.detach().cpu(), tc.detach()) < TOL
    md = AG.pos_to_motion(fd)
    mc = torch.diff(fc, dim=1)
    tgt = _r(3, 8, 104, seed=32)
    sd_ = td[0] + 0.1 * td[1] + 0.05 * td[2] + AG.mse_loss(md, tgt.to(DEV))
    sc_ = tc[0] + 0.1 * tc[1] + 0.05 * tc[2] + TF.mse_loss(mc, tgt)
    assert rel_err(sd_.detach().cpu(), sc_.detach()) < TOL
    sd_.backward()
    sc_.backward()
    _check_grads({'fake': (fd.grad, fc.grad)})
    # interp / mean / repeat
    hd, hc = _leaf(_r(2, 6, 8, 15, seed=33))
    od = AG._InterpTime.apply(hd, 64)
    oc = TF.interpolate(hc, size=(64, 1), mode='bilinear').squeeze(-1)
    assert rel_err(od.detach().cpu(), oc.detach()) < TOL
    go = _r(2, 6, 64, seed=34)
    od.backward(go.to(DEV))
    oc.backward(go)
    _check_grads({'interp': (hd.grad, hc.grad)})
    ad, ac = _leaf(_r(2, 6, 5, seed=35))
    ed = AG._RepeatTime.apply(AG._MeanTime.apply(ad) * 2.0, 5)
    ec = (ac.mean(2) * 2.0).unsqueeze(2).repeat(1, 1, 5)
    ge = _r(2, 6, 5, seed=36)
    ed.backward(ge.to(DEV))
    ec.backward(ge)
    _check_grads({'mean/repeat': (ad.grad, ac.grad)})


def test_adam_matches_torch():
    from a2m.optim import FlatAdam
    ps = [torch.nn.Parameter(_r(7, 5, seed=40)), torch.nn.Parameter(_r(11, seed=41))]
    pd = [torch.nn.Parameter(p.detach().clone().to(DEV)) for p in ps]
    ref = torch.optim.Adam(ps, lr=1e-3)
    opt = FlatAdam(pd, lr=1e-3)
    for step in range(3):
        grads = [_r(*p.shape, seed=50 + step * 2 + i) for i, p in enumerate(ps)]
        ref.zero_grad()
        opt.zero_grad()
        for p, q, g in zip(ps, pd, grads):
            p.grad = g.clone()
            q.grad = g.to(DEV)   # a fresh tensor, as autograd hands it over: gathered by step()
        ref.step()
        opt.step()
    for p, q in zip(ps, pd):
        assert rel_err(q.detach().cpu(), p.detach()) < 1e-6
    # every parameter (and its gradient view) starts on a 64-byte boundary of the flat buffers
    for q in pd:
        assert q.data_ptr() % 64 == 0 and q.grad.data_ptr() % 64 == 0


@pytest.mark.parametrize('M,N,K,batch', [(64, 64, 172032, 1), (64, 64, 172032, 4), (64, 64, 40960, 1),
                                         (32, 256, 4096, 1), (320, 256, 4096, 1)])
def test_gemm_many_splits_vs_fp64(M, N, K, batch):
    """Weight-gradient shapes of a training step (graph layers: 64 x 64 outputs over every node;
    SelfAttention Q|K|V): the planner splits K up to 256 ways and the split-K reduce runs its
    16-lane variant for few outputs; compared with an fp64 matmul."""
    from a2m import functional as F
    A = _r(batch, M, K, seed=80)
    B = _r(batch, N, K, seed=81)
    C = torch.empty(batch, M, N, device=DEV)
    F.gemm(M, N, K, A.to(DEV), K, 1, B.to(DEV), K, 1, C, N, 1, batch=batch, a_bs=M * K, b_bs=N * K,
           c_bs=M * N)
    ref = torch.bmm(A.double(), B.double().transpose(1, 2))
    assert rel_err(C.cpu().double(), ref) < TOL


def test_dropout_mask_statistics():
    from a2m import functional as F
    x = torch.ones(1 << 20, device=DEV)
    y = F.dropout(x, 0.2, 1234)
    keep = (y != 0).float().mean().item()
    assert abs(keep - 0.8) < 0.005
    assert torch.allclose(y[y != 0], torch.full_like(y[y != 0], 1.25))
    assert torch.equal(F.dropout(x, 0.2, 1234), y) and not torch.equal(F.dropout(x, 0.2, 99), y)


def _bn_cancelled(name):
    import re
    return name.endswith(('.conv.bias', '.conv_transpose.bias', '.key_conv.bias')) or \
        re.fullmatch(r'conv[123](\.\d)?\.(0|4|9)\.bias', name) is not None


def _grad_errors(module, t, f64, sens, prefix):
    """Per sampled parameter: (name, GPU error vs the exact gradient, reference fp32 error vs the
    exact gradient, the exact gradient's own change under a 1e-7 relative input perturbation),
    all relative to the gradient's scale.  The exact gradient is the fp64 oracle at the fixture's
    sampled indices (oracle/make_f64_grads.py), the sensitivity oracle/make_f64_sensitivity.py."""
    out = []
    params = dict(module.named_parameters())
    for i, n in enumerate(t[f'{prefix}_names']):
        if _bn_cancelled(n):
            continue
        g = params[n].grad.detach().double().reshape(-1).cpu().numpy()
        ix = t[f'{prefix}_idx'][i]
        ok = ix >= 0
        ref = t[f'{prefix}_val'][i][ok]
        exact = f64[f'{prefix}_val'][i][ok]
        scale = max(np.sqrt(t[f'{prefix}_sumsq'][i] / max(g.size, 1)), np.abs(exact).max(), 1e-12)
        out.append((str(n), np.abs(g[ix[ok]] - exact).max() / scale, np.abs(ref - exact).max() / scale,
                    sens[f'{prefix}_sens'][i] / scale))
    return out


# GAT attention vectors: their gradient is a sum over the edge softmax's adjoint, which sums to zero
# over each destination's in-edges, so the exact gradient is a small remainder of cancelling terms
# and its relative error is set by the terms' scale (D's hand_gat.att_dst: 3.65e-3 against the
# reference's 1.3e-5 in every round since round 4, the same value run to run -- summation order,
# not noise).  They get an fp32 floor at the terms' scale.
_CANCELLING = ('.att_src', '.att_dst')
_CANCEL_FLOOR = 1e-3
# A parameter whose EXACT gradient moves by s (relative to its scale) when the input is perturbed
# at fp32's rounding scale (oracle/make_f64_sensitivity.py) cannot be held below ~s by any fp32
# implementation: it also passes within _SENS_MULT x s.  This binds on 3 of the 260 G-step
# parameters of each fixture (tests/test_oracle_golden.py test_f64_sensitivity_fixture) -- at B = 2
# body_gcn5.att_dst (s = 5.6e-2: a pre-activation logit 8.8e-7 of its scale from the leaky-ReLU
# kink), where the reference's own 1.1e-3 error is one draw from that range.
_SENS_MULT = 3.0


def _check_grad_errors(errs, prefix, med_ratio, max_floor, max_ratio):
    """Median GPU error <= med_ratio x the reference's median error; every parameter within
    max_ratio x max(the reference's own error on that parameter, max_floor), or within
    _SENS_MULT x the exact gradient's own fp32-input sensitivity where that is larger.  max_floor
    is an fp32-noise scale (relative to the gradient's scale): it only binds where the
    reference's own error is itself below it, so a parameter the reference gets to 4e-5 cannot
    pass at 5e-2 (the old absolute 5 % floor could hide a >1,000x
    regression)."""
    e = np.array([x[1] for x in errs])
    r = np.array([x[2] for x in errs])
    floor = [max(max_floor, _CANCEL_FLOOR) if x[0].endswith(_CANCELLING) else max_floor for x in errs]
    bound = [max(max_ratio * max(x[2], f), _SENS_MULT * x[3]) for x, f in zip(errs, floor)]
    bad = [(x, b) for x, b in zip(errs, bound) if x[1] > b]
    ratios = sorted(((x[1] / b, x[0]) for x, b in zip(errs, bound)), reverse=True)
    print(f'{prefix}: sensitivity-bound parameters '
          f'{[(x[0], round(float(x[3]), 4)) for x, f in zip(errs, floor) if _SENS_MULT * x[3] > max_ratio * max(x[2], f)]}')
    print(f'{prefix}: median err vs exact {np.median(e):.2e} (reference fp32 {np.median(r):.2e}, '
          f'ratio {np.median(e) / max(np.median(r), 1e-30):.2f}), max {e.max():.2e} '
          f'(reference {r.max():.2e}); worst {sorted(errs, key=lambda x: -x[1])[:3]}; '
          f'largest err / bound: {[(n, round(float(q), 3)) for q, n in ratios[:5]]}')
    assert not bad, bad[:10]
    assert np.median(e) <= med_ratio * np.median(r), (np.median(e), np.median(r))


# Train-step fixtures (oracle/make_fixtures.py, oracle/make_fixtures_r2.py) and the bounds each
# is held to.  Forward values are held to north_star's 1e-4 at B=16; gradients against the
# exact (fp64) gradient, as multiples of the reference's own fp32 error -- see
# test_train_step_vs_reference.
STEP_CASES = {
    # B=16: the gradient bounds DESIGN.md 2.3 states
    # (every parameter within 12x max(reference error, 1e-4); the round-5 bound was max(5 %, 8x).
    # The largest per-parameter ratios seen on the round-6 code: 8.2 (a ChannelAttention fc weight,
    # 2.9e-2 vs the reference's 3.5e-3), 5.5, 4.9 -- another summation order of an ill-conditioned
    # step, DESIGN.md 2.3 -- while a regression like round 5's conv3.9.weight (5e-2 against 4.2e-5,
    # 1,200x) now fails)
    'b16': dict(fixture='train_step_b16t64', tol_out=1e-4, med=2.0, floor=1e-4, ratio=12.0),
    # B=2: batch-statistics BN over 8-16 values in D; outputs at 4e-4 and looser gradient
    # bounds, 30x max(reference error, 2e-3) (kept as a second, smaller case; the round-1 bound was
    # max(60 %, 10x); the largest ratios on the round-6 code: 20 (unet.up_attention.gamma, 2.0e-2
    # against 4.8e-4), 12, 11)
    'b2': dict(fixture='train_step_b2t64', tol_out=4e-4, med=8.0, floor=2e-3, ratio=30.0),
}


@pytest.mark.parametrize('case', ['b16', 'b2'])
def test_train_step_vs_reference(case, g_state, d_state):
    """One G-step (G + D forward in train mode, all G losses, backward) and one D-step, p=0,
    fixed labels (version5_model_train.py:350-405), against the reference's outputs and sampled
    gradients.

    Gradients are measured against the EXACT gradient (the fp64 oracle at the same indices)
    and bounded by multiples of the reference's own fp32 error there: the G-step is
    ill-conditioned in fp32 (the reference's own gradients sit a median 0.3-0.5 % from the
    exact ones, up to 3-7 % on single parameters; tests/golden/*_f64.npz), so an fp32
    implementation with another summation order cannot track the reference's rounding, only
    the true gradient.  Each backward op on identical inputs agrees to <= 2e-4 (the per-op tests
    above), the encoder chain to 2e-5 (test_encoder_chain_vs_fp64) and every loss term's
    dL/dfake to 2e-5 (test_loss_gradients_vs_fp64)."""
    from a2m import autograd as AG
    from a2m.real_motion_model import SelfAttention_D, SelfAttention_G
    c = STEP_CASES[case]
    t = golden(c['fixture'] + '.npz')
    f64 = golden(c['fixture'] + '_f64.npz')
    sens = golden(c['fixture'] + '_f64_sens.npz')
    z = t if 'audio' in t.files else golden('g_eval_b2t64.npz')
    g = SelfAttention_G(p=0.0)
    g.load_state_dict(g_state, strict=False)
    d = SelfAttention_D(out_channels=64, p=0.0)
    d.load_state_dict(d_state, strict=False)
    g, d = g.to(DEV).train(), d.to(DEV).train()
    audio = torch.from_numpy(z['audio']).to(DEV)
    pose = torch.from_numpy(z['real_pose']).to(DEV)
    B = audio.shape[0]
    tol = c['tol_out']
    fake_pose, internal = g(audio, real_pose=pose)
    assert rel_err(fake_pose.detach().cpu(), t['fake_pose']) < TOL
    fake_d, _ = d(AG.pos_to_motion(fake_pose))
    print(f'{case}: fake_d {rel_err(fake_d.detach().cpu(), t["fake_d"]):.2e}')
    assert rel_err(fake_d.detach().cpu(), t['fake_d']) < tol
    terms = AG.motion_terms(fake_pose, pose)
    valid = torch.full((B, 4), 0.93, device=DEV)
    adv = AG.mse_loss(fake_d, valid)
    loss = terms[0] + adv + 0.1 * terms[1] + 0.05 * terms[2] + internal[0] + internal[1]
    parts = torch.stack([terms[0], adv, terms[1], terms[2], internal[0], internal[1]]).detach().cpu().numpy()
    print(f'{case}: parts {np.abs(parts - t["parts"]) / np.abs(t["parts"])}')
    assert np.all(np.abs(parts - t['parts']) <= tol * np.abs(t['parts']))
    assert rel_err(loss.detach().cpu(), t['G_loss']) < tol
    loss.backward()
    eg = _grad_errors(g, t, f64, sens, 'gG')
    d.zero_grad()
    with torch.no_grad():
        fp2, _ = g(audio)
    fd2, _ = d(AG.pos_to_motion(fp2))
    rd2, _ = d(AG.pos_to_motion(pose))
    dl = AG.mse_loss(rd2, valid) + AG.mse_loss(fd2, torch.full((B, 4), 0.07, device=DEV))
    print(f'{case}: d_fake {rel_err(fd2.detach().cpu(), t["d_fake"]):.2e} d_real '
          f'{rel_err(rd2.detach().cpu(), t["d_real"]):.2e} D_loss {rel_err(dl.detach().cpu(), t["D_loss"]):.2e}')
    assert rel_err(fd2.detach().cpu(), t['d_fake']) < tol and rel_err(rd2.detach().cpu(), t['d_real']) < TOL
    assert rel_err(dl.detach().cpu(), t['D_loss']) < tol
    dl.backward()
    ed = _grad_errors(d, t, f64, sens, 'gD')
    _check_grad_errors(eg, f'{case} gG', c['med'], c['floor'], c['ratio'])
    _check_grad_errors(ed, f'{case} gD', c['med'], c['floor'], c['ratio'])


def test_encoder_chain_vs_fp64(g_state):
    """The 2-D encoder (5 conv/BN-train/LeakyReLU layers + bilinear resample) forward and
    backward under a fixed upstream gradient, against the fp64 oracle: a well-conditioned
    chain, so the HIP path must be as exact as fp32 allows."""
    from a2m import autograd as AG
    from a2m.real_motion_model import SelfAttention_G
    from oracle import model
    g = SelfAttention_G(p=0.0)
    g.load_state_dict(g_state, strict=False)
    enc = g.audio_encoder.to(DEV).train()
    audio = torch.from_numpy(golden('g_eval_b2t64.npz')['audio'])
    sd = {k: v.double().requires_grad_('running' not in k) for k, v in g_state.items()
          if k.startswith('audio_encoder') and v.is_floating_point()}
    y64 = model.audio_encoder(model.Ctx(sd, True), audio.double())
    gy = _r(*y64.shape, seed=7).double()
    y64.backward(gy)
    y = AG.audio_encoder(enc, audio.to(DEV), audio.shape[1])
    y.backward(gy.float().to(DEV))
    assert rel_err(y.detach().cpu().double(), y64.detach()) < 1e-5
    for n, p in enc.named_parameters():
        k = 'audio_encoder.' + n
        if k.endswith('conv.bias'):   # cancelled by the batch-statistics BN that follows
            continue
        assert rel_err(p.grad.cpu().double(), sd[k].grad) < 2e-5, k


def test_loss_gradients_vs_fp64(d_state):
    """dL/dfake of every G-step loss term (motion L1, smoothness, jerk, bone length, angle,
    adversarial through the train-mode discriminator) at the reference's fake pose, against
    the fp64 oracle on the same input."""
    from a2m import autograd as AG
    from a2m.real_motion_model import SelfAttention_D
    from oracle import model
    X = torch.from_numpy(golden('train_step_b2t64.npz')['fake_pose'])
    pose = torch.from_numpy(golden('g_eval_b2t64.npz')['real_pose'])
    d = SelfAttention_D(out_channels=64, p=0.0)
    d.load_state_dict(d_state, strict=False)
    d = d.to(DEV).train()
    for p in d.parameters():
        p.requires_grad_(False)
    ds = {k: (v.double() if v.is_floating_point() else v) for k, v in d_state.items()}
    lbl = 0.93
    cpu = {'l1': lambda x: model.motion_terms(pose.double(), x)[0],
           'smooth': lambda x: model.motion_terms(pose.double(), x)[1],
           'jerk': lambda x: model.motion_terms(pose.double(), x)[2],
           'bone': lambda x: model.bone_length_loss(pose.double(), x),
           'angle': model.angle_loss,
           'adv': lambda x: TF.mse_loss(model.discriminator(ds, torch.diff(x, dim=1), train=True),
                                        torch.full((2, 4), lbl, dtype=torch.float64))}
    gpu = {'l1': lambda x: AG.motion_terms(x, pose.to(DEV))[0],
           'smooth': lambda x: AG.motion_terms(x, pose.to(DEV))[1],
           'jerk': lambda x: AG.motion_terms(x, pose.to(DEV))[2],
           'bone': lambda x: AG._PoseLosses.apply(x, pose.to(DEV), (0.7, 0.3))[0],
           'angle': lambda x: AG._PoseLosses.apply(x, pose.to(DEV), (0.7, 0.3))[1],
           'adv': lambda x: AG.mse_loss(d(AG.pos_to_motion(x))[0], torch.full((2, 4), lbl, device=DEV))}
    for name in cpu:
        x64 = X.double().requires_grad_(True)
        cpu[name](x64).backward()
        xg = X.clone().to(DEV).requires_grad_(True)
        gpu[name](xg).backward()
        assert rel_err(xg.grad.cpu().double(), x64.grad) < 2e-5, name


def test_trainer_iteration_runs_and_learns():
    """GANTrainer: g_freq=3, d_freq=1 with dropout on; losses finite, parameters move."""
    from a2m.real_motion_model import SelfAttention_D, SelfAttention_G
    from a2m.training import GANTrainer
    from oracle import synth
    from a2m.mel_features import log_mel_batch
    torch.manual_seed(0)
    g = SelfAttention_G(p=0.2).to(DEV).train()
    d = SelfAttention_D(out_channels=64).to(DEV).train()
    tr = GANTrainer(g, d, lr=1e-4)
    wav = torch.from_numpy(synth.speech_like(4, synth.samples_for_frames(64), seed=2)).to(DEV)
    with torch.no_grad():
        audio = log_mel_batch(wav)
    pose = torch.from_numpy(synth.pose_targets(4, 64, seed=3)).to(DEV)
    w0 = g.unet.final_conv.weight.detach().clone()
    dl, gl = tr.iteration(audio, pose, epoch=0, g_freq=3, d_freq=1)
    assert torch.isfinite(dl) and torch.isfinite(gl)
    assert not torch.equal(w0, g.unet.final_conv.weight.detach())
    assert len(tr.dyn.d_loss_history) == 1


# version5_model_train.py:208-248 as written: the drop-in modules must train under the
# reference's own loop body, torch.optim.Adam and torch.nn losses (not a2m's fused ones)
def _pos_to_motion(pose_batch):
    return torch.diff(pose_batch, n=1, dim=1)


def _temporal_smoothness(motion_seq):
    acceleration = motion_seq[:, 1:] - motion_seq[:, :-1]
    return torch.mean(torch.norm(acceleration, dim=-1))


def _jerk(motion_seq):
    acceleration = motion_seq[:, 1:] - motion_seq[:, :-1]
    jerk = acceleration[:, 1:] - acceleration[:, :-1]
    return torch.mean(torch.norm(jerk, dim=-1))


def test_reference_loop_body_with_torch_adam(g_state, d_state):
    """One iteration of version5_model_train.py:350-405 unchanged (3 G-steps, 1 D-step,
    torch.optim.Adam(lr=1e-3) over all parameters, L1/MSE from torch.nn, p=0, fixed labels) on
    the a2m G / D, against the reference's own run (tests/golden/loop_b16t64.npz).

    The first G_loss is the step's forward (held at 1e-4).  Later losses follow Adam updates:
    Adam's first step moves every weight by ~lr*sign(grad), so weights whose exact gradient is
    below the fp32 noise of the ill-conditioned G-step (test_train_step_vs_reference) move
    either way in any fp32 implementation, and the loop is chaotic from there.  Measured with
    rounding alone (tools/loop_spread.py, profiles/r02_loop_spread.txt; two runs, since CPU
    fp32 is itself thread-order dependent): the fp32 vs the fp64 oracle on CPU, same weights
    and inputs, have G-step 2 / 3 losses 0.1-0.5 % apart and the D loss 0.6-1.7 %; the
    reference's own fp32 run and the fp32 oracle's differ by up to 2.0 % at G-step 3, and the
    pose after the iteration differs by 79-150 % between any two of them.  Steps 2-3 and the D
    loss are held at 5e-2; the pose after the iteration only to its magnitude."""
    from a2m.real_motion_model import SelfAttention_D, SelfAttention_G
    t = golden('train_step_b16t64.npz')
    ref = golden('loop_b16t64.npz')
    generator = SelfAttention_G(p=0.0)
    generator.load_state_dict(g_state, strict=False)
    discriminator = SelfAttention_D(out_channels=64, p=0.0)
    discriminator.load_state_dict(d_state, strict=False)
    generator, discriminator = generator.to(DEV).train(), discriminator.to(DEV).train()
    audio = torch.from_numpy(t['audio']).to(DEV)
    real_pose = torch.from_numpy(t['real_pose']).to(DEV)
    optimizer_G = torch.optim.Adam(generator.parameters(), lr=10e-4)
    optimizer_D = torch.optim.Adam(discriminator.parameters(), lr=10e-4)
    motion_reg_loss, g_loss = torch.nn.L1Loss(), torch.nn.MSELoss()
    d_loss1, d_loss2 = torch.nn.MSELoss(), torch.nn.MSELoss()
    valid = torch.full((audio.shape[0], 4), 0.93, device=DEV)
    fake = torch.full((audio.shape[0], 4), 0.07, device=DEV)
    real_motion = _pos_to_motion(real_pose)
    g_losses = []
    for gen_step in range(3):
        optimizer_G.zero_grad()
        fake_pose, internal_losses = generator(audio, real_pose=real_pose)
        fake_motion = _pos_to_motion(fake_pose)
        fake_d, _ = discriminator(fake_motion)
        G_loss = motion_reg_loss(real_motion, fake_motion) + 1.0 * g_loss(fake_d, valid)
        G_loss += 0.1 * _temporal_smoothness(fake_motion) + 0.05 * _jerk(fake_motion)
        for loss in internal_losses:
            G_loss += loss
        G_loss.backward()
        optimizer_G.step()
        g_losses.append(G_loss.item())
    optimizer_D.zero_grad()
    with torch.no_grad():
        fake_pose_detached, _ = generator(audio)
        fake_motion_detached = _pos_to_motion(fake_pose_detached)
    fake_d, _ = discriminator(fake_motion_detached.detach())
    real_d, _ = discriminator(real_motion)
    D_loss = d_loss1(real_d, valid) + 1.0 * d_loss2(fake_d, fake)
    D_loss.backward()
    optimizer_D.step()
    with torch.no_grad():
        fp_after, _ = generator(audio)
    rg = np.abs(np.array(g_losses) - ref['g_losses']) / np.abs(ref['g_losses'])
    rd = abs(D_loss.item() - ref['d_losses'][0]) / abs(ref['d_losses'][0])
    print(f'loop: G_loss rel err {rg}, D_loss {rd:.2e}, pose after {rel_err(fp_after.cpu(), ref["fake_pose_after"]):.2e}')
    assert rg[0] < TOL
    assert np.all(rg[1:] < 5e-2) and rd < 5e-2
    a, b = np.abs(fp_after.cpu().numpy()).max(), np.abs(ref['fake_pose_after']).max()
    assert np.isfinite(fp_after.cpu().numpy()).all() and 0.5 < a / b < 2.0


@pytest.mark.parametrize('B,Ci,Co,T,k,s,p', [
    (8, 48, 64, 64, 3, 1, 1),     # stride 1, 3 taps: the tap conv of dY (halo layout)
    (6, 40, 96, 16, 3, 1, 1),
    (8, 48, 64, 64, 4, 2, 1),     # stride 2: the ConvTranspose phases (2 + 2 taps)
    (12, 40, 32, 32, 3, 2, 1),    # stride 2, k 3: phases of 1 and 2 taps
    (4, 64, 64, 128, 4, 2, 1),
    (5, 24, 40, 60, 3, 1, 1),     # clips that do not tile 64 rows: the phase GEMM
])
@pytest.mark.parametrize('accumulate', [False, True])
def test_conv1d_dgrad_paths(B, Ci, Co, T, k, s, p, accumulate):
    """conv1d data gradient on each path a2m_conv2d_dgrad_f32 takes, against the fp64 gradient
    (and accumulating into an existing dx)."""
    from a2m import functional as F
    Tout = (T + 2 * p - k) // s + 1
    dy = _r(B, Co, Tout, seed=31).to(DEV)
    w = _r(Co, Ci, k, seed=32, scale=(k * Co) ** -0.5).to(DEV)
    base = _r(B, Ci, T, seed=33).to(DEV)
    dx = base.clone() if accumulate else None
    out = F.conv_dgrad(dy, w, (B, Ci, T), s, p, dx=dx, accumulate=accumulate)
    ref = torch.nn.grad.conv1d_input((B, Ci, T), w.double(), dy.double(), stride=s, padding=p)
    if accumulate:
        ref = ref + base.double()
    assert rel_err(out.double().cpu(), ref.cpu()) < TOL
