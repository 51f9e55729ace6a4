"""bf16 operand precision of the GEMM engine (BASELINE configs[4]: bf16 with fp32 master weights).

The engine rounds each operand to bf16 (RNE) where it enters LDS and accumulates the exact bf16
products in fp32, so on operands that are already bf16 values it must agree with an fp64
product to fp32 accumulation accuracy -- that is the exactness check.  Whole-model runs are
compared with the fp32 path at the tolerance bf16 inputs allow (measured, stated per test).
"""
import numpy as np
import pytest
import torch

from conftest import golden, rel_err

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _r16(t):
    return t.bfloat16().float()


@pytest.mark.parametrize('M,N,K', [(256, 4096, 768), (300, 1000, 500), (256, 512, 12288),
                                   (2560, 2048, 2048)])
def test_bf16_gemm_matches_fp64_on_bf16_operands(M, N, K):
    import a2m
    from a2m import functional as F
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g)
    B = torch.randn(N, K, generator=g)
    ref = _r16(A).double() @ _r16(B).double().t()
    C = torch.empty(M, N, device=DEV)
    with a2m.gemm_precision('bf16'):
        F.gemm(M, N, K, A.to(DEV), K, 1, B.to(DEV), K, 1, C, N, 1)
    assert rel_err(C.cpu().double(), ref) < 1e-5
    # and the fp32 path on the unrounded operands is what it was (precision restored)
    assert a2m.set_gemm_precision('fp32') == 'fp32'
    F.gemm(M, N, K, A.to(DEV), K, 1, B.to(DEV), K, 1, C, N, 1)
    assert rel_err(C.cpu().double(), A.double() @ B.double().t()) < 1e-5


@pytest.mark.parametrize('Ci,Co,T,k,s,p', [(256, 256, 64, 3, 1, 1), (512, 1024, 32, 4, 2, 1),
                                           (64, 128, 64, 1, 1, 0)])
def test_bf16_conv1d_gathered_operands(Ci, Co, T, k, s, p):
    """conv1d through the gathered (im2col / row-vector) loaders, bf16 staging."""
    import a2m
    from a2m import functional as F
    g = torch.Generator().manual_seed(Ci + Co)
    x = torch.randn(8, Ci, T, generator=g)
    w = torch.randn(Co, Ci, k, generator=g) * 0.05
    ref = torch.nn.functional.conv1d(_r16(x).double(), _r16(w).double(), stride=s, padding=p)
    with a2m.gemm_precision('bf16'):
        y = F.conv1d(x.to(DEV), w.to(DEV), None, s, p)
    assert rel_err(y.cpu().double(), ref) < 1e-5


@pytest.mark.parametrize('C,T,res', [(256, 64, True), (128, 48, False)])
def test_bf16_fused_eval_attention_exact_on_bf16_operands(C, T, res):
    """The fused eval attention in bf16 mode (its QKV projection on the bf16 MFMA) on x and
    weights that are already bf16 values: against an fp64 SelfAttention of the same values
    (scores, softmax and PV are fp32 in every mode), and against the engine's bf16 QKV GEMM +
    attention core path (A2M_ATTN_EVAL_BF16=0's route)."""
    import a2m
    from a2m import functional as F
    g = torch.Generator().manual_seed(C + T)
    B = 6
    x = _r16(torch.randn(B, C, T, generator=g))
    ws = [_r16(torch.randn(o, C, generator=g) * C ** -0.5) for o in (C // 8, C // 8, C)]
    bs = [torch.randn(o, generator=g) * 0.1 for o in (C // 8, C // 8, C)]
    gamma = torch.tensor([0.7])
    r = torch.randn(B, C, T, generator=g) if res else None
    q = torch.einsum('oc,bct->bot', ws[0].double(), x.double()) + bs[0].double()[:, None]
    k = torch.einsum('oc,bct->bot', ws[1].double(), x.double()) + bs[1].double()[:, None]
    v = torch.einsum('oc,bct->bot', ws[2].double(), x.double()) + bs[2].double()[:, None]
    att = torch.softmax(torch.einsum('bci,bcj->bij', q, k), dim=-1)
    ref = 0.7 * torch.einsum('bcj,bij->bci', v, att) + x.double() + (r.double() if res else 0.0)
    dv = lambda t: None if t is None else t.to(DEV)  # noqa: E731
    args = [dv(ws[0]), dv(bs[0]), dv(ws[1]), dv(bs[1]), dv(ws[2]), dv(bs[2]), dv(gamma)]
    with a2m.gemm_precision('bf16'):
        fused = F.self_attention(dv(x), *args, res=dv(r), cache={}).cpu()
        prev = F._ATTN_EVAL_BF16
        F._ATTN_EVAL_BF16 = False
        try:
            packed = F.self_attention(dv(x), *args, res=dv(r), cache={}).cpu()
        finally:
            F._ATTN_EVAL_BF16 = prev
    assert rel_err(fused.double(), ref) < 1e-5, rel_err(fused.double(), ref)
    assert rel_err(fused, packed) < 1e-5, rel_err(fused, packed)


def test_bf16_generator_eval_close_to_fp32(g_state):
    """G eval (B=2, T=64 fixture) with bf16 GEMM operands vs the reference's fp32 output.
    Measured bound: bf16 rounding (2^-9 relative per operand) through the 40-odd GEMMs of G."""
    import a2m
    from a2m.real_motion_model import SelfAttention_G
    z = golden('g_eval_b2t64.npz')
    m = SelfAttention_G(p=0.0)
    m.load_state_dict(g_state, strict=False)
    m = m.to(DEV).eval()
    audio = torch.from_numpy(z['audio']).to(DEV)
    with torch.no_grad(), a2m.gemm_precision('bf16'):
        out, _ = m(audio, real_pose=torch.from_numpy(z['real_pose']).to(DEV))
    err = rel_err(out.cpu(), z['pose'])
    print(f'bf16 G eval rel err vs reference fp32: {err:.2e}')
    assert 1e-6 < err < 3e-2
    with torch.no_grad():
        out32, _ = m(audio)
    assert rel_err(out32.cpu(), z['pose']) < 1e-4


def _agreement(ga, gb, shapes):
    """(global cosine of the concatenated gradients, median per-tensor cosine over weight tensors
    (dim >= 2)).  Biases and scalars are left out of the median: several have mathematically
    zero gradients (conv biases ahead of train-mode BatchNorm, key_conv biases under the row
    softmax), so both precisions hold pure rounding noise there."""
    a = torch.cat([ga[n] for n in ga])
    b = torch.cat([gb[n] for n in ga])
    glob = (torch.dot(a, b) / (a.norm() * b.norm())).item()
    cos = [(torch.dot(ga[n], gb[n]) / (ga[n].norm() * gb[n].norm() + 1e-30)).item()
           for n in ga if len(shapes[n]) >= 2 and ga[n].norm() > 0]
    return glob, np.array(cos)


def test_bf16_train_gradients_track_fp32(g_state, d_state):
    """Backward in bf16 vs fp32 at B=8, p=0: G through motion L1 + smoothness + bone length, D
    through its MSE on real motion; gradient cosines.  Two terms are left out because their
    gradients are not continuous in the forward values at this scale: the adversarial term (at
    small batch it passes through train-mode BatchNorm over 16 values in D, the amplification
    that already costs fp32 0.5 %) and the joint-angle hinge penalties
    (real_motion_model.py:350-447: indicator gradients that flip when a 1e-2 bf16 deviation
    moves an angle across a range edge)."""
    import a2m
    from a2m import autograd as AG
    from a2m.real_motion_model import SelfAttention_D, SelfAttention_G
    from oracle import synth
    B = 8
    g_ = torch.Generator().manual_seed(5)
    audio = (torch.randn(B, 64, 128, generator=g_) * 2.0 - 3.0).to(DEV)
    pose = torch.from_numpy(synth.pose_targets(B, 64, seed=6)).to(DEV)
    grads = {}
    for prec in ('fp32', 'bf16'):
        g = SelfAttention_G(p=0.0)
        g.load_state_dict(g_state, strict=False)
        d = SelfAttention_D(out_channels=64, p=0.0)
        d.load_state_dict(d_state, strict=False)
        g, d = g.to(DEV).train(), d.to(DEV).train()
        with a2m.gemm_precision(prec):
            fake_pose, internal = g(audio, real_pose=pose)
            terms = AG.motion_terms(fake_pose, pose)
            loss = terms[0] + 0.1 * terms[1] + 0.05 * terms[2] + internal[0]
            loss.backward()
            rd, _ = d(AG.pos_to_motion(pose))
            dl = AG.mse_loss(rd, torch.full((B, 4), 0.93, device=DEV))
            dl.backward()
        assert torch.isfinite(loss) and torch.isfinite(dl)
        grads[prec] = ({n: p.grad.detach().double().flatten() for n, p in g.named_parameters() if p.grad is not None},
                       {n: p.grad.detach().double().flatten() for n, p in d.named_parameters() if p.grad is not None})
        shapes = {**{n: tuple(p.shape) for n, p in g.named_parameters()},
                  **{n: tuple(p.shape) for n, p in d.named_parameters()}}
    gg, cg = _agreement(grads['fp32'][0], grads['bf16'][0], shapes)
    gd, cd = _agreement(grads['fp32'][1], grads['bf16'][1], shapes)
    print(f'bf16 vs fp32 gradients: G global cosine {gg:.5f}, weights median {np.median(cg):.5f} '
          f'min {cg.min():.4f}; D global {gd:.5f}, weights median {np.median(cd):.5f} min {cd.min():.4f}')
    # measured on MI355X: G global 0.886, weights median 0.945; D global 0.998, median 0.991.
    # D's gradient (one forward, no softmax attention over long rows) tracks fp32 closely; G's
    # passes through three unscaled-softmax attentions (model_layers.py:140-141, no 1/sqrt(d))
    # and 26 train-mode BatchNorms, which amplify the 2^-9 operand rounding.  Bounds sit below
    # the measurement; the exactness of each bf16 backward GEMM is checked separately.
    assert gg > 0.8 and gd > 0.99
    assert np.median(cg) > 0.9 and np.median(cd) > 0.98


@pytest.mark.parametrize('two_d,k,s,p', [(False, 3, 1, 1), (False, 4, 2, 1), (True, 4, 2, 1),
                                         (True, 3, 1, 1)])
def test_bf16_conv_backward_exact_on_bf16_operands(two_d, k, s, p):
    """dgrad and wgrad GEMMs (phase-decomposed dgrad, k-run wgrad loaders) in bf16 vs fp64
    autograd on the bf16-rounded operands (dy, w for dgrad; dy, x for wgrad)."""
    import a2m
    from a2m import functional as F
    g = torch.Generator().manual_seed(k * 10 + s)
    if two_d:
        x = torch.randn(4, 64, 16, 24, generator=g)
        w = torch.randn(128, 64, k, k, generator=g) * 0.05
        conv = lambda a, b: torch.nn.functional.conv2d(a, b, stride=s, padding=p)  # noqa: E731
        pad = (p, p)
    else:
        x = torch.randn(8, 128, 64, generator=g)
        w = torch.randn(256, 128, k, generator=g) * 0.05
        conv = lambda a, b: torch.nn.functional.conv1d(a, b, stride=s, padding=p)  # noqa: E731
        pad = p
    xr = _r16(x).double().requires_grad_(True)
    wr = _r16(w).double().requires_grad_(True)
    y = conv(xr, wr)
    dy = torch.randn(y.shape, generator=g)
    y.backward(_r16(dy).double())
    with a2m.gemm_precision('bf16'):
        dx = F.conv_dgrad(dy.to(DEV), w.to(DEV), tuple(x.shape), s, pad)
        dw = F.conv_wgrad(dy.to(DEV), x.to(DEV), tuple(w.shape), s, pad)
    assert rel_err(dx.cpu().double(), xr.grad) < 1e-5
    assert rel_err(dw.cpu().double(), wr.grad) < 1e-5


def test_bf16_trainer_iteration_learns():
    """GANTrainer iteration (3 G-steps + 1 D-step, dropout on) under bf16: finite, moves."""
    import a2m
    from a2m.real_motion_model import SelfAttention_D, SelfAttention_G
    from a2m.training import GANTrainer
    from oracle import synth
    torch.manual_seed(0)
    g = SelfAttention_G(p=0.2).to(DEV).train()
    d = SelfAttention_D(out_channels=64).to(DEV).train()
    tr = GANTrainer(g, d, lr=1e-4)
    audio = (torch.randn(8, 64, 128) * 2.0 - 3.0).to(DEV)
    pose = torch.from_numpy(synth.pose_targets(8, 64, seed=3)).to(DEV)
    w0 = g.unet.final_conv.weight.detach().clone()
    with a2m.gemm_precision('bf16'):
        dl, gl = tr.iteration(audio, pose, epoch=0, g_freq=3, d_freq=1)
        dl2, gl2 = tr.iteration(audio, pose, epoch=1, g_freq=3, d_freq=1)
    assert all(torch.isfinite(v) for v in (dl, gl, dl2, gl2))
    assert not torch.equal(w0, g.unet.final_conv.weight.detach())
