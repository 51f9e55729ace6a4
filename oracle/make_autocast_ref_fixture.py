"""configs[4]'s bf16 step measured on the REFERENCE's own modules under torch.autocast.  TEST
INFRASTRUCTURE ONLY: run in the build container (CPU, needs /root/reference), writes
tests/golden/bf16_autocast_ref.json.

oracle/make_autocast_fixture.py measures what torch.autocast does to the training step through
the oracle's functional restatement (oracle.model); VERDICT r05 weak item 3 asked for the same
figures from the reference itself, whose nn.Module ops and PyG layers (here the restatement of
oracle/pyg_restatement.py, PyG being absent) could cast differently under autocast.  This script
loads the reference through the fixture harness of oracle/make_fixtures.py (import stubs for the
data-only modules, Skeleton2D by path, the up_attention shape fix), builds SelfAttention_G /
SelfAttention_D (real_motion_model.py) with the weights of test_bf16_train_step_b32
(weights seeds 1234 / 1235, p = 0), and runs the G-step + D-step of version5_model_train.py:
350-405 (the loss of :367-377, fixed labels 0.93 / 0.07) on its inputs (B = 32 x 64 frames,
audio randn(seed 21) * 2 - 3, pose synth.pose_targets(seed 22)) in fp32 and under
torch.autocast('cpu', dtype=torch.bfloat16).  It records the same figures as the oracle's
fixture: G / D gradient cosines against fp32 (global over the parameters whose true gradient is
not identically zero, median over weight tensors), the losses, and the pose error in train and
eval mode.  tests/test_oracle_golden.py checks that the oracle-under-autocast figures agree with
these.  Only numbers are written; nothing of the reference is copied.

    python -m oracle.make_autocast_ref_fixture
"""
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from oracle import synth  # noqa: E402
from oracle.make_autocast_fixture import GOLDEN, bn_cancelled  # noqa: E402
from oracle.make_fixtures import build_models, in_tmp_cwd, load_reference  # noqa: E402


def ref_step(ml, rmm, audio, pose, bf16):
    """One G-step + one D-step on fresh reference modules (same weights each call)."""
    g, d = build_models(ml, rmm, p=0.0)
    g.train()
    d.train()
    B = audio.shape[0]
    valid, fake_l = torch.full((B, 4), 0.93), torch.full((B, 4), 0.07)
    ctx = torch.autocast('cpu', dtype=torch.bfloat16) if bf16 else torch.autocast('cpu', enabled=False)
    real_motion = torch.diff(pose, dim=1)
    with ctx:
        fake_pose, internal = g(audio, real_pose=pose)
        fake_motion = torch.diff(fake_pose, dim=1)
        fake_d, _ = d(fake_motion)
        acc = fake_motion[:, 1:] - fake_motion[:, :-1]
        jerk = acc[:, 1:] - acc[:, :-1]
        l1 = torch.nn.L1Loss()(real_motion, fake_motion.float())
        adv = torch.nn.MSELoss()(fake_d.float(), valid)
        smooth = torch.mean(torch.norm(acc.float(), dim=-1))
        jk = torch.mean(torch.norm(jerk.float(), dim=-1))
        g_loss = l1 + adv + 0.1 * smooth + 0.05 * jk + internal[0].float() + internal[1].float()
    g_loss.backward()
    gg = {n: p.grad.detach().double().flatten().clone() for n, p in g.named_parameters() if p.grad is not None}
    gshape = {n: tuple(p.shape) for n, p in g.named_parameters()}
    d.zero_grad()
    with ctx:
        with torch.no_grad():
            fp2, _ = g(audio)
            fm2 = torch.diff(fp2, dim=1)
        fd2, _ = d(fm2.detach())
        rd2, _ = d(real_motion)
        d_loss = torch.nn.MSELoss()(rd2.float(), valid) + torch.nn.MSELoss()(fd2.float(), fake_l)
    d_loss.backward()
    dg = {n: p.grad.detach().double().flatten().clone() for n, p in d.named_parameters() if p.grad is not None}
    dshape = {n: tuple(p.shape) for n, p in d.named_parameters()}
    ge, _ = build_models(ml, rmm, p=0.0)     # eval mode on the initial running statistics
    ge.eval()
    with torch.no_grad(), ctx:
        pe, _ = ge(audio)
    return dict(gg=gg, dg=dg, gshape=gshape, dshape=dshape, g_loss=g_loss.item(), d_loss=d_loss.item(),
                pose_train=fake_pose.detach().float(), pose_eval=pe.float())


def agree(a, b, shapes):
    names = [n for n in a if not bn_cancelled(n) and a[n].norm() > 0]
    x, y = torch.cat([a[n] for n in names]), torch.cat([b[n] for n in names])
    glob = (torch.dot(x, y) / (x.norm() * y.norm())).item()
    med = float(np.median([(torch.dot(a[n], b[n]) / (a[n].norm() * b[n].norm())).item()
                           for n in names if len(shapes[n]) >= 2]))
    return glob, med


def rel(a, b):
    return (a - b).abs().max().item() / b.abs().max().item()


def main():
    t0 = time.time()
    cwd = os.getcwd()
    in_tmp_cwd()
    try:
        _, ml, rmm = load_reference()
        torch.manual_seed(0)
        gen = torch.Generator().manual_seed(21)
        audio = torch.randn(32, 64, 128, generator=gen) * 2.0 - 3.0
        pose = torch.from_numpy(synth.pose_targets(32, 64, seed=22))
        f32 = ref_step(ml, rmm, audio, pose, False)
        b16 = ref_step(ml, rmm, audio, pose, True)
    finally:
        os.chdir(cwd)
    cg = agree(f32['gg'], b16['gg'], f32['gshape'])
    cd = agree(f32['dg'], b16['dg'], f32['dshape'])
    out = {
        'source': 'oracle/make_autocast_ref_fixture.py: the reference real_motion_model.py modules (fixture harness '
                  'of oracle/make_fixtures.py), G-step + D-step of version5_model_train.py:350-405, fp32 vs '
                  'torch.autocast(cpu, bfloat16), inputs of test_bf16_train_step_b32',
        'torch': torch.__version__,
        'g_cos_global': cg[0], 'g_cos_weight_median': cg[1],
        'd_cos_global': cd[0], 'd_cos_weight_median': cd[1],
        'g_loss_fp32': f32['g_loss'], 'g_loss_bf16': b16['g_loss'],
        'd_loss_fp32': f32['d_loss'], 'd_loss_bf16': b16['d_loss'],
        'pose_rel_err_train': rel(b16['pose_train'], f32['pose_train']),
        'pose_rel_err_eval': rel(b16['pose_eval'], f32['pose_eval']),
        'seconds': round(time.time() - t0, 1),
    }
    with open(os.path.join(GOLDEN, 'bf16_autocast_ref.json'), 'w') as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
