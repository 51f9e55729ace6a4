"""configs[4]'s bf16 training step pinned against the reference's own bf16 behaviour.  TEST
INFRASTRUCTURE ONLY: run in the build container (CPU), writes tests/golden/bf16_autocast.json.

The reference trains under torch.autocast (BASELINE configs[4]: "bf16"); the reference's G-step
and D-step (version5_model_train.py:350-405) are restated by oracle.model (pinned to the
reference's own outputs by tests/test_oracle_golden.py).  This script runs that restated step
twice on exactly the inputs of tests/test_gpu_configs.py::test_bf16_train_step_b32 -- B = 32
clips x 64 frames, audio randn(seed 21) * 2 - 3, pose synth.pose_targets(seed 22), G / D
weights weights.make_state_dict(seed 1234 / 1235), p = 0, fixed labels (0.93, 0.07) -- once in
fp32 and once under torch.autocast('cpu', dtype=torch.bfloat16) (convs, linears and matmuls in
bf16, BatchNorm / LayerNorm / softmax / losses in fp32: torch's own autocast policy), and
records what autocast does to the step: the G and D gradient cosines against fp32 (global over
the parameters whose true gradient is not identically zero, and the median over weight
tensors), the loss changes, and the pose error in train mode (batch statistics) and in eval
mode (running statistics) -- the figures the GPU test compares a2m's bf16 mode with.

    python -m oracle.make_autocast_fixture
"""
import json
import os
import re
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from oracle import model, synth, weights  # noqa: E402

GOLDEN = os.path.join(REPO, 'tests', 'golden')


def bn_cancelled(name):
    """Parameters whose true gradient is identically zero (a bias ahead of a train-mode
    BatchNorm, the key bias under the softmax): their computed gradient is rounding noise."""
    return name.endswith(('.conv.bias', '.conv_transpose.bias', '.key_conv.bias')) or \
        re.fullmatch(r'conv[123](\.\d)?\.(0|4|9)\.bias', name) is not None


def leaf(sd):
    return {k: v.clone().requires_grad_(v.is_floating_point() and 'running' not in k) for k, v in sd.items()}


def step(gsd, dsd, audio, pose, bf16):
    """One G-step and one D-step (version5_model_train.py:350-405, p = 0, fixed labels):
    (G grads, D grads, G_loss, D_loss, train-mode pose)."""
    B = audio.shape[0]
    valid, fake_l = torch.full((B, 4), 0.93), torch.full((B, 4), 0.07)
    ctx = torch.autocast('cpu', dtype=torch.bfloat16) if bf16 else torch.autocast('cpu', enabled=False)
    gs, ds = leaf(gsd), leaf(dsd)
    with ctx:
        fake, internal = model.generator(gs, audio, real_pose=pose, train=True)
        fd = model.discriminator(ds, torch.diff(fake, dim=1), train=True)
        l1, sm, jk = model.motion_terms(pose, fake)
        adv = torch.nn.functional.mse_loss(fd.float(), valid)
        g_loss = l1 + adv + 0.1 * sm + 0.05 * jk + internal[0] + internal[1]
    g_loss.backward()
    gg = {k: v.grad.detach().double().flatten().clone() for k, v in gs.items() if v.grad is not None}
    ds2 = leaf(dsd)
    with ctx:
        rd = model.discriminator(ds2, torch.diff(pose, dim=1), train=True)
        fd2 = model.discriminator(ds2, torch.diff(fake.detach(), dim=1), train=True)
        d_loss = torch.nn.functional.mse_loss(rd.float(), valid) + torch.nn.functional.mse_loss(fd2.float(), fake_l)
    d_loss.backward()
    dg = {k: v.grad.detach().double().flatten().clone() for k, v in ds2.items() if v.grad is not None}
    return gg, dg, g_loss.item(), d_loss.item(), fake.detach().float()


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
    torch.manual_seed(0)
    with open(os.path.join(GOLDEN, 'state_dict_keys.json')) as f:
        keys = json.load(f)
    gsd = {k: torch.from_numpy(np.asarray(v)) for k, v in weights.make_state_dict(keys['G'], seed=1234).items()}
    dsd = {k: torch.from_numpy(np.asarray(v)) for k, v in weights.make_state_dict(keys['D'], seed=1235).items()}
    gen = torch.Generator().manual_seed(21)
    audio = torch.randn(32, 64, 128, generator=gen) * 2.0 - 3.0
    pose = torch.from_numpy(synth.pose_targets(32, 64, seed=22))
    f32 = step(gsd, dsd, audio, pose, False)
    b16 = step(gsd, dsd, audio, pose, True)
    cg = agree(f32[0], b16[0], keys['G'])
    cd = agree(f32[1], b16[1], keys['D'])
    with torch.no_grad():
        pe32, _ = model.generator(gsd, audio, train=False)
        with torch.autocast('cpu', dtype=torch.bfloat16):
            pe16, _ = model.generator(gsd, audio, train=False)
    out = {
        'source': 'oracle/make_autocast_fixture.py: oracle.model G-step + D-step (version5_model_train.py:350-405 '
                  'restated), fp32 vs torch.autocast(cpu, bfloat16), inputs of test_bf16_train_step_b32',
        'torch': torch.__version__,
        'g_cos_global': cg[0], 'g_cos_weight_median': cg[1],
        'd_cos_global': cd[0], 'd_cos_weight_median': cd[1],
        'g_loss_fp32': f32[2], 'g_loss_bf16': b16[2], 'd_loss_fp32': f32[3], 'd_loss_bf16': b16[3],
        'pose_rel_err_train': rel(b16[4], f32[4]),
        'pose_rel_err_eval': rel(pe16.float(), pe32),
        'seconds': round(time.time() - t0, 1),
    }
    with open(os.path.join(GOLDEN, 'bf16_autocast.json'), 'w') as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
