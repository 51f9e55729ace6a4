"""How far apart do two exact-arithmetic-equivalent runs of the reference loop body get?

Runs version5_model_train.py:350-405 (3 G-steps, 1 D-step, torch.optim.Adam lr 1e-3, p=0,
fixed labels) on the fp32 and the fp64 oracle (CPU) from the same weights and inputs as
tests/golden/loop_b16t64.npz, and prints the relative spread of every loss and of the pose
after the iteration.  That spread is what rounding alone does to the loop; the GPU loop test
bounds are set from it.

    python tools/loop_spread.py [B]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))

from conftest import golden, golden_keys  # noqa: E402
from oracle import model, weights  # noqa: E402


def run(dtype, B):
    torch.set_default_dtype(dtype)
    keys = golden_keys()
    t = golden('train_step_b16t64.npz')
    audio = torch.from_numpy(t['audio'][:B]).to(dtype)
    real_pose = torch.from_numpy(t['real_pose'][:B]).to(dtype)
    gs = {k: (v.to(dtype) if v.is_floating_point() else v) for k, v in weights.make_state_dict(keys['G'], 1234).items()}
    ds = {k: (v.to(dtype) if v.is_floating_point() else v) for k, v in weights.make_state_dict(keys['D'], 1235).items()}
    gp = [v.requires_grad_(True) for k, v in gs.items() if v.is_floating_point() and 'running' not in k]
    dp = [v.requires_grad_(True) for k, v in ds.items() if v.is_floating_point() and 'running' not in k]
    opt_g, opt_d = torch.optim.Adam(gp, lr=10e-4), torch.optim.Adam(dp, lr=10e-4)
    valid, fake = torch.full((B, 4), 0.93), torch.full((B, 4), 0.07)
    real_motion = torch.diff(real_pose, dim=1)
    gl = []
    for _ in range(3):
        opt_g.zero_grad()
        fp, internal = model.generator(gs, audio, real_pose=real_pose, train=True)
        fm = torch.diff(fp, dim=1)
        fd = model.discriminator(ds, fm, train=True)
        l1, sm, jk = model.motion_terms(real_pose, fp)
        loss = l1 + torch.nn.functional.mse_loss(fd, valid) + 0.1 * sm + 0.05 * jk + internal[0] + internal[1]
        loss.backward()
        opt_g.step()
        gl.append(loss.item())
    opt_d.zero_grad()
    with torch.no_grad():
        fp2, _ = model.generator(gs, audio, train=True)
    fd2 = model.discriminator(ds, torch.diff(fp2, dim=1).detach(), train=True)
    rd2 = model.discriminator(ds, real_motion, train=True)
    dl = torch.nn.functional.mse_loss(rd2, valid) + torch.nn.functional.mse_loss(fd2, fake)
    dl.backward()
    opt_d.step()
    with torch.no_grad():
        after, _ = model.generator(gs, audio, train=True)
    return np.array(gl), dl.item(), after.double().numpy()


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    g32, d32, a32 = run(torch.float32, B)
    g64, d64, a64 = run(torch.float64, B)
    print('G losses fp32', g32, 'fp64', g64, 'rel', np.abs(g32 - g64) / np.abs(g64))
    print('D loss rel', abs(d32 - d64) / abs(d64))
    print('pose after rel (max|d| / max|ref|)', np.abs(a32 - a64).max() / np.abs(a64).max())
    if B == 16:
        ref = golden('loop_b16t64.npz')
        print('reference fp32 vs oracle fp32: G', np.abs(ref['g_losses'] - g32) / np.abs(g32),
              'pose after', np.abs(ref['fake_pose_after'] - a32).max() / np.abs(a32).max())


if __name__ == '__main__':
    main()
