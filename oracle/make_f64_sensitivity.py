"""TEST INFRASTRUCTURE — fp32-input-rounding sensitivity of the exact train-step gradients.

tests/test_gpu_train.py bounds every sampled gradient of the train-step fixtures against the
exact (fp64) gradient, as a multiple of the reference's own fp32 error there.  For a few
parameters that multiple is meaningless: the EXACT gradient itself moves by several percent of
its scale when the input is perturbed at fp32's rounding scale (relative 1e-7).  The GAT attention
vectors are the case in point -- their gradient is the remainder of an edge-softmax adjoint that
sums to zero over each destination, and at B = 2 one of body_gcn5's pre-activation logits sits at
8.8e-7 of its scale from the leaky-ReLU kink, so a 1e-7 input perturbation moves
body_gcn5.att_dst's exact gradient by 9 % of its scale.  Any fp32 implementation with another
summation order lands anywhere in that range; the reference's own 0.1 % there is one draw.

This script measures that sensitivity: the oracle in float64 (as oracle/make_f64_grads.py) on
the fixture's inputs with the audio multiplied by (1 + 1e-7 * N(0, 1)) for two seeds, and records
per parameter the largest change of the sampled gradient entries (absolute; the test divides by
the same scale it uses for the errors).

    python oracle/make_f64_sensitivity.py [train_step_b2t64 | train_step_b16t64]
        # writes tests/golden/<name>_f64_sens.npz
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, 'tests', 'golden')

from oracle import model  # noqa: E402
from oracle.make_f64_grads import _sample, _state  # noqa: E402

REL_NOISE = 1e-7
SEEDS = (1, 2)


def _grads(keys, t, z, noise_seed):
    """Sampled G-step and D-step gradients (make_f64_grads.main's step) on perturbed audio."""
    gs, ds = _state(keys['G'], 1234), _state(keys['D'], 1235)
    audio = torch.from_numpy(z['audio']).double()
    if noise_seed is not None:
        g = torch.Generator().manual_seed(noise_seed)
        audio = audio * (1.0 + REL_NOISE * torch.randn(audio.shape, generator=g))
    pose = torch.from_numpy(z['real_pose']).double()
    B = audio.shape[0]
    fake, internal = model.generator(gs, audio, real_pose=pose, train=True)
    fd = model.discriminator(ds, torch.diff(fake, dim=1), train=True)
    l1, sm, jk = model.motion_terms(pose, fake)
    loss = l1 + torch.nn.functional.mse_loss(fd, torch.full((B, 4), 0.93)) + 0.1 * sm + 0.05 * jk \
        + internal[0] + internal[1]
    loss.backward()
    gG = _sample(gs, t, 'gG')
    for v in ds.values():
        v.grad = None
    with torch.no_grad():
        fp2, _ = model.generator(gs, audio, train=True)
    fd2 = model.discriminator(ds, torch.diff(fp2, dim=1), train=True)
    rd2 = model.discriminator(ds, torch.diff(pose, dim=1), train=True)
    dl = torch.nn.functional.mse_loss(rd2, torch.full((B, 4), 0.93)) + \
        torch.nn.functional.mse_loss(fd2, torch.full((B, 4), 0.07))
    dl.backward()
    return gG, _sample(ds, t, 'gD')


def main(name='train_step_b2t64'):
    torch.set_default_dtype(torch.float64)
    with open(os.path.join(GOLDEN, 'state_dict_keys.json')) as f:
        keys = json.load(f)
    t = dict(np.load(os.path.join(GOLDEN, name + '.npz')))
    z = t if 'audio' in t else np.load(os.path.join(GOLDEN, 'g_eval_b2t64.npz'))
    f64 = np.load(os.path.join(GOLDEN, name + '_f64.npz'))
    g0, d0 = _grads(keys, t, z, None)
    # the unperturbed run must reproduce the committed exact gradients
    assert np.allclose(g0, f64['gG_val'], rtol=1e-9, atol=1e-14), 'gG differs from the _f64 fixture'
    assert np.allclose(d0, f64['gD_val'], rtol=1e-9, atol=1e-14), 'gD differs from the _f64 fixture'
    sg, sd = np.zeros(g0.shape[0]), np.zeros(d0.shape[0])
    for s in SEEDS:
        g1, d1 = _grads(keys, t, z, s)
        sg = np.maximum(sg, np.abs(g1 - g0).max(axis=1))
        sd = np.maximum(sd, np.abs(d1 - d0).max(axis=1))
    out = {'gG_sens': sg, 'gD_sens': sd, 'rel_noise': np.array(REL_NOISE), 'seeds': np.array(SEEDS)}
    np.savez_compressed(os.path.join(GOLDEN, name + '_f64_sens.npz'), **out)
    print('wrote', name + '_f64_sens.npz')


if __name__ == '__main__':
    main(*sys.argv[1:])
