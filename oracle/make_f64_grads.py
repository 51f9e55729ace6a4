"""TEST INFRASTRUCTURE — fp64 gradients for the train-step fixture.

The reference's fp32 gradients of the deepest generator layers (the audio encoder, ~60
layers below the loss, through 20 training-mode BatchNorms) carry 0.2-0.5 % rounding
error of their own relative to the exact gradient; an fp32 GPU implementation with a
different summation order lands an independent ~0.5 % away, so "GPU vs reference fp32"
cannot be held to a few 1e-3 there.  This script evaluates the oracle (pinned to the
reference in fp32 by tests/test_oracle_golden.py) in float64 at the SAME sampled indices
as tests/golden/train_step_b2t64.npz, so the GPU test can measure both implementations
against the exact gradient: the GPU must be as close to it as the reference itself is.

    python oracle/make_f64_grads.py [train_step_b2t64 | train_step_b16t64]
        # writes tests/golden/<name>_f64.npz (default train_step_b2t64)
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, 'tests', 'golden')

from oracle import model, weights  # noqa: E402


def _state(keys, seed):
    sd = weights.make_state_dict(keys, seed=seed)
    out = {}
    for k, v in sd.items():
        v = v.double() if v.is_floating_point() else v
        if v.is_floating_point() and 'running' not in k:
            v.requires_grad_(True)
        out[k] = v
    return out


def _sample(state, t, prefix):
    vals = []
    for i, n in enumerate(t[f'{prefix}_names']):
        g = state[str(n)].grad
        g = g.reshape(-1).numpy() if g is not None else np.zeros(state[str(n)].numel())
        ix = t[f'{prefix}_idx'][i]
        vals.append(np.where(ix >= 0, g[np.maximum(ix, 0)], 0.0))
    return np.stack(vals)


def main(name='train_step_b2t64'):
    torch.set_default_dtype(torch.float64)
    with open(os.path.join(GOLDEN, 'state_dict_keys.json')) as f:
        keys = json.load(f)
    t = dict(np.load(os.path.join(GOLDEN, name + '.npz')))
    z = t if 'audio' in t else np.load(os.path.join(GOLDEN, 'g_eval_b2t64.npz'))
    gs, ds = _state(keys['G'], 1234), _state(keys['D'], 1235)
    audio = torch.from_numpy(z['audio']).double()
    pose = torch.from_numpy(z['real_pose']).double()
    B = audio.shape[0]
    fake, internal = model.generator(gs, audio, real_pose=pose, train=True)
    fd = model.discriminator(ds, torch.diff(fake, dim=1), train=True)
    l1, sm, jk = model.motion_terms(pose, fake)
    loss = l1 + torch.nn.functional.mse_loss(fd, torch.full((B, 4), 0.93)) + 0.1 * sm + 0.05 * jk \
        + internal[0] + internal[1]
    loss.backward()
    out = {'gG_val': _sample(gs, t, 'gG'), 'G_loss': loss.detach().numpy()}
    for v in ds.values():
        v.grad = None
    with torch.no_grad():
        fp2, _ = model.generator(gs, audio, train=True)
    fd2 = model.discriminator(ds, torch.diff(fp2, dim=1), train=True)
    rd2 = model.discriminator(ds, torch.diff(pose, dim=1), train=True)
    dl = torch.nn.functional.mse_loss(rd2, torch.full((B, 4), 0.93)) + \
        torch.nn.functional.mse_loss(fd2, torch.full((B, 4), 0.07))
    dl.backward()
    out.update(gD_val=_sample(ds, t, 'gD'), D_loss=dl.detach().numpy())
    rel = abs(dl.item() - float(t['D_loss'])) / abs(float(t['D_loss']))
    assert rel < 1e-4, f'fp64 D loss disagrees with the reference fixture: {rel}'
    np.savez_compressed(os.path.join(GOLDEN, name + '_f64.npz'), **out)
    print('wrote', name + '_f64.npz', {k: v.shape for k, v in out.items()})


if __name__ == '__main__':
    main(*sys.argv[1:])
