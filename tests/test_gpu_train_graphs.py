"""The training iteration replayed from HIP graphs (GANTrainer(graphs=True)):
the G-step and D-step bodies of version5_model_train.py:350-405 (forward, losses, backward,
gradient gather, Adam) are captured once and replayed per step, with the reference's host
decisions (frequencies, learning rates, labels) between replays.

  - the replayed iterations equal the eager iterations bit for bit (p = 0, fixed labels), across
    a learning-rate change (the device lr FlatAdam reads) and an iteration that skips D;
  - dropout masks stay fresh per replay: a captured dropout launch whose seed is baked draws a
    new mask each replay through the device seed counter, and equals the eager launch at the
    same counter value;
  - with dropout on (p = 0.2 / 0.3, the bench configuration) the replayed iterations train:
    finite losses, the weights move, the counter advances once per step.
"""
import pytest
import torch

from test_gpu_configs import _models

pytestmark = pytest.mark.gpu
DEV = torch.device('cuda', 0)


def _batch(B, seed=31):
    from oracle import synth
    gen = torch.Generator().manual_seed(seed)
    audio = (torch.randn(B, 64, 128, generator=gen) * 2.0 - 3.0).to(DEV)
    pose = torch.from_numpy(synth.pose_targets(B, 64, seed=seed + 1)).to(DEV)
    return audio, pose


def _trainer(graphs, **kw):
    from a2m.training import GANTrainer
    g, d = _models(DEV)
    return GANTrainer(g, d, lr=1e-4, fixed_labels=(0.93, 0.07), graphs=graphs, **kw)


def test_graph_replay_equals_eager():
    """Six iterations (3 G + 1 D each; G captured at its third step, D at its third), an lr
    change before iteration 4 and a D-skipping iteration: parameters, Adam moments, running
    statistics and every loss bitwise equal to the eager trainer's."""
    audio, pose = _batch(8)
    runs = {}
    for graphs in (False, True):
        tr = _trainer(graphs)
        losses = []
        for it in range(6):
            if it == 3:
                for opt in (tr.opt_G, tr.opt_D):
                    opt.param_groups[0]['lr'] *= 0.5
            d_freq = 0 if it == 4 else 1
            dl, gl = tr.iteration(audio, pose, epoch=it, g_freq=3, d_freq=d_freq, sync_losses=False)
            losses.append((gl.item(), dl.item()))
        torch.cuda.synchronize()
        bufs = {n: b.detach().clone() for n, b in list(tr.G.named_buffers()) + list(tr.D.named_buffers())}
        runs[graphs] = dict(losses=losses, G=tr.opt_G.flat.clone(), D=tr.opt_D.flat.clone(),
                            mG=tr.opt_G.exp_avg_sq.clone(), mD=tr.opt_D.exp_avg.clone(), bufs=bufs,
                            steps=(tr.opt_G.step_count, tr.opt_D.step_count),
                            captured=(tr._captured['g'] is not None, tr._captured['d'] is not None))
    e, g = runs[False], runs[True]
    assert g['captured'] == (True, True)
    assert e['steps'] == g['steps'] == (18, 5), (e['steps'], g['steps'])
    assert e['losses'] == g['losses'], (e['losses'], g['losses'])
    for k in ('G', 'D', 'mG', 'mD'):
        assert torch.equal(e[k], g[k]), (k, (e[k] - g[k]).abs().max().item())
    for n, v in e['bufs'].items():
        assert torch.equal(v, g['bufs'][n]), n


def test_graph_dropout_masks_fresh_per_replay():
    """A dropout launch captured with its seed baked: each replay (counter + 1 inside the graph)
    draws a different mask, and replay k equals the eager launch at counter value k."""
    from a2m import functional as F
    x = torch.ones(1 << 16, device=DEV)
    ctr = torch.zeros(1, dtype=torch.int64, device=DEV)
    seed = 0x1234567
    g = torch.cuda.CUDAGraph()
    F.set_dropout_seed_offset(ctr)
    try:
        F.dropout(x, 0.3, seed)   # warm-up outside the capture
        with torch.cuda.graph(g):
            ctr.add_(1)
            y = F.dropout(x, 0.3, seed)
    finally:
        F.set_dropout_seed_offset(None)
    ctr.zero_()
    outs = []
    for _ in range(3):
        g.replay()
        outs.append(y.clone())
    torch.cuda.synchronize()
    assert ctr.item() == 3
    for a in outs:
        frac = (a == 0).float().mean().item()
        assert 0.28 < frac < 0.32, frac
    assert not torch.equal(outs[0], outs[1]) and not torch.equal(outs[1], outs[2])
    # eager at the same counter values
    for k, a in enumerate(outs, start=1):
        ctr.fill_(k)
        F.set_dropout_seed_offset(ctr)
        try:
            ref = F.dropout(x, 0.3, seed)
        finally:
            F.set_dropout_seed_offset(None)
        assert torch.equal(ref, a), k
    # no counter registered: the plain seed (eager bits unchanged)
    assert torch.equal(F.dropout(x, 0.3, seed), F.dropout(x, 0.3, seed))


def test_graph_training_with_dropout():
    """The bench configuration (p = 0.2 in G, 0.3 in D, noisy labels) on replayed graphs."""
    from a2m.real_motion_model import SelfAttention_D, SelfAttention_G
    from a2m.training import GANTrainer
    torch.manual_seed(5)
    g = SelfAttention_G(time_steps=64, p=0.2).to(DEV).train()
    d = SelfAttention_D(out_channels=64).to(DEV).train()
    tr = GANTrainer(g, d, lr=1e-4, label_seed=7, graphs=True)
    audio, pose = _batch(8)
    w0 = tr.opt_G.flat.clone()
    hist = []
    for it in range(4):
        dl, gl = tr.iteration(audio, pose, epoch=it, g_freq=3, d_freq=1)
        hist.append((gl.item(), dl.item()))
    torch.cuda.synchronize()
    assert tr._captured['g'] is not None and tr._captured['d'] is not None
    assert all(torch.isfinite(torch.tensor(h)).all() for h in hist), hist
    assert not torch.equal(w0, tr.opt_G.flat)
    # one counter step per G / D step: 12 G + 4 D
    assert tr._seed_ctr.item() == 16, tr._seed_ctr.item()
    assert len(tr.dyn.d_loss_history) == 4
