"""Data-parallel GAN step on CPU: two gloo ranks, each on half the clips.
After one GANTrainer iteration the all-reduced G and D gradients must equal the single-process
whole-batch gradients, and the loss history must match.  After further iterations both ranks
must hold bitwise-identical parameters and loss histories (so every rank takes the same
DynamicGANTraining branches).

The HIP kernels cannot run here, so the test swaps the trainer's device ops for their oracle
equivalents (torch-CPU restatements of version5_model_train.py:208-248 and torch.optim.Adam)
and uses small torch G/D models with the reference's call contract.  What is under test is
the host-side DP logic: flat-gradient all-reduce, loss synchronisation, D frozen in the
G-steps, optimiser bookkeeping.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

B, T, FD = 8, 16, 104


class TinyG(torch.nn.Module):
    """Several parameters, so a small bucket size cuts the flat gradient into many buckets."""

    def __init__(self):
        super().__init__()
        self.inp = torch.nn.Linear(128, 48)
        self.mid = torch.nn.ModuleList([torch.nn.Linear(48, 48) for _ in range(3)])
        self.lin = torch.nn.Linear(48, FD)

    def forward(self, audio, real_pose=None):
        h = torch.tanh(self.inp(audio))
        for m in self.mid:
            h = torch.tanh(m(h)) + h
        pose = self.lin(h)
        internal = [(pose ** 2).mean() * 1e-3]
        if real_pose is not None:
            internal.insert(0, (pose - real_pose).abs().mean() * 1e-2)
        return pose, internal


class TinyD(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.lin = torch.nn.Linear(FD, 1)
        self.aux = torch.nn.Linear(8, 3)   # never used in forward, like SelfAttention_D's aux head

    def forward(self, x, audio=None, aux_labels=None):
        y = self.lin(x)                            # [B, T-1, 1]
        return y[:, :4, 0], []


def _patch_ops():
    """Oracle stand-ins for the trainer's HIP ops (test-only)."""
    from a2m import autograd as AG
    from a2m import functional as F
    from oracle import model as OM

    def motion_terms(fake, real):
        return torch.stack(OM.motion_terms(real, fake))

    def adam_(p, g, m, v, lr, b1, b2, eps, wd, step):
        m.mul_(b1).add_(g, alpha=1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        denom = (v / (1 - b2 ** step)).sqrt_().add_(eps)
        p.addcdiv_(m, denom, value=-lr / (1 - b1 ** step))

    AG.pos_to_motion = lambda x: torch.diff(x, dim=1)
    AG.motion_terms = motion_terms
    AG.mse_loss = torch.nn.functional.mse_loss
    F.adam_ = adam_
    def gather_segments_(dst, segs):
        for o, t in segs:
            dst[o:o + t.numel()].copy_(t.reshape(-1))
        return dst

    F.gather_segments_ = gather_segments_


def _data():
    g = torch.Generator().manual_seed(3)
    return torch.randn(B, T, 128, generator=g), torch.randn(B, T, FD, generator=g)


def _models():
    torch.manual_seed(11)
    return TinyG(), TinyD()


CONFIGS = {
    # round-1 behaviour: fixed labels, one bucket per network
    'fixed': dict(fixed_labels=(0.93, 0.07)),
    # bucketed overlapped reduce (buckets of ~2.3k floats, several per network) and smoothed
    # noisy labels drawn for the global batch from the shared generator and sliced per rank
    'buckets': dict(bucket_mb=0.009, label_seed=5),
    # the same with bf16 buckets on the wire (configs[4])
    'bf16': dict(bucket_mb=0.009, label_seed=5, grad_reduce_dtype=torch.bfloat16),
}


def _run(rank, world, cfg='fixed'):
    from a2m.training import GANTrainer
    _patch_ops()
    G, D = _models()
    tr = GANTrainer(G, D, lr=1e-2, **CONFIGS[cfg])
    if world > 1 and cfg != 'fixed':
        assert len(tr.red_G.buckets) > 3 and len(tr.red_D.buckets) >= 1
    audio, pose = _data()
    if world > 1:
        shard = B // world
        audio, pose = audio[rank * shard:(rank + 1) * shard], pose[rank * shard:(rank + 1) * shard]
    tr.iteration(audio, pose, epoch=0, g_freq=1, d_freq=1)
    grads = (tr.opt_G.flat_grad.clone(), tr.opt_D.flat_grad.clone(),
             list(tr.dyn.d_loss_history), list(tr.dyn.g_loss_history))
    for epoch in range(1, 3):
        tr.iteration(audio, pose, epoch=epoch, g_freq=3, d_freq=1)
    params = (tr.opt_G.flat.clone(), tr.opt_D.flat.clone(), list(tr.dyn.d_loss_history),
              list(tr.dyn.g_loss_history))
    if world > 1 and cfg != 'fixed':
        # after the first backward the reducer knows which parameters get gradients: every
        # G bucket but the last launches from a grad hook while the backward is still running
        # (the last one completes with the final gradient, i.e. when the backward ends)
        assert tr.red_G.in_backward >= len(tr.red_G.buckets) - 1, (tr.red_G.in_backward, len(tr.red_G.buckets))
    return grads, params


def _plain(res):
    """numpy copies: torch tensors sent through a Queue need the sender alive."""
    return tuple(tuple(x.numpy() if torch.is_tensor(x) else x for x in part) for part in res)


def _worker(rank, world, port, q, cfg='fixed'):
    if world == 1:                    # single-process reference, no process group
        q.put(('ref', _plain(_run(0, 1, cfg))))
        return
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        q.put((rank, _plain(_run(rank, world, cfg))))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


@pytest.mark.timeout(300)
@pytest.mark.parametrize('cfg', ['fixed', 'buckets', 'bf16'])
def test_dp_two_ranks_matches_single_process(cfg):
    """Two ranks on half the batch each == one process on the whole batch: gradients after
    the all-reduce (first iteration), loss histories, then bitwise-identical replicas.  With
    bf16 buckets the gradients carry bf16 rounding (8 significant bits)."""
    # every run happens in a spawned child: the op stand-ins never leak into this process
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(0, 1, port, q, cfg))]
    procs += [ctx.Process(target=_worker, args=(r, 2, port, q, cfg)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    ref = res['ref']
    (rg, rd, rdh, rgh), _ = ref
    tol = 8e-3 if cfg == 'bf16' else 1e-5
    for r in (0, 1):
        (g, d, dh, gh), _ = res[r]
        assert abs(g - rg).max() <= tol * abs(rg).max(), ('G grad', r, abs(g - rg).max() / abs(rg).max())
        assert abs(d - rd).max() <= tol * abs(rd).max(), ('D grad', r)
        ltol = 1e-3 if cfg == 'bf16' else 1e-5   # the D loss follows a bf16-reduced G update
        assert dh == pytest.approx(rdh, rel=ltol) and gh == pytest.approx(rgh, rel=ltol)
    p0, p1 = res[0][1], res[1][1]
    assert (p0[0] == p1[0]).all() and (p0[1] == p1[1]).all()         # bitwise-identical replicas
    assert p0[2] == p1[2] and p0[3] == p1[3]                        # identical branch inputs


def _syncbn_worker(rank, world, port, q):
    """SyncBN host plumbing over a real gloo group: the group seen by the BN wrappers during a
    GANTrainer(sync_bn=True) iteration, the float64 SUM all-reduce, and restoration after."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from a2m import functional as F
        from a2m.training import GANTrainer
        _patch_ops()
        seen = []

        class RecG(TinyG):
            def forward(self, audio, real_pose=None):
                seen.append(F._sync_world())
                return super().forward(audio, real_pose)

        torch.manual_seed(11)
        tr = GANTrainer(RecG(), TinyD(), lr=1e-2, fixed_labels=(0.93, 0.07), sync_bn=True)
        audio, pose = _data()
        tr.iteration(audio[rank::world], pose[rank::world], epoch=0, g_freq=1, d_freq=1)
        after = F._sync_world()
        prev = F.set_sync_bn_group(dist.group.WORLD)
        t = torch.tensor([[1.5 + rank, 2.0 * rank]], dtype=torch.float64)
        F._allreduce_sum_(t)
        F.set_sync_bn_group(prev)
        q.put((rank, (tr.sync_bn, seen, after, t.tolist())))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_syncbn_plumbing_two_ranks():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_syncbn_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    for r in (0, 1):
        sync_bn, seen, after, t = res[r]
        assert sync_bn and seen and all(w == 2 for w in seen)   # every BN in the step sees 2 ranks
        assert after == 0                                       # per-rank statistics restored
        assert t == [[1.5 + 2.5, 2.0]]                          # SUM over the ranks, float64


def _mismatch_worker(rank, world, port, q, bad_step=1, check_every=None, flush=False):
    """Rank 1 sends a gradient through a parameter outside the learnt set on step `bad_step`
    (0-based iteration): both ranks must raise together (no rank left waiting in a bucket
    all-reduce) -- at once on the synchronously checked first steps, at the next periodic check
    (GradReducer.CHECK_EVERY) or at GANTrainer.flush() after them."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from a2m.training import GANTrainer
        _patch_ops()

        class BranchG(TinyG):
            use_extra = False

            def __init__(self):
                super().__init__()
                self.extra = torch.nn.Linear(48, 48)

            def forward(self, audio, real_pose=None):
                if self.use_extra:
                    audio = audio.clone()
                    pose, internal = super().forward(audio, real_pose)
                    return pose + self.extra.weight.sum() * 0, internal
                return super().forward(audio, real_pose)

        torch.manual_seed(11)
        g = BranchG()
        tr = GANTrainer(g, TinyD(), lr=1e-2, fixed_labels=(0.93, 0.07), bucket_mb=0.009)
        if check_every:
            tr.red_G.CHECK_EVERY = tr.red_D.CHECK_EVERY = check_every
        audio, pose = _data()
        at = None
        try:
            for it in range(bad_step + 4):
                g.use_extra = rank == 1 and it == bad_step
                at = it
                tr.iteration(audio[rank::world], pose[rank::world], epoch=it, g_freq=1, d_freq=1)
            at = 'flush'
            if flush:
                tr.flush()
            q.put((rank, 'no error'))
        except RuntimeError as e:
            q.put((rank, f'raised at {at}: ' + str(e)[:60]))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize('bad_step,check_every,flush,where', [
    (1, None, False, 1),          # a synchronously checked step: raises in that step
    (3, 2, False, 4),             # G's 4th finish() is a check step (4 % 2): read at the next finish()
    (3, 50, True, 'flush')])      # no check before the end: GANTrainer.flush() raises
def test_grad_reducer_mismatch_raises_on_every_rank(bad_step, check_every, flush, where):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mismatch_worker, args=(r, 2, port, q, bad_step, check_every, flush))
             for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    assert all(v.startswith(f'raised at {where}: GradReducer') for v in res.values()), res


def _seed_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from a2m.training import GANTrainer
        _patch_ops()
        torch.manual_seed(100 + rank)       # ranks differ; rank 0's seed must win
        tr = GANTrainer(TinyG(), TinyD(), lr=1e-2)
        real, fake = tr._labels(0, 4, torch.device('cpu'))
        q.put((rank, (real.numpy(), fake.numpy())))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_label_seed_follows_rank0_manual_seed():
    """label_seed=None: the labels follow torch.manual_seed (the reference draws them from the
    global RNG), and every rank slices the same global-batch draw (rank 0's seed)."""
    from a2m.training import DynamicGANTraining
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_seed_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(30)
        assert p.exitcode == 0
    gen = torch.Generator().manual_seed(100)
    dyn = DynamicGANTraining(g_lr=5e-3, d_lr=1e-2)
    real = dyn.get_smooth_labels(0, 8, 'cpu', True, generator=gen).numpy()
    fake = dyn.get_smooth_labels(0, 8, 'cpu', False, generator=gen).numpy()
    for r in (0, 1):
        assert (res[r][0] == real[4 * r:4 * r + 4]).all() and (res[r][1] == fake[4 * r:4 * r + 4]).all()
