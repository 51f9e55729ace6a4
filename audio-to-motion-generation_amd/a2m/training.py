"""The per-clip GAN training step of version5_model_train.py on the HIP path, data-parallel
over clips with one process per GPU.

  DynamicGANTraining   version5_model_train.py:12-180 (host-side schedule: G/D step counts,
                       learning-rate adaptation, smoothed noisy labels)
  pos_to_motion        :208-213        compute_temporal_smoothness_loss :216-230
  compute_jerk_loss    :233-248        one iteration (G steps, then D steps) :342-414

Data parallelism: every rank runs the step on its shard of the batch.
Gradients of the network being stepped are averaged by GradReducer: the optimiser's flat
gradient buffer is cut into buckets in reverse parameter order (the order backward produces
them); a bucket closes once it holds at least bucket_mb (25 MB by default), and each bucket's all-reduce (RCCL over xGMI on MI355X, gloo in CPU tests)
is launched from a post-accumulate-grad hook as soon as its last gradient lands, so it runs
on the communication stream while the rest of the backward computes.  Buckets launch strictly
in order, so every rank issues the same collective sequence.  Optionally the buckets travel
in bf16 (configs[4]).  The two scalar losses are averaged before they enter the schedule so
every rank takes identical branches; smoothed labels are drawn for the global batch from a
generator seeded identically on every rank and sliced per rank.  BatchNorm uses per-rank
batch statistics by default (PyTorch DDP default) or SyncBN.  The discriminator's parameters
are frozen during the G steps: the reference computes their gradients there and throws them
away (optimizer_D.zero_grad() at :388).
"""
import contextlib
import time

import numpy as np
import torch
import torch.distributed as dist

from . import autograd as AG
from . import functional as F
from .optim import FlatAdam, flat_order


class DynamicGANTraining:
    def __init__(self, g_lr=5e-6, d_lr=10e-6):
        self.g_lr_initial = self.g_lr_current = g_lr
        self.d_lr_initial = self.d_lr_current = d_lr
        self.d_loss_history, self.g_loss_history = [], []
        self.d_strong_threshold, self.g_weak_threshold, self.g_strong_threshold = 0.20, 0.80, 0.10
        self.d_train_freq, self.g_train_freq = 1, 3
        self.min_d_freq, self.max_d_freq, self.min_g_freq, self.max_g_freq = 1, 2, 2, 6
        self.real_label_smooth, self.fake_label_smooth = 0.98, 0.02
        self.dynamic_smooth = False
        self.verbose = False

    def _say(self, msg):
        if self.verbose:
            print(msg)

    def update_loss_history(self, d_loss, g_loss):
        self.d_loss_history = (self.d_loss_history + [d_loss])[-100:]
        self.g_loss_history = (self.g_loss_history + [g_loss])[-100:]

    def get_recent_avg_loss(self, window=10):
        d, g = self.d_loss_history, self.g_loss_history
        if len(d) >= window:
            d, g = d[-window:], g[-window:]
        return np.mean(d), np.mean(g)

    def should_train_discriminator(self):
        if not self.d_loss_history:
            return True
        d, g = self.get_recent_avg_loss()
        return not (d < self.d_strong_threshold and g > self.g_weak_threshold)

    def adjust_training_frequency(self, epoch):
        if len(self.d_loss_history) >= 10:
            d, g = self.get_recent_avg_loss()
            ratio = d / (g + 1e-8)
            if ratio < 0.15 or d < 0.1:
                self.d_train_freq = max(1, self.d_train_freq - 1)
                self.g_train_freq = min(self.max_g_freq, self.g_train_freq + 1)
                self._say(f'D too strong: G={self.g_train_freq}, D={self.d_train_freq}')
            elif ratio > 2.5:
                self.d_train_freq = min(self.max_d_freq, self.d_train_freq + 1)
                self.g_train_freq = max(self.min_g_freq, self.g_train_freq - 1)
                self._say(f'G too strong: G={self.g_train_freq}, D={self.d_train_freq}')
        return self.g_train_freq, self.d_train_freq

    def adjust_learning_rates(self, optimizer_g, optimizer_d, epoch):
        if len(self.d_loss_history) < 10:
            g_lr, d_lr = self.g_lr_initial, self.d_lr_initial
        else:
            d, g = self.get_recent_avg_loss()
            if d < self.d_strong_threshold:
                self.d_lr_current *= 0.9
                self.g_lr_current *= 1.05
            elif d > 0.65 and g < 0.3:
                self.d_lr_current *= 1.05
                self.g_lr_current *= 0.9
            g_lr, d_lr = self.g_lr_current, self.d_lr_current
        for grp in optimizer_g.param_groups:
            grp['lr'] = g_lr
        for grp in optimizer_d.param_groups:
            grp['lr'] = d_lr

    def get_smooth_labels(self, epoch, batch_size, device, is_real=True, generator=None):
        """Annealed smoothed labels with Gaussian noise (version5_model_train.py:137-180): the
        noise std falls linearly 0.01 -> 0.002 over epochs 0..60, the label value starts 0.05
        further from 0/1; with dynamic_smooth a strong D (G) widens the real (fake) labels.
        Same draw as the reference (torch.normal over [B, 4]), so a shared seed gives the same
        labels; DP ranks draw the global batch from a shared generator and slice their shard."""
        if epoch < 0:
            progress, noise_std = 0.0, 0.01
        elif epoch > 60:
            progress, noise_std = 1.0, 0.002
        else:
            progress = epoch / 60
            noise_std = 0.01 - progress * (0.01 - 0.002)
        recent_d, recent_g = self.get_recent_avg_loss() if len(self.d_loss_history) >= 10 else (0.5, 0.5)
        if is_real:
            val, lo, hi = self.real_label_smooth - 0.05 * (1 - progress), 0.85, 1.0
            if self.dynamic_smooth and recent_d < self.d_strong_threshold:
                val, noise_std = max(0.97, val - 0.1), noise_std + 0.01
        else:
            val, lo, hi = self.fake_label_smooth + 0.05 * (1 - progress), 0.0, 0.15
            if self.dynamic_smooth and recent_g < self.g_strong_threshold:
                val, noise_std = min(0.03, val + 0.1), noise_std + 0.01
        labels = torch.ones(batch_size, 4, device=device).fill_(val)
        noise = torch.normal(0, noise_std, labels.shape, device=device, generator=generator)
        return torch.clamp(labels + noise, lo, hi).requires_grad_(False)


def pos_to_motion(pose):
    return AG.pos_to_motion(pose)


def compute_temporal_smoothness_loss_and_jerk(fake_pose, real_pose):
    """[L1(real motion, fake motion), smoothness, jerk] from POSES (fused kernel)."""
    return AG.motion_terms(fake_pose, real_pose)


class GradReducer:
    """Bucketed, backward-overlapped gradient averaging over a FlatAdam's flat gradient.

    Buckets are contiguous slices of `opt.flat_grad` holding whole parameters, filled from the
    last parameter backwards (~bucket_mb each).  A post-accumulate-grad hook on every parameter
    counts arrivals; when a bucket's last expected gradient has landed, the bucket's gradients
    are gathered into its slice (one segment-gather launch) and an async all-reduce of the slice
    is started -- but only in bucket order, so all ranks issue identical collective sequences.
    The set of parameters that receive gradients is learnt on the first backward (which reduces
    everything at finish()); afterwards a parameter arriving in an already launched bucket is an
    error, never a silent miss.  finish() gathers and reduces what is left, waits, and divides
    by the world size.  reduce_dtype=torch.bfloat16 halves the bytes on the wire (configs[4]).
    force=True arms the reducer also for a one-rank group (the RCCL path exercised on one GPU,
    tests/test_gpu_rccl.py).

    Plan checks: the ranks agree, through a small MAX all-reduce of an error flag, that no rank
    saw a gradient outside the plan and that all learnt the same parameter set, so a violation
    fails every rank together instead of leaving one blocked in a bucket all-reduce.  That
    collective runs on the first SYNC_CHECK_STEPS steps (read back at once: a device sync) and
    then only every CHECK_EVERY steps, read back at the next finish() so the host keeps running
    ahead; a violation seen in between is kept (sticky) and raised at the next check on every
    rank.  flush() runs a check now and reads it -- call it where the ranks must agree that
    training was sound (end of training, before a checkpoint: GANTrainer.flush()).
    """

    SYNC_CHECK_STEPS = 2
    CHECK_EVERY = 50

    def __init__(self, opt, world, group=None, bucket_mb=25.0, reduce_dtype=None, force=False):
        self.opt, self.world, self.group = opt, world, group
        self.force = force
        self.reduce_dtype = reduce_dtype
        self.steps = 0
        self._pending_flag = None
        self._sticky_error = None  # a violation seen since the last check
        spans = list(opt._spans())
        cap = max(int(bucket_mb * (1 << 20) / 4), 1)
        # buckets tile [0, numel) of the flat gradient (alignment padding included: it stays
        # zero), closed from the end of the buffer towards its start
        self.buckets = []          # (lo, hi, member parameter indices), in launch order
        hi, cur = opt.flat_grad.numel(), []
        for i in reversed(range(len(spans))):
            cur.append(i)
            if hi - spans[i][0] >= cap or i == 0:
                lo = 0 if i == 0 else spans[i][0]
                self.buckets.append((lo, hi, cur))
                hi, cur = lo, []
        self.bucket_of = {}
        for b, (_, _, members) in enumerate(self.buckets):
            for i in members:
                self.bucket_of[i] = b
        self.expected = None       # learnt: parameter indices that receive gradients
        self._hooks = [p.register_post_accumulate_grad_hook(self._make_hook(i))
                       for i, p in enumerate(opt.params)]
        self._reset()

    def _reset(self):
        self.arrived = set()
        self.pending = [None] * len(self.buckets)
        if self.expected is not None:
            self.pending = [sum(1 for i in m if i in self.expected) for _, _, m in self.buckets]
        self.next = 0
        self.handles = []
        self.active = False
        self.in_backward = 0       # buckets launched from hooks, i.e. overlapped with backward
        self.error = None

    def begin(self):
        """Arm the hooks for one backward (call after zero_grad, before backward)."""
        self._reset()
        self.active = self.world > 1 or self.force

    def _make_hook(self, i):
        def hook(p):
            if not self.active:
                return
            self.arrived.add(i)
            if self.expected is None:
                return
            b = self.bucket_of[i]
            if i not in self.expected or b < self.next:
                # not raised here: the other ranks would block in their next bucket's
                # all-reduce.  finish() launches every bucket in order regardless, then all
                # ranks agree on the error and raise together
                self.error = (f'GradReducer: gradient of parameter {i} arrived after its bucket '
                              f'was reduced (the set of parameters with gradients changed)')
                return
            self.pending[b] -= 1
            while self.next < len(self.buckets) and self.pending[self.next] == 0:
                self._launch(self.next)
                self.next += 1
                self.in_backward += 1
        return hook

    def _gather(self, b):
        o_spans = list(self.opt._spans())
        segs, seat = [], []
        for i in self.buckets[b][2]:
            p = self.opt.params[i]
            o, k = o_spans[i]
            view = self.opt.flat_grad[o:o + k]
            if p.grad is None:
                seat.append((p, view))
            elif p.grad.data_ptr() != view.data_ptr():
                segs.append((o, p.grad.contiguous()))
                seat.append((p, view))
        F.gather_segments_(self.opt.flat_grad, segs)
        for p, view in seat:
            p.grad = view.view_as(p)

    def _launch(self, b):
        self._gather(b)
        lo, hi, _ = self.buckets[b]
        sl = self.opt.flat_grad[lo:hi]
        buf = sl if self.reduce_dtype is None else sl.to(self.reduce_dtype)
        work = dist.all_reduce(buf, group=self.group, async_op=True)
        self.handles.append((sl, buf, work))

    @torch.no_grad()
    def finish(self):
        """Reduce the buckets not yet launched, wait for all, average.  Returns flat_grad.
        Inside a HIP-graph capture (GANTrainer(graphs=True)) the plan is frozen: every replay
        issues exactly the captured bucket all-reduces in the captured order on every rank, so
        the host-side plan checks (which read a flag back) are skipped there; a capture with a
        plan violation raises here at once."""
        if not self.active:
            self.opt.collect_grads()
            return self.opt.flat_grad
        capturing = torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
        while self.next < len(self.buckets):
            self._launch(self.next)
            self.next += 1
        if self.expected is None:
            self.expected = set(self.arrived)
        elif self.error is None and not self.arrived <= self.expected:
            self.error = 'GradReducer: parameters outside the learnt set received gradients'
        for sl, buf, work in self.handles:
            work.wait()
            if buf is not sl:
                sl.copy_(buf)
        if capturing:
            self.active = False
            if self.error:
                raise RuntimeError(self.error)
            if self.world > 1:
                self.opt.flat_grad.div_(self.world)
            return self.opt.flat_grad
        if self.error and self._sticky_error is None:
            self._sticky_error = self.error
        self.steps += 1
        self.active = False
        # every rank has issued the same bucket sequence; on check steps, agree on whether any
        # rank saw a gradient outside the plan (or learnt a different parameter set)
        prev, self._pending_flag = self._pending_flag, None
        if prev is not None:
            self._check_flag(prev)
        if self.steps <= self.SYNC_CHECK_STEPS:
            self._check_flag(self._flag())
        elif self.steps % self.CHECK_EVERY == 0:
            self._pending_flag = self._flag()
        if self.world > 1:
            self.opt.flat_grad.div_(self.world)
        return self.opt.flat_grad

    def _flag(self):
        n = len(self.expected) if self.expected is not None else 0
        flag = torch.tensor([1.0 if self._sticky_error else 0.0, n, -n], dtype=torch.float64,
                            device=self.opt.flat_grad.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self.group)
        return flag

    @torch.no_grad()
    def flush(self):
        """Collective (every rank at the same point): read any outstanding check, run one now,
        raise on every rank if any saw a violation since the last check."""
        if not (self.world > 1 or self.force) or self.expected is None:
            return
        prev, self._pending_flag = self._pending_flag, None
        if prev is not None:
            self._check_flag(prev)
        self._check_flag(self._flag())

    def _check_flag(self, flag):
        f = flag.tolist()
        if f[0] > 0 or f[1] != -f[2]:
            self._pending_flag = None
            msg = self._sticky_error or self.error
            self._sticky_error = None
            raise RuntimeError(msg or 'GradReducer: a rank received gradients outside the '
                                      'learnt parameter set')


class _CapturedStep:
    """One G-step or D-step body captured as a HIP graph: private static copies of its inputs
    (each call copies the caller's tensors in), the graph, and its loss output."""

    def __init__(self, key, inputs):
        self.key, self.inputs = key, inputs
        self.graph = torch.cuda.CUDAGraph()
        self.loss = None


class GANTrainer:
    """One version5_model_train.py iteration per call, optionally data-parallel."""

    # eager steps of each kind before its body is captured (the first ones learn the bucket plan,
    # fill the host-side caches and grow the workspaces)
    GRAPH_WARMUP = 2

    def __init__(self, generator, discriminator, lr=10e-4, lambda_gan=1.0, lambda_d=1.0,
                 dynamic=None, fixed_labels=None, process_group=None, sync_bn=False,
                 bucket_mb=25.0, grad_reduce_dtype=None, label_seed=None, force_collectives=False,
                 graphs=False):
        """label_seed: seed of the generator the noisy GAN labels are drawn from; None (the
        default) derives it from torch.initial_seed() of rank 0, so the labels follow the
        caller's torch.manual_seed like the reference's global-RNG draw (an unseeded process
        draws different labels each run, as the reference does).  With several ranks the seed
        is broadcast here, at construction, not inside a step.  force_collectives: run the
        data-parallel machinery (bucketed gradient all-reduce, SyncBN) also when the process
        group has one rank -- the RCCL path on one GPU (tests/test_gpu_rccl.py).

        graphs: capture the G-step body (forward, losses, backward, gradient gather, bucket
        all-reduces when data-parallel over RCCL, Adam) and the D-step body as HIP graphs after
        GRAPH_WARMUP eager steps of each, and replay them: one graph launch per step instead of
        ~500-1,000 dependent kernel launches.  The reference's host decisions stay on the host,
        between replays (G/D frequencies, should_train_discriminator, the learning rates, which
        reach the device through FlatAdam.use_device_hyper); the labels are drawn eagerly per
        iteration and copied into the graph's inputs; dropout masks stay fresh per step through a
        device seed counter (a2m_set_dropout_seed_offset).  Needs one rank, or a process group on
        the nccl (RCCL) backend, whose collectives the capture records.  A new input shape or
        GEMM precision recaptures."""
        self.G, self.D = generator, discriminator
        self.opt_G = FlatAdam(flat_order(generator), lr=lr)
        self.opt_D = FlatAdam(flat_order(discriminator), lr=lr)
        self.dyn = dynamic if dynamic is not None else DynamicGANTraining(g_lr=lr / 2, d_lr=lr)
        self.lambda_gan, self.lambda_d = lambda_gan, lambda_d
        self.fixed_labels = fixed_labels          # (valid, fake) values for deterministic runs
        self.pg = process_group
        dp = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(process_group) if dp else 1
        self.rank = dist.get_rank(process_group) if dp else 0
        # SyncBN: BatchNorm statistics all-reduced over the DP group, so the
        # ranks normalise over the whole batch like the single-device reference step
        force = bool(force_collectives) and dp
        self.sync_bn = bool(sync_bn) and (self.world > 1 or force)
        self.red_G = GradReducer(self.opt_G, self.world, process_group, bucket_mb, grad_reduce_dtype, force)
        self.red_D = GradReducer(self.opt_D, self.world, process_group, bucket_mb, grad_reduce_dtype, force)
        self.label_seed = label_seed
        self._label_gen = None
        self.last_d_loss = None
        self.graphs = bool(graphs)
        self._collectives = self.world > 1 or force
        self._captured = {'g': None, 'd': None}
        self._warm = {'g': 0, 'd': 0}
        self._seed_ctr = None
        if self.graphs:
            dev = next(generator.parameters()).device
            if dev.type != 'cuda':
                raise RuntimeError('GANTrainer(graphs=True) needs the models on a ROCm device')
            if self._collectives and dist.get_backend(process_group) != 'nccl':
                raise RuntimeError('GANTrainer(graphs=True) with data parallelism needs the nccl '
                                   '(RCCL) backend: gloo collectives cannot be captured')
            self._seed_ctr = torch.zeros(1, dtype=torch.int64, device=dev)
            self._cap_stream = torch.cuda.Stream(device=dev)
            self.opt_G.use_device_hyper()
            self.opt_D.use_device_hyper()
        if fixed_labels is None and label_seed is None and self.world > 1:
            # agree on the label seed now (a collective), not lazily inside the first step
            dev = next(generator.parameters()).device
            self.label_seed = self._shared_label_seed(dev if dev.type == 'cuda' else torch.device('cpu'))

    def _allreduce_(self, t):
        if self.world > 1:
            dist.all_reduce(t, group=self.pg)
            t.div_(self.world)

    def _shared_label_seed(self, dev):
        """label_seed, or (None) a seed that follows the user's torch.manual_seed like the
        reference's global-RNG draw (version5_model_train.py:169,178): torch.initial_seed() of
        rank 0, broadcast so every rank draws the same global-batch labels."""
        if self.label_seed is not None:
            return int(self.label_seed)
        seed = torch.initial_seed() & ((1 << 62) - 1)
        if self.world > 1:
            t = torch.tensor([seed], dtype=torch.int64, device=dev)
            dist.broadcast(t, src=dist.get_global_rank(self.pg, 0) if self.pg is not None else 0,
                           group=self.pg)
            seed = int(t.item())
        return seed

    def _labels(self, epoch, B, dev):
        """Labels for this rank's shard: the global batch (B x world) is drawn from a generator
        seeded identically on every rank and sliced, so a DP run sees the labels of the
        single-device run of the whole batch."""
        if self.fixed_labels is not None:
            v, f = self.fixed_labels
            return torch.full((B, 4), v, device=dev), torch.full((B, 4), f, device=dev)
        if self._label_gen is None or self._label_gen.device != torch.device(dev):
            self._label_gen = torch.Generator(device=dev).manual_seed(self._shared_label_seed(dev))
        Bg, lo = B * self.world, B * self.rank
        real = self.dyn.get_smooth_labels(epoch, Bg, dev, True, generator=self._label_gen)
        fake = self.dyn.get_smooth_labels(epoch, Bg, dev, False, generator=self._label_gen)
        return real[lo:lo + B], fake[lo:lo + B]

    # ---------------------------------------------------------------- HIP-graph replay
    def _body(self, fn, args):
        """Run one step body with the dropout seed counter registered and advanced (graph mode:
        eager warm-up steps, the capture, and hence every replay)."""
        if self._seed_ctr is None:
            return fn(*args)
        F.set_dropout_seed_offset(self._seed_ctr)
        try:
            self._seed_ctr.add_(1)
            return fn(*args)
        finally:
            F.set_dropout_seed_offset(None)

    def _graphed(self, kind, fn, opt, args):
        """One step of `kind` ('g' / 'd'): eager for the first GRAPH_WARMUP calls, then captured
        once (the capture records, it does not run: its call replays right after) and replayed."""
        key = tuple((tuple(a.shape), a.dtype) for a in args) + (F.N.lib.a2m_get_gemm_precision(),)
        st = self._captured[kind]
        if st is not None and st.key != key:
            st = self._captured[kind] = None
        if st is None:
            if self._warm[kind] < self.GRAPH_WARMUP:
                self._warm[kind] += 1
                return self._body(fn, args)
            st = _CapturedStep(key, [a.detach().clone() for a in args])
            torch.cuda.synchronize()
            if self._collectives:
                # RCCL's watchdog thread polls the events of finished eager collectives (every
                # ~100 ms); HIP refuses a query on an event whose stream has since joined a capture
                # (hipErrorCapturedEvent), so let it retire them before the NCCL stream is captured
                time.sleep(0.5)
            steps = opt.step_count
            # each graph keeps its own memory pool: a host cache can drop a buffer that one graph
            # still writes on replay, and only that graph's own recapture may reuse it
            # with collectives, thread-local capture: RCCL's watchdog thread keeps querying the
            # events of earlier (eager) collectives while this thread captures
            mode = 'thread_local' if self._collectives else 'global'
            with torch.cuda.graph(st.graph, stream=self._cap_stream, capture_error_mode=mode):
                st.loss = self._body(fn, st.inputs)
            opt.step_count = steps          # the capture recorded the step; the replay below runs it
            self._captured[kind] = st
        for dst, a in zip(st.inputs, args):
            if dst.data_ptr() != a.data_ptr():
                dst.copy_(a)
        opt.sync_hyper()
        st.graph.replay()
        opt.step_count += 1
        F.bump_weights_epoch()
        return st.loss.clone()

    def _graphs_on(self):
        return self.graphs and torch.cuda.is_available()

    def g_step(self, audio, real_pose, valid):
        if self._graphs_on():
            return self._graphed('g', self._g_step, self.opt_G, (audio, real_pose, valid))
        return self._body(self._g_step, (audio, real_pose, valid))

    def d_step(self, audio, real_motion, valid, fake):
        if self._graphs_on():
            return self._graphed('d', self._d_step, self.opt_D, (audio, real_motion, valid, fake))
        return self._body(self._d_step, (audio, real_motion, valid, fake))

    def _g_step(self, audio, real_pose, valid):
        self.opt_G.zero_grad()
        self.red_G.begin()
        fake_pose, internal = self.G(audio, real_pose=real_pose)
        fake_d, _ = self.D(pos_to_motion(fake_pose))
        terms = compute_temporal_smoothness_loss_and_jerk(fake_pose, real_pose)
        g_loss = terms[0] + self.lambda_gan * AG.mse_loss(fake_d, valid) + 0.1 * terms[1] + 0.05 * terms[2]
        for loss in internal:
            g_loss = g_loss + loss
        g_loss.backward()
        self.red_G.finish()
        self.opt_G.step()
        return g_loss.detach()

    def _d_step(self, audio, real_motion, valid, fake):
        self.opt_D.zero_grad()
        with torch.no_grad():
            fp, _ = self.G(audio)
            fm = pos_to_motion(fp)
        self.red_D.begin()
        fake_d, _ = self.D(fm.detach())
        real_d, _ = self.D(real_motion)
        d_loss = AG.mse_loss(real_d, valid) + self.lambda_d * AG.mse_loss(fake_d, fake)
        d_loss.backward()
        self.red_D.finish()
        self.opt_D.step()
        return d_loss.detach()

    @contextlib.contextmanager
    def sync_bn_scope(self):
        """BatchNorm statistics over the DP group inside the block when sync_bn is on (iteration()
        enters it; g_step / d_step called directly need it for SyncBN)."""
        if not self.sync_bn:
            yield
            return
        prev = F.set_sync_bn_group(self.pg if self.pg is not None else dist.group.WORLD)
        try:
            yield
        finally:
            F.set_sync_bn_group(prev)

    def flush(self):
        """Collective: both gradient reducers' plan checks, now (end of training, before a
        checkpoint); raises on every rank if any rank's gradients left the learnt plan."""
        self.red_G.flush()
        self.red_D.flush()

    def iteration(self, audio, real_pose, epoch=0, g_freq=None, d_freq=None, sync_losses=True):
        """version5_model_train.py:330-414 for one batch; returns (D_loss, G_loss) tensors."""
        with self.sync_bn_scope():
            return self._iteration(audio, real_pose, epoch, g_freq, d_freq, sync_losses)

    def _iteration(self, audio, real_pose, epoch, g_freq, d_freq, sync_losses):
        dev = audio.device
        gf = g_freq if g_freq is not None else self.dyn.g_train_freq
        df = d_freq if d_freq is not None else self.dyn.d_train_freq
        valid, fake = self._labels(epoch, audio.shape[0], dev)
        real_motion = pos_to_motion(real_pose)
        d_params = [p for p in self.D.parameters()]
        for p in d_params:
            p.requires_grad_(False)
        try:
            for _ in range(gf):
                g_loss = self.g_step(audio, real_pose, valid)
        finally:
            for p in d_params:
                p.requires_grad_(True)
        d_loss = None
        if self.dyn.should_train_discriminator():
            for _ in range(df):
                d_loss = self.d_step(audio, real_motion, valid, fake)
        if d_loss is None:  # reference reuses the last logged D loss when D is skipped
            d_loss = self.last_d_loss if self.last_d_loss is not None else torch.ones((), device=dev)
        self.last_d_loss = d_loss
        if sync_losses:
            pair = torch.stack([d_loss.reshape(()), g_loss.reshape(())])
            self._allreduce_(pair)
            d_val, g_val = pair.tolist()
            self.dyn.update_loss_history(d_val, g_val)
        return d_loss, g_loss
