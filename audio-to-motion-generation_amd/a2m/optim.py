"""Adam over a flat parameter buffer (torch.optim.Adam semantics, the optimiser of
version5_model_train.py:285-286), one fused HIP kernel per step.

On construction the module's parameters are re-seated as views of one contiguous buffer.
zero_grad() leaves .grad unset, so autograd's AccumulateGrad keeps each fresh gradient tensor
as it is (no per-parameter add kernel), and collect_grads() gathers them into one contiguous
gradient buffer with a few segment-gather launches; the data-parallel all-reduce then runs
over contiguous buckets of `flat_grad` (training.GradReducer), and the update is one launch
over `flat`.  `param_groups[0]['lr']` may be changed between steps
(DynamicGANTraining.adjust_learning_rates does).

Every parameter starts on a 64-byte boundary of the buffer (ALIGN floats): the GEMM engine
stages a 16-byte-aligned weight as a dense operand, a misaligned one through the slower
gathered path (SelfAttention's 1-element gamma would otherwise shift every later weight).
The padding holds zeros and its gradient stays zero.
"""
ALIGN = 16
import torch

from . import functional as F


def flat_order(module):
    """module.parameters() in FlatAdam placement order: each SelfAttention's query / key / value
    weights back to back, then their biases (then gamma), so its stacked QKV operand is a view of
    the flat buffer (functional.stacked_qkv) instead of a copy per weight version -- 80 launches
    an iteration of the training step.  Every other parameter keeps module order."""
    from .model_layers import SelfAttention
    order, seen = [], set()

    def add(p):
        if id(p) not in seen:
            seen.add(id(p))
            order.append(p)
    grouped = {}
    for m in module.modules():
        if isinstance(m, SelfAttention):
            wq, bq, wk, bk, wv, bv, g = m.weights()
            grouped[id(wq)] = (wq, wk, wv, bq, bk, bv, g)
    members = {id(p) for ps in grouped.values() for p in ps}
    for p in module.parameters():
        if id(p) in grouped:
            for q in grouped[id(p)]:
                add(q)
        elif id(p) not in members:
            add(p)
    return order


class FlatAdam:
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        self.params = [p for p in params if p.requires_grad]
        dev = self.params[0].device
        n = sum(-(-p.numel() // ALIGN) * ALIGN for p in self.params)
        self.flat = torch.zeros(n, device=dev)
        self.flat_grad = torch.zeros(n, device=dev)
        self.exp_avg = torch.zeros(n, device=dev)
        self.exp_avg_sq = torch.zeros(n, device=dev)
        for p, (off, k) in zip(self.params, self._spans()):
            self.flat[off:off + k].copy_(p.detach().reshape(-1))
            p.data = self.flat[off:off + k].view_as(p)
            p.grad = self.flat_grad[off:off + k].view_as(p)
        self.param_groups = [dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)]
        self.step_count = 0
        self._dev_hyper = None     # (lr float32[1], step int32[1]) once use_device_hyper() is called
        self._dev_lr = None

    def zero_grad(self, set_to_none=False):
        """Zero the flat gradient and detach .grad from it: autograd then hands each parameter
        its fresh gradient tensor (no per-parameter add), and collect_grads() gathers them all
        into `flat_grad` in a few launches."""
        self.flat_grad.zero_()
        for p in self.params:
            p.grad = None

    @torch.no_grad()
    def collect_grads(self):
        """Gather every .grad that is not already its view of `flat_grad` into the flat buffer
        (a2m_gather_segments_f32) and re-seat .grad as that view.  Call before reducing
        `flat_grad` across ranks; step() calls it too (a no-op the second time)."""
        segs, seat = [], []
        for p, (o, k) in zip(self.params, self._spans()):
            view = self.flat_grad[o:o + k]
            if p.grad is None:
                seat.append((p, view))
            elif p.grad.data_ptr() != view.data_ptr():
                segs.append((o, p.grad.contiguous()))
                seat.append((p, view))
        F.gather_segments_(self.flat_grad, segs)
        for p, view in seat:
            p.grad = view.view_as(p)

    def _spans(self):
        off = 0
        for p in self.params:
            yield off, p.numel()
            off += -(-p.numel() // ALIGN) * ALIGN

    def use_device_hyper(self):
        """Keep the learning rate and the step count in device memory (a2m_adam_dev_f32), so a
        step captured in a HIP graph reads the current values when replayed: the launch advances
        the device step itself, and sync_hyper() rewrites the device lr when param_groups' lr
        changed (DynamicGANTraining).  Bitwise the same update as the host-argument launch."""
        if self._dev_hyper is None:
            dev = self.flat.device
            self._dev_hyper = (torch.zeros(1, device=dev), torch.zeros(1, dtype=torch.int32, device=dev))
            self._dev_lr = None
        self._dev_hyper[1].fill_(self.step_count)
        self.sync_hyper()

    def sync_hyper(self):
        """Write param_groups' lr to the device copy if it changed (stream-ordered, outside any
        captured region)."""
        lr = float(self.param_groups[0]['lr'])
        if self._dev_hyper is not None and lr != self._dev_lr:
            self._dev_hyper[0].fill_(lr)
            self._dev_lr = lr

    @torch.no_grad()
    def step(self):
        self.collect_grads()
        self.step_count += 1
        g = self.param_groups[0]
        if self._dev_hyper is not None:
            if not torch.cuda.is_current_stream_capturing():
                self.sync_hyper()
            F.adam_dev_(self.flat, self.flat_grad, self.exp_avg, self.exp_avg_sq, self._dev_hyper[0],
                        g['betas'][0], g['betas'][1], g['eps'], g['weight_decay'], self._dev_hyper[1])
        else:
            F.adam_(self.flat, self.flat_grad, self.exp_avg, self.exp_avg_sq, g['lr'], g['betas'][0],
                    g['betas'][1], g['eps'], g['weight_decay'], self.step_count)
        F.bump_weights_epoch()   # the HIP update is invisible to torch's version counters

    def state_dict(self):
        return {'step': self.step_count, 'exp_avg': self.exp_avg.clone(), 'exp_avg_sq': self.exp_avg_sq.clone(),
                'param_groups': [dict(g) for g in self.param_groups]}

    def load_state_dict(self, sd):
        self.step_count = sd['step']
        if self._dev_hyper is not None:
            self._dev_hyper[1].fill_(self.step_count)
            self._dev_lr = None
        self.exp_avg.copy_(sd['exp_avg'])
        self.exp_avg_sq.copy_(sd['exp_avg_sq'])
        self.param_groups = [dict(g) for g in sd['param_groups']]
        self.sync_hyper()
