"""Drivers shared by oracle/make_fixtures_r2.py (which runs them on the REFERENCE's code) and
the CPU tests (which run them on a2m's).  TEST INFRASTRUCTURE ONLY.

  run_schedule       drives a DynamicGANTraining-like class through a fixed loss sequence the
                     way version5_model_train.py:330-414 calls it and records every decision
  window_case_data   the synthetic recordings of the windowing fixture's cases
"""
import numpy as np
import torch


class _Opt:
    def __init__(self, lr):
        self.param_groups = [{'lr': lr}, {'lr': lr}]


# (d_loss, g_loss) per batch: neutral start, a strong discriminator, a strong generator, then a
# swing back -- enough history to reach every branch of :53-133
DYN_LOSSES = ([(0.5, 0.6)] * 12 + [(0.05, 1.2)] * 14 + [(0.9, 0.2)] * 14 + [(0.75, 0.35)] * 8 +
              [(0.15, 0.9)] * 12 + [(0.12, 0.05)] * 20 + [(0.3, 0.3)] * 90)


def run_schedule(cls, losses=DYN_LOSSES, dynamic_smooth=False, label_epochs=(0, 30, 61, -1)):
    """Drives a DynamicGANTraining-like class the way version5_model_train.py:330-414 does and
    records every decision.  Shared by the fixture (reference class) and the CPU test (a2m)."""
    lr = 10e-4
    dyn = cls(g_lr=lr / 2, d_lr=lr)
    dyn.dynamic_smooth = dynamic_smooth
    og, od = _Opt(lr), _Opt(lr)
    rec = {'g_freq': [], 'd_freq': [], 'g_lr': [], 'd_lr': [], 'train_d': [], 'recent': [],
           'labels_real': [], 'labels_fake': []}
    epoch = 0
    for i, (dl, gl) in enumerate(losses):
        if i % 4 == 0:   # an "epoch" every 4 batches: frequency and LR adaptation at its start
            gf, df = dyn.adjust_training_frequency(epoch)
            dyn.adjust_learning_rates(og, od, epoch)
            epoch += 1
        rec['g_freq'].append(gf)
        rec['d_freq'].append(df)
        rec['g_lr'].append(og.param_groups[0]['lr'])
        rec['d_lr'].append(od.param_groups[0]['lr'])
        rec['train_d'].append(bool(dyn.should_train_discriminator()))
        if i % 8 == 0:
            for e in label_epochs:
                torch.manual_seed(1000 + i + e)
                rec['labels_real'].append(dyn.get_smooth_labels(e, 3, 'cpu', is_real=True).tolist())
                rec['labels_fake'].append(dyn.get_smooth_labels(e, 3, 'cpu', is_real=False).tolist())
        dyn.update_loss_history(dl, gl)
        rec['recent'].append([float(v) for v in dyn.get_recent_avg_loss()])
    return rec


def window_case_data(ci, lp, la):
    """Synthetic recordings of one windowing case (numpy PCG64: bit-identical everywhere, so
    the test regenerates them instead of reading them from the fixture)."""
    pose = np.random.default_rng([51, ci, 0]).standard_normal((lp, 104)).astype(np.float32)
    audio = np.random.default_rng([51, ci, 1]).standard_normal((la, 128)).astype(np.float32)
    r = np.random.default_rng([51, ci, 2])
    mean = r.standard_normal(104).astype(np.float32)
    std = r.uniform(0.5, 2.0, 104).astype(np.float32)
    std[3] = 1e-9
    return pose, audio, mean, std
