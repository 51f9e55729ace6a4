"""Neck-subtraction normalisation of poses on the device.

  get_mean_std_necksub(dataloader)   normalization_tools.py:24-45
  get_mean_std(dataloader)           normalization_tools.py:7-21
  necksub_normalize(pose, mean, std) version5_model_train.py:298-304 (also :309-316 for dev)
  denormalize(pose, mean, std)       generate_motion_video.py:259-260

Same statistics as the reference: the mean over batches of per-batch means (every batch
weighted equally, whatever its size), std = sqrt(E[x^2] - mean^2), and for the neck-subtracted
variant std[0] = std[52] = 1 (the neck itself is identically zero).  Batches may live on the
host (as the reference's loader yields them) or on the GPU; the reduction runs on the GPU.
"""
import torch

from . import functional as F
from ._native import check, lib

_P = F._p


def _moments(batches, necksub):
    acc, n, dev = None, 0, None
    for pose in batches:
        pose = pose if pose.is_cuda else pose.to('cuda')
        dev = pose.device
        pose = pose.float().contiguous()
        assert pose.shape[-1] == 104, 'poses are [B, T, 104]'
        if acc is None:
            acc = torch.zeros(208, dtype=torch.float64, device=dev)
        frames = pose.numel() // 104
        check(lib.a2m_pose_moments_f32(_P(pose), frames, int(necksub), _P(acc), F._stream()))
        n += 1
    if n == 0:
        raise ValueError('no batches')
    mean = acc[:104] / n
    std = (acc[104:] / n - mean * mean).sqrt()
    if necksub:
        std[0] = 1.0
        std[52] = 1.0
    return mean.float(), std.float()


def _train_batches(dataloader):
    return (batch['pose/data'] for batch in dataloader.train)


def get_mean_std_necksub(dataloader):
    """normalization_tools.get_mean_std_necksub: (mean[104], std[104]) of neck-subtracted poses."""
    return _moments(_train_batches(dataloader), True)


def get_mean_std(dataloader):
    """normalization_tools.get_mean_std: (mean[104], std[104]) of the raw poses."""
    return _moments(_train_batches(dataloader), False)


def necksub_normalize(pose, mean, std, out=None):
    """((pose - neck) - mean) / std for pose [..., 104] on the device."""
    F._check_dev(pose, mean, std, out)
    pose = pose.contiguous()
    if out is None:
        out = torch.empty_like(pose)
    check(lib.a2m_pose_normalize_f32(_P(pose), pose.numel() // 104, _P(mean.contiguous()),
                                     _P(std.contiguous()), _P(out), F._stream()))
    return out


def denormalize(pose, mean, std, out=None):
    """pose * std + mean (the generator's normalised output back to neck-relative pixels)."""
    F._check_dev(pose, mean, std, out)
    pose = pose.contiguous()
    if out is None:
        out = torch.empty_like(pose)
    check(lib.a2m_pose_denormalize_f32(_P(pose), pose.numel() // 104, _P(mean.contiguous()),
                                       _P(std.contiguous()), _P(out), F._stream()))
    return out
