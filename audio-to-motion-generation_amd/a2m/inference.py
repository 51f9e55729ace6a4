"""Inference surface of generate_motion_video.py, on the device.

  load_generator(path)      :237-238  construct + load_state_dict (weights_only) + eval
  generate(g, audio, ...)   :247-260  generator(audio) on normalised audio features, then the
                                      normalised poses mapped back: pose * std + mean
  planar_frames(pose)       :262-266  [B, T, 104] -> [B, T, 2, 52] (x row, y row) for plotting

Plotting and ffmpeg (:23-207) stay host-side reference code (out of scope).
"""
import torch

from .normalization import denormalize
from .real_motion_model import SelfAttention_G


def load_generator(path, device='cuda', **kwargs):
    g = SelfAttention_G(**kwargs)
    g.load_state_dict(torch.load(path, map_location='cpu', weights_only=True))
    return g.to(device).eval()


@torch.no_grad()
def generate(generator, audio, pose_mean=None, pose_std=None):
    """audio [B, T, 128] (device) -> poses [B, T, 104]; de-normalised when mean/std are given."""
    pose, _ = generator(audio)
    if pose_mean is not None:
        pose = denormalize(pose, pose_mean.to(pose.device), pose_std.to(pose.device))
    return pose


def planar_frames(pose):
    B, T, _ = pose.shape
    return pose.reshape(B, T, 2, -1)
