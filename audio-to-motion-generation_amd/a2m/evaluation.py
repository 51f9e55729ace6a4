"""PCK on the device: motion_evaluation.py:4-22 (52 keypoints) and
pose_video/evaluation.py:4-21 (48 keypoints; the keypoint count is taken from the input).

compute_pck(pred, gt, alpha=0.2): pred, gt [N, 2, K] (x row, y row) -> [N], the fraction of
keypoints whose distance to gt is <= alpha * max(x extent, y extent) of that sample's gt.
numpy in -> numpy out (like the reference); device tensors in -> device tensor out.
"""
import numpy as np
import torch

from . import functional as F
from ._native import check, lib


def compute_pck(pred, gt, alpha=0.2):
    as_numpy = not torch.is_tensor(gt)
    g = torch.as_tensor(np.asarray(gt, np.float32)).cuda() if as_numpy else gt
    p = torch.as_tensor(np.asarray(pred, np.float32)).cuda() if as_numpy else pred
    F._check_dev(p.float(), g.float())
    g, p = g.float().contiguous(), p.float().contiguous()
    if g.dim() != 3 or g.shape[1] != 2 or tuple(p.shape) != tuple(g.shape):
        raise ValueError(f'pred and gt must both be [N, 2, K]; got {tuple(p.shape)}, {tuple(g.shape)}')
    N, _, K = g.shape
    out = torch.empty(N, dtype=torch.float64, device=g.device)
    check(lib.a2m_pck_f32(F._p(p), F._p(g), N, K, float(alpha), F._p(out), F._stream()))
    return out.cpu().numpy() if as_numpy else out
