"""TEST INFRASTRUCTURE — numpy restatement of the evaluation / normalisation rows of SURVEY.md
8(f), pinned by tests/golden/eval_norm.npz (generated from the reference by
oracle/make_fixtures_eval.py).

  necksub_moments    normalization_tools.py:24-45 (one batch's contribution)
  mean_std_necksub   normalization_tools.py:24-45 (mean of per-batch means; std[0]=std[52]=1)
  normalize          version5_model_train.py:298-304 / generate_motion_video.py:247-254
  denormalize        generate_motion_video.py:259-260
  compute_pck        motion_evaluation.py:4-22 (K = 52) / pose_video/evaluation.py:4-21 (K = 48)
"""
import numpy as np


def necksub(pose):
    """[B, T, 104] planar (x block, y block) -> minus the neck (joint 0) per frame."""
    B, T, _ = pose.shape
    p = pose.reshape(B, T, 2, -1)
    return (p - p[:, :, :, :1]).reshape(B, T, -1)


def necksub_moments(pose):
    """(mean over (B, T) of the neck-subtracted pose, mean of its squares), float64."""
    p = necksub(np.asarray(pose, np.float64))
    return p.mean(axis=(0, 1)), (p * p).mean(axis=(0, 1))


def mean_std_necksub(batches):
    s1 = np.zeros(104)
    s2 = np.zeros(104)
    for b in batches:
        m1, m2 = necksub_moments(b)
        s1 += m1
        s2 += m2
    n = len(batches)
    mean = s1 / n
    std = np.sqrt(s2 / n - mean ** 2)
    std[0] = 1.0
    std[52] = 1.0
    return mean, std


def normalize(pose, mean, std):
    return ((necksub(np.asarray(pose, np.float64)) - mean) / std).astype(np.float32)


def denormalize(pose, mean, std):
    return (np.asarray(pose, np.float64) * std + mean).astype(np.float32)


def compute_pck(pred, gt, alpha=0.2):
    """pred, gt [N, 2, K] -> [N] fraction of keypoints within alpha * max(extent_x, extent_y)."""
    pred, gt = np.asarray(pred, np.float64), np.asarray(gt, np.float64)
    ext = np.maximum(np.abs(gt[:, 0].max(1) - gt[:, 0].min(1)), np.abs(gt[:, 1].max(1) - gt[:, 1].min(1)))
    dist = np.sqrt(((gt - pred) ** 2).sum(axis=1))
    return (dist <= (ext * alpha)[:, None]).mean(axis=1)
