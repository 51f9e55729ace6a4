"""Skeleton topology constants (replaces pats/data_loading/skeleton.py:94-150).

Skeleton2D in the reference reads a dataset CSV in its constructor (skeleton.py:23) only to
serve these constants; here they are plain data, and the graph / triple construction of
SelfAttention_G.__init__ (real_motion_model.py:42-63, 280-304) is restated over them.
"""
import torch

PARENTS = [-1,
           0, 1, 2,
           0, 4, 5,
           0, 7, 7,
           6,
           10, 11, 12, 13, 10, 15, 16, 17, 10, 19, 20, 21, 10, 23, 24, 25, 10, 27, 28, 29,
           3,
           31, 32, 33, 34, 31, 36, 37, 38, 31, 40, 41, 42, 31, 44, 45, 46, 31, 48, 49, 50]

JOINT_NAMES = (['Neck', 'RShoulder', 'RElbow', 'RWrist', 'LShoulder', 'LElbow', 'LWrist',
                'Nose', 'REye', 'LEye', 'LHandRoot'] +
               [f'LHand{f}{i}' for f in ('Thumb', 'Index', 'Middle', 'Ring', 'Little') for i in range(1, 5)] +
               ['RHandRoot'] +
               [f'RHand{f}{i}' for f in ('Thumb', 'Index', 'Middle', 'Ring', 'Little') for i in range(1, 5)])

FPS = 15
NUM_BODY, NUM_HAND, FEAT = 10, 42, 64


class Skeleton2D:
    """Constant-only stand-in for pats.data_loading.Skeleton2D (no dataset access)."""
    parents = PARENTS
    joint_names = JOINT_NAMES
    root = 0

    @property
    def joint_subset(self):
        return list(range(7)) + list(range(10, len(PARENTS)))

    def fs(self, modality=None):
        return FPS


def edge_index(lo, n):
    """Directed edges (parent->child, child->parent) of joints [lo, lo+n) whose parent is in
    the same range, in the reference's order (real_motion_model.py:43-60)."""
    edges = []
    for i in range(n):
        par = PARENTS[lo + i]
        par = par - lo if lo <= par < lo + n else -1
        if par != -1:
            edges.append([par, i])
            edges.append([i, par])
    return torch.tensor(edges, dtype=torch.long).t().contiguous()


def in_neighbour_csr(ei, n):
    """CSR over targets: for node i the sources of edges into i, in edge order (the order a
    PyG scatter visits them).  Raises ValueError for topologies beyond the graph kernels'
    limits (include/a2m.h): <= 128 nodes, in-degree <= 7 (8 with GAT's self loop), and
    ptr + idx entries <= 256 (the block-local CSR the kernels stage in LDS)."""
    src, dst = ei[0].tolist(), ei[1].tolist()
    if n > 128:
        raise ValueError(f'graph of {n} nodes: the graph kernels support at most 128')
    ptr, idx = [0], []
    for i in range(n):
        idx += [s for s, d in zip(src, dst) if d == i]
        ptr.append(len(idx))
        if ptr[-1] - ptr[-2] > 7:
            raise ValueError(f'node {i} has in-degree {ptr[-1] - ptr[-2]}: the graph kernels '
                             f'support at most 7 (+ the GAT self loop)')
    if len(ptr) + len(idx) > 256:
        raise ValueError(f'{len(idx)} edges over {n} nodes: the graph kernels hold at most '
                         f'{256 - (n + 1)} edges for this node count')
    return torch.tensor(ptr, dtype=torch.int32), torch.tensor(idx, dtype=torch.int32)


def triples(lo, n):
    """(parent, joint, first child) chains inside [lo, lo+n) (real_motion_model.py:280-304)."""
    out = []
    for i in range(n):
        p = PARENTS[lo + i]
        if not (lo <= p < lo + n):
            continue
        for j in range(i + 1, n):
            if PARENTS[lo + j] == lo + i:
                out.append((p - lo, i, j))
                break
    return out
