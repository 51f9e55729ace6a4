"""Restatement of the two PyTorch-Geometric layers the reference uses.  TEST ORACLE ONLY.

PyG is not installed in the image and the reference pins no version
(no requirements file), so these are written from PyG's documented default semantics:

GATConv(in, out, heads=H, concat=False)   (reference real_motion_model.py:78,557)
    x' = lin(x)                    lin: Linear(in, H*out, bias=False)  -> view [N, H, out]
    a_src[n,h] = <x'[n,h], att_src[h]> ; a_dst[n,h] = <x'[n,h], att_dst[h]>
    edges: remove self loops, then add one self loop per node (add_self_loops=True)
    e[j->i,h] = leaky_relu(a_src[j,h] + a_dst[i,h], 0.2)
    alpha = softmax of e over the incoming edges of i  (max-subtracted, +1e-16 in denom)
    out[i,h] = sum_j alpha[j->i,h] * x'[j,h]
    out = mean_h out[:, h] + bias       (concat=False)
    state_dict: lin.weight, att_src [1,H,out], att_dst [1,H,out], bias [out]
    (older PyG spelled lin as lin_src/lin_dst; the product loader accepts both)

GraphConv(in, out)  aggr='add'             (reference real_motion_model.py:79,105)
    out = lin_rel(sum_{j->i} x_j) + lin_root(x_i)
    state_dict: lin_rel.weight, lin_rel.bias, lin_root.weight  (lin_root has no bias)

edge_index convention: row 0 = source j, row 1 = target i (flow source_to_target).
GNN parity against real PyG is therefore "parity unpinned"; it is pinned only against
this restatement executed inside the reference model (tests/golden/*).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


def _add_self_loops(edge_index, num_nodes):
    keep = edge_index[0] != edge_index[1]
    ei = edge_index[:, keep]
    loop = torch.arange(num_nodes, device=edge_index.device, dtype=edge_index.dtype)
    return torch.cat([ei, torch.stack([loop, loop])], dim=1)


def _segment_softmax(src, index, num_nodes):
    # src [E, H]; softmax over entries that share index (the target node)
    H = src.shape[1]
    idx = index.view(-1, 1).expand(-1, H)
    mx = torch.full((num_nodes, H), float('-inf'), dtype=src.dtype, device=src.device)
    mx = mx.scatter_reduce(0, idx, src, reduce='amax', include_self=True)
    out = (src - mx.gather(0, idx)).exp()
    den = torch.zeros((num_nodes, H), dtype=src.dtype, device=src.device).index_add_(0, index, out)
    return out / (den.gather(0, idx) + 1e-16)


class GATConv(nn.Module):
    def __init__(self, in_channels, out_channels, heads=1, concat=True, negative_slope=0.2,
                 dropout=0.0, add_self_loops=True, bias=True):
        super().__init__()
        self.in_channels, self.out_channels, self.heads = in_channels, out_channels, heads
        self.concat, self.negative_slope, self.add_loops = concat, negative_slope, add_self_loops
        self.lin = nn.Linear(in_channels, heads * out_channels, bias=False)
        self.att_src = nn.Parameter(torch.empty(1, heads, out_channels))
        self.att_dst = nn.Parameter(torch.empty(1, heads, out_channels))
        if bias:
            self.bias = nn.Parameter(torch.empty(heads * out_channels if concat else out_channels))
        else:
            self.register_parameter('bias', None)
        nn.init.xavier_uniform_(self.lin.weight)
        nn.init.xavier_uniform_(self.att_src)
        nn.init.xavier_uniform_(self.att_dst)
        if self.bias is not None:
            nn.init.zeros_(self.bias)

    def forward(self, x, edge_index):
        N = x.shape[0]
        H, C = self.heads, self.out_channels
        xp = self.lin(x).view(N, H, C)
        a_src = (xp * self.att_src).sum(-1)
        a_dst = (xp * self.att_dst).sum(-1)
        ei = _add_self_loops(edge_index, N) if self.add_loops else edge_index
        src, dst = ei[0], ei[1]
        e = F.leaky_relu(a_src[src] + a_dst[dst], self.negative_slope)
        alpha = _segment_softmax(e, dst, N)
        msg = xp[src] * alpha.unsqueeze(-1)
        # PyG scatters into an output of the message dtype (fp32 under autocast: bf16 x * fp32 alpha)
        out = torch.zeros((N, H, C), dtype=msg.dtype, device=x.device).index_add_(0, dst, msg)
        out = out.reshape(N, H * C) if self.concat else out.mean(dim=1)
        if self.bias is not None:
            out = out + self.bias
        return out


class GraphConv(nn.Module):
    def __init__(self, in_channels, out_channels, aggr='add', bias=True):
        super().__init__()
        self.lin_rel = nn.Linear(in_channels, out_channels, bias=bias)
        self.lin_root = nn.Linear(in_channels, out_channels, bias=False)

    def forward(self, x, edge_index):
        src, dst = edge_index[0], edge_index[1]
        agg = torch.zeros_like(x).index_add_(0, dst, x[src])
        return self.lin_rel(agg) + self.lin_root(x)


class Data:
    def __init__(self, x=None, edge_index=None):
        self.x, self.edge_index = x, edge_index


class Batch(Data):
    @classmethod
    def from_data_list(cls, data_list):
        xs, eis, off = [], [], 0
        for d in data_list:
            xs.append(d.x)
            eis.append(d.edge_index + off)
            off += d.x.shape[0]
        return cls(x=torch.cat(xs, 0), edge_index=torch.cat(eis, 1))
