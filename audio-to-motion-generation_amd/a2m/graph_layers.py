"""Parameter containers for the two PyTorch-Geometric layers the reference uses, with PyG's
state_dict names so reference checkpoints load unchanged:

  GATConv(64, 64, heads=4, concat=False)  lin.weight [256,64], att_src/att_dst [1,4,64], bias [64]
  GraphConv(64, 64)                        lin_rel.weight/.bias, lin_root.weight

Older PyG releases saved GATConv's projection as lin_src.weight (+ an alias lin_dst.weight);
those keys are accepted on load.  The compute lives in the fused HIP graph-layer kernel
(a2m.functional.graph_layer); these modules carry no forward of their own.
"""
import math

import torch
import torch.nn as nn


class GATConv(nn.Module):
    def __init__(self, in_channels, out_channels, heads=1, concat=True, negative_slope=0.2,
                 dropout=0.0, add_self_loops=True, bias=True, **kwargs):
        super().__init__()
        assert not concat and add_self_loops and dropout == 0.0
        self.in_channels, self.out_channels, self.heads = in_channels, out_channels, heads
        self.negative_slope = negative_slope
        self.lin = nn.Linear(in_channels, heads * out_channels, bias=False)
        self.att_src = nn.Parameter(torch.empty(1, heads, out_channels))
        self.att_dst = nn.Parameter(torch.empty(1, heads, out_channels))
        self.bias = nn.Parameter(torch.empty(out_channels)) if bias else None
        self._U = {}   # attention projections for the fused eval stack (functional.graph_att_proj)
        self._Wh = {}  # bf16 weight copies for the bf16 mode's fused stack (functional.graph_weights_bf16)
        self.reset_parameters()

    def reset_parameters(self):
        for t in (self.lin.weight, self.att_src, self.att_dst):
            a = math.sqrt(6.0 / (t.shape[-2] + t.shape[-1]))
            nn.init.uniform_(t, -a, a)
        if self.bias is not None:
            nn.init.zeros_(self.bias)

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys,
                              unexpected_keys, error_msgs):
        old = prefix + 'lin_src.weight'
        if old in state_dict and prefix + 'lin.weight' not in state_dict:
            state_dict[prefix + 'lin.weight'] = state_dict.pop(old)
            state_dict.pop(prefix + 'lin_dst.weight', None)
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys,
                                      unexpected_keys, error_msgs)


class GraphConv(nn.Module):
    def __init__(self, in_channels, out_channels, aggr='add', bias=True, **kwargs):
        super().__init__()
        assert aggr == 'add'
        self.lin_rel = nn.Linear(in_channels, out_channels, bias=bias)
        self.lin_root = nn.Linear(in_channels, out_channels, bias=False)
        self._Wh = {}  # bf16 weight copies for the bf16 mode's fused stack (functional.graph_weights_bf16)
