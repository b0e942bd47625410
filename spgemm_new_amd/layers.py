"""SAGE layers over the MaxK aggregation (the integration of utils/models.py:199-257).

The reference's SAGE.forward per layer (utils/models.py:230, 242-253):

    x_agg = SpGEMMFunction.apply(x, (indptr, indices, values), maxk)   # MaxK + A . X^
    x = fc_self(x) + fc_neigh(x_agg)

``MaxKSAGELayer`` is that layer (dropout / norm are the caller's, as in the
reference loop).  ``MaxKRelSAGELayer`` is its multi-relation form for graphs
with R edge features (ogbn-proteins, BASELINE config 5; the reference instead
sums the 8 edge features into node features, utils/proteins_loader.py:41-44):
one fused aggregation Y[q] = A_q . X^ for all relations (SpGEMMMultiFunction),
then a per-relation neighbour weight, x = fc_self(x) + sum_q Y[q] W_q + b.
The dense parts are torch matmuls (hipBLASLt); the aggregation is the HIP path.
A rank of a row-partitioned graph passes its PartitionedMaxK instead of the
graph tuple (PartitionedSpGEMMFunction / PartitionedSpGEMMMultiFunction).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from .models import (PartitionedSpGEMMFunction, PartitionedSpGEMMMultiFunction,
                     SpGEMMFunction, SpGEMMMultiFunction)


class MaxKSAGELayer(nn.Module):
    def __init__(self, hidden: int, maxk: int):
        super().__init__()
        self.maxk = maxk
        self.fc_self = nn.Linear(hidden, hidden)
        self.fc_neigh = nn.Linear(hidden, hidden)

    def forward(self, graph, x: torch.Tensor) -> torch.Tensor:
        """graph: (indptr, indices, values) or a rank's PartitionedMaxK."""
        if isinstance(graph, tuple):
            agg = SpGEMMFunction.apply(x, graph, self.maxk)
        else:
            agg = PartitionedSpGEMMFunction.apply(x, graph, self.maxk)
        return self.fc_self(x) + self.fc_neigh(agg)


class MaxKRelSAGELayer(nn.Module):
    def __init__(self, hidden: int, maxk: int, num_rel: int):
        super().__init__()
        self.maxk, self.num_rel = maxk, num_rel
        self.fc_self = nn.Linear(hidden, hidden)
        self.w_rel = nn.Parameter(torch.empty(num_rel, hidden, hidden))
        self.b_rel = nn.Parameter(torch.zeros(hidden))
        bound = 1.0 / math.sqrt(hidden * num_rel)
        nn.init.uniform_(self.w_rel, -bound, bound)

    def forward(self, graph, x: torch.Tensor, values: torch.Tensor | None = None) -> torch.Tensor:
        """graph: (indptr, indices) with values fp32[E, R], or a rank's
        PartitionedMaxK built with values [E, R]."""
        if isinstance(graph, tuple):
            agg = SpGEMMMultiFunction.apply(x, graph, values, self.maxk)     # [R, V, h]
        else:
            agg = PartitionedSpGEMMMultiFunction.apply(x, graph, self.maxk)
        neigh = torch.bmm(agg, self.w_rel).sum(0)                          # sum_q Y_q W_q
        return self.fc_self(x) + neigh + self.b_rel
