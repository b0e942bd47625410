#!/usr/bin/env python3
"""TILE plan statistics on one shape: record groups (of 4) per wave and chunk,
half 0 / half 1 split, padding share.  Development tool.

usage: tools/exp_tile_stats.py [graph] [k]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd.graphs import CONFIGS, synthetic_csr_gpu  # noqa: E402

graph = sys.argv[1] if len(sys.argv) > 1 else "reddit"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 32
dev = torch.device("cuda:0")
V, E = CONFIGS[graph]
indptr, indices = synthetic_csr_gpu(V, E, device=dev)
values = torch.rand(E, device=dev)
g = S.MaxKGraph(indptr, indices, values)
plan = g.tile_plan(K)
L = S.tile.ring_format()[0] - 1
hdr = plan["headers"].view(-1, 4)
hs = plan["header_start"].long()
nch = plan["num_chunks"].long()
waves = 16
cnts = []
for wg in range(nch.numel()):
    n = int(nch[wg])
    for w in range(waves):
        b = int(hs[wg * waves + w])
        cnts.append(hdr[b + L:b + L + n, 0])
c = torch.cat(cnts).long()
n0, n1 = c & 0xFFFF, c >> 16
groups = (n0 + n1) // 4
print(f"{graph} k={K}: wave-chunks {c.numel()}, records {int((n0 + n1).sum())} "
      f"(edges {E}, padding {(int((n0 + n1).sum()) - E) / E:.1%})")
print(f"  records per wave-chunk mean {float((n0 + n1).float().mean()):.2f} max {int((n0 + n1).max())}")
h = torch.bincount(groups, minlength=12)[:12].tolist()
print("  groups histogram 0..11:", h, " >11:", int((groups > 11).sum()))
print(f"  groups in the loop (beyond 4): {int((groups - 4).clamp(min=0).sum())} of {int(groups.sum())}")
