#!/usr/bin/env python3
"""How often the two edges of one LOCAL wave-instruction (k=32: records 2i, 2i+1 of a
wave's list) share their source row, and how often they could (same-row runs
re-aligned to even positions).  Development tool."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd.graphs import CONFIGS, synthetic_csr_gpu  # noqa: E402

dev = torch.device("cuda:0")
V, E = CONFIGS["reddit"]
indptr, indices = synthetic_csr_gpu(V, E, device=dev)
g = S.MaxKGraph(indptr, indices)
plan = g.local_plan(32)
erc = plan["edge_rc"].long()
woff = plan["woff"].long()
row = erc & 0xffffff
W = plan["num_waves"]
# pair index within each wave's list
wave_of = torch.repeat_interleave(torch.arange(W, device=dev), woff[1:] - woff[:-1])
pos = torch.arange(erc.numel(), device=dev) - woff[wave_of]
even = (pos % 2 == 0) & (pos + 1 < (woff[wave_of + 1] - woff[wave_of]))
idx = torch.nonzero(even).squeeze(1)
aligned = (row[idx] == row[idx + 1]).float().mean().item()
same_next = (row[:-1] == row[1:]) & (wave_of[:-1] == wave_of[1:])
print(f"W={W} edges={erc.numel()} aligned same-source pairs: {aligned * 100:.2f}% of pairs; "
      f"adjacent same-source: {same_next.float().mean().item() * 100:.2f}% of neighbours")
