#!/usr/bin/env python3
"""Forward SpGEMM time alone on a BASELINE graph (min of 3 x reps).  Development tool.

usage: tools/exp_fwd_time.py [graph] [k] [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd.graphs import CONFIGS, synthetic_csr_gpu  # noqa: E402

graph = sys.argv[1] if len(sys.argv) > 1 else "reddit"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 32
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
dev = torch.device("cuda:0")
V, E = CONFIGS[graph]
indptr, indices = synthetic_csr_gpu(V, E, device=dev)
values = torch.rand(E, device=dev)
X = torch.rand((V, 256), device=dev)
data, sel = S.topk_cbsr(X, K)
g = S.MaxKGraph(indptr, indices, values)
y = g.forward(data, sel, 256, edge_sel=False)
torch.cuda.synchronize()
best = 1e9
for _ in range(3):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.forward(data, sel, 256, out=y, edge_sel=False)
    b.record()
    b.synchronize()
    best = min(best, a.elapsed_time(b) / reps)
print(f"{graph} k={K}: forward {best:.3f} ms", flush=True)
