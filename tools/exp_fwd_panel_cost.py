#!/usr/bin/env python3
"""Forward time against the merge-path panel cost (MaxKGraph(panel_cost=...)) on
one graph, AUTO=fixed (Reddit: column-blocked, 4 blocks).  Development tool.

usage: MAXK_AUTO=fixed tools/exp_fwd_panel_cost.py [graph] [k] [costs ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd import ops  # noqa: E402
from spgemm_new_amd.graphs import CONFIGS, synthetic_csr_gpu  # noqa: E402

graph = sys.argv[1] if len(sys.argv) > 1 else "reddit"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 32
costs = [int(c) for c in sys.argv[3:]] or [1024, 2048, 4096, 8192]
dev = torch.device("cuda:0")
V, E = CONFIGS[graph]
indptr, indices = synthetic_csr_gpu(V, E, device=dev)
gen = torch.Generator(device=dev)
gen.manual_seed(1)
values = torch.rand(E, generator=gen, device=dev)
X = torch.rand((V, 256), generator=gen, device=dev)
data, sel = S.topk_cbsr(X, K)
y = torch.empty((V, 256), device=dev)
for c in costs:
    g = S.MaxKGraph(indptr, indices, values, panel_cost=c)
    g.forward(data, sel, 256, out=y)
    torch.cuda.synchronize()
    t = min(ops._min_ms(lambda: g.forward(data, sel, 256, out=y), reps=20) for _ in range(3))
    print(f"{graph} k={K} panel_cost {c}: panels {g.num_panels} fwd {t:.3f} ms "
          f"blocks {g._fwd_blocks}  checksum {y.double().sum().item():.9e}", flush=True)
    del g
    torch.cuda.empty_cache()
