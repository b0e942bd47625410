#!/usr/bin/env python3
"""TILE backward run-to-run bit equality on a BASELINE graph (n calls).  Development tool.

usage: tools/exp_tile_determinism.py [graph] [k] [n]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd import _lib  # noqa: E402
from spgemm_new_amd.graphs import CONFIGS, synthetic_csr_gpu  # noqa: E402

graph = sys.argv[1] if len(sys.argv) > 1 else "products"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 32
n = int(sys.argv[3]) if len(sys.argv) > 3 else 6
dev = torch.device("cuda:0")
V, E = CONFIGS[graph]
indptr, indices = synthetic_csr_gpu(V, E, device=dev)
g = S.MaxKGraph(indptr, indices, torch.rand(E, device=dev))
G = torch.rand((V, 256), device=dev)
_, sel = S.topk_cbsr(torch.rand((V, 256), device=dev), K)
assert g.tile_plan(K) is not None
ref = g.backward(G, sel, algo=_lib.MAXK_BWD_TILE)
st = g.backward(G, sel, algo=_lib.MAXK_BWD_STAGED)
bad = 0
for i in range(n):
    d = g.backward(G, sel, algo=_lib.MAXK_BWD_TILE)
    if not torch.equal(d, ref):
        bad += 1
        print(f"  call {i}: differs in {int((d != ref).sum())} entries, max {float((d - ref).abs().max()):.3e}")
rel = float((ref - st).abs().max() / st.abs().max())
print(f"{graph} k={K}: {n} repeat calls, {bad} differ; TILE vs STAGED max rel {rel:.2e}", flush=True)
