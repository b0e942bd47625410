#!/usr/bin/env python3
"""TILE backward alone on the bench graph: mean ms over `reps` calls (best of 3
runs) and a checksum of dXs, for comparing builds of the library (MAXK_LIB).
Development tool.

usage: MAXK_LIB=... tools/exp_tile_time.py [graph] [k] [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd import _lib  # noqa: E402
from spgemm_new_amd.graphs import CONFIGS, synthetic_csr_gpu  # noqa: E402

graph = sys.argv[1] if len(sys.argv) > 1 else "reddit"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 32
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
dev = torch.device("cuda:0")
V, E = CONFIGS[graph]
indptr, indices = synthetic_csr_gpu(V, E, device=dev)
gen = torch.Generator(device=dev)
gen.manual_seed(1)
values = torch.rand(E, generator=gen, device=dev)
X = torch.rand((V, 256), generator=gen, device=dev)
G = torch.rand((V, 256), generator=gen, device=dev)
data, sel = S.topk_cbsr(X, K)
g = S.MaxKGraph(indptr, indices, values)
if g.tile_plan(K) is None:
    print(f"{graph} k={K}: no TILE plan")
    sys.exit(0)
dx = torch.empty((V, K), device=dev)


def call():
    g.backward(G, sel, out=dx, algo=_lib.MAXK_BWD_TILE)


call()
torch.cuda.synchronize()
best = float("inf")
for _ in range(3):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        call()
    b.record()
    b.synchronize()
    best = min(best, a.elapsed_time(b) / reps)
print(f"{graph} k={K} tile {best:.3f} ms  checksum {dx.double().sum().item():.9e}", flush=True)
