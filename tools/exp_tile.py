#!/usr/bin/env python3
"""TILE backward vs LOCAL on one shape: plan build time, plan shape, timing of
each alone, and max difference.  Development tool.

usage: tools/exp_tile.py [graph] [reps]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd import _lib  # noqa: E402
from spgemm_new_amd.graphs import CONFIGS, synthetic_csr_gpu  # noqa: E402


def ev(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps


graph = sys.argv[1] if len(sys.argv) > 1 else "reddit"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
K = int(sys.argv[3]) if len(sys.argv) > 3 else 32
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
t0 = time.time()
plan = g.tile_plan(K)
torch.cuda.synchronize()
print(f"{graph}: plan {time.time() - t0:.2f} s", flush=True)
if plan is None:
    print("no TILE plan (segment overflow)")
    sys.exit(0)
print(f"  groups {plan['num_groups']} x {plan['group_size']}, workgroups {plan['num_workgroups']}, "
      f"chunks/WG max {int(plan['num_chunks'].max())} mean "
      f"{plan['num_chunks'].float().mean().item():.0f}, records {plan['records'].shape[0] / 1e6:.1f} M "
      f"({plan['records'].shape[0] / E:.2f} per edge)", flush=True)
dx_t = torch.empty((V, K), device=dev)
dx_l = torch.empty((V, K), device=dev)
g.backward(G, sel, out=dx_t, algo=_lib.MAXK_BWD_TILE)
g.backward(G, sel, out=dx_l, algo=_lib.MAXK_BWD_LOCAL)
torch.cuda.synchronize()
diff = (dx_t - dx_l).abs().max().item()
print(f"  max |tile - local| = {diff:.3e} (max |local| {dx_l.abs().max().item():.3e})", flush=True)
t_tile = ev(lambda: g.backward(G, sel, out=dx_t, algo=_lib.MAXK_BWD_TILE), reps)
t_loc = ev(lambda: g.backward(G, sel, out=dx_l, algo=_lib.MAXK_BWD_LOCAL), reps)
print(f"  tile {t_tile:.3f} ms   local {t_loc:.3f} ms", flush=True)
