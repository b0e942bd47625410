#!/usr/bin/env python3
"""Timing emulation of an 8-wave TILE workgroup: with a
library built with -DTILE_EMU8 (tools/variants/lib_emu8.so) the plan puts each
group's records on waves 0-7 only (slot registers aliased, results wrong),
so 8 waves per CU carry twice the records while all 16 still run the DMA
sweep; groups may hold 2752 destinations (85 groups x 3 source ranges on
Reddit).  Times the given shapes (G,GS,P; default: the library's own shape).
Development tool.

usage: MAXK_LIB=... tools/exp_tile_emu8.py [graph] [reps] [G,GS,P ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd import _lib, ops, tile  # noqa: E402
from spgemm_new_amd.graphs import CONFIGS, synthetic_csr_gpu  # noqa: E402

graph = sys.argv[1] if len(sys.argv) > 1 else "reddit"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
shapes = [tuple(int(x) for x in s.split(",")) for s in sys.argv[3:]] or [None]
if "emu8" in os.environ.get("MAXK_LIB", ""):
    tile.max_group = lambda k: 2752 if k == 32 else 1376
K = 32
dev = torch.device("cuda:0")
V, E = CONFIGS[graph]
indptr, indices = synthetic_csr_gpu(V, E, device=dev)
gen = torch.Generator(device=dev)
gen.manual_seed(1)
values = torch.rand(E, generator=gen, device=dev)
X = torch.rand((V, 256), generator=gen, device=dev)
data, sel = S.topk_cbsr(X, K)
G = torch.rand((V, 256), generator=gen, device=dev)
g = S.MaxKGraph(indptr, indices, values)
dx = torch.empty((V, K), device=dev)
for shape in shapes:
    plan = tile.build(g.indptr, g.indices, g.values, V, V, k=K, shape=shape)
    if plan is None:
        print(shape, "no plan", flush=True)
        continue
    plan["values_key"], plan["values_ref"] = ops._tensor_key(g.values), g.values
    plan["part"] = torch.empty(max(1, plan["part_planes"] * V * K), device=dev)
    g._tile[K] = plan
    g.backward(G, sel, out=dx, algo=_lib.MAXK_BWD_TILE)
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(3):
        best = min(best, ops._min_ms(lambda: g.backward(G, sel, out=dx, algo=_lib.MAXK_BWD_TILE),
                                     reps=reps))
    nch = plan["num_chunks"].float()
    print(f"{graph} shape {plan['num_groups']} x {plan['group_size']} over "
          f"{plan['num_workgroups']} WGs: chunks/WG mean {nch.mean().item():.0f} max "
          f"{int(nch.max())}, records {plan['records'].shape[0] / 1e6:.1f} M: tile {best:.3f} ms",
          flush=True)
