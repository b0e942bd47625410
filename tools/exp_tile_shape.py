#!/usr/bin/env python3
"""TILE backward time against the plan shape (groups x group size x
workgroups) on one graph: checks how the time splits between the rows a
workgroup sweeps and the records it processes.  Development tool.

usage: tools/exp_tile_shape.py [graph] [reps] [G,GS,P ...]  (P = G * S: S equal
source ranges per group; other P: pieces straddling groups)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd import _lib, ops, tile  # noqa: E402
from spgemm_new_amd.graphs import CONFIGS, synthetic_csr_gpu  # noqa: E402

graph = sys.argv[1] if len(sys.argv) > 1 else "reddit"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
world = 1
if graph.count("/"):                      # e.g. reddit/8: rank 0's row block of world 8
    graph, world = graph.split("/")[0], int(graph.split("/")[1])
shapes = [tuple(int(x) for x in s.split(",")) for s in sys.argv[3:]] or [None]
K = int(os.environ.get("TILE_K", "32"))
dev = torch.device("cuda:0")
V, E = CONFIGS[graph]
indptr, indices = synthetic_csr_gpu(V, E, device=dev)
gen = torch.Generator(device=dev)
gen.manual_seed(1)
values = torch.rand(E, generator=gen, device=dev)
X = torch.rand((V, 256), generator=gen, device=dev)
data, sel = S.topk_cbsr(X, K)
C = V                                     # destination columns (all nodes)
if world > 1:
    V = -(-V // world)
    E = int(indptr[V].item())
    indptr, indices, values = indptr[: V + 1].contiguous(), indices[:E].contiguous(), values[:E]
G = torch.rand((V, 256), generator=gen, device=dev)
g = S.MaxKGraph(indptr, indices, values, num_cols=C)
dx = torch.empty((C, K), device=dev)
ref = None
for shape in shapes:
    plan = tile.build(g.indptr, g.indices, g.values, V, C, k=K, shape=shape)
    if plan is None:
        print(shape, "no plan", flush=True)
        continue
    plan["values_key"], plan["values_ref"] = ops._tensor_key(g.values), g.values
    P = plan["num_workgroups"]
    plan["part"] = torch.empty(max(1, plan["part_planes"] * C * K), device=dev)
    g._tile[K] = plan
    g.backward(G, sel, out=dx, algo=_lib.MAXK_BWD_TILE)
    torch.cuda.synchronize()
    if ref is None:
        ref = dx.clone()
    diff = (dx - ref).abs().max().item()
    t = ops._min_ms(lambda: g.backward(G, sel, out=dx, algo=_lib.MAXK_BWD_TILE), reps=reps)
    nch = plan["num_chunks"].float()
    per_wg = [sum(int(nch[pc[0]]) for pc in tile.pieces_of(w, V, plan["num_groups"], P))
              for w in range(P)]
    print(f"{graph} shape {plan['num_groups']} x {plan['group_size']} over {P} WGs "
          f"(planes {plan['part_planes']}): tile {t:.3f} ms, chunks/WG max {max(per_wg)} "
          f"mean {sum(per_wg) / len(per_wg):.0f}, |diff| {diff:.2e}", flush=True)
