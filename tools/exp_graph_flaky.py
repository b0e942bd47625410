#!/usr/bin/env python3
"""Reproducer: captured step (top-k, forward, backward, scatter) replayed on new
inputs vs the same step run eagerly.  Reports which outputs differ.  Development tool."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd import _lib  # noqa: E402
from spgemm_new_amd.graphs import small_csr  # noqa: E402

dev = torch.device("cuda:0")
algo_name = sys.argv[1] if len(sys.argv) > 1 else "atomic"
k = int(sys.argv[2]) if len(sys.argv) > 2 else 8
skip = set(sys.argv[3].split(",")) if len(sys.argv) > 3 else set()
algo = {"atomic": _lib.MAXK_BWD_ATOMIC, "local": _lib.MAXK_BWD_LOCAL,
        "staged": _lib.MAXK_BWD_STAGED}[algo_name]
indptr, indices = small_csr(3000, seed=21)
values = np.random.default_rng(2).random(len(indices), dtype=np.float32)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
v, h = len(indptr) - 1, 256
g = S.MaxKGraph(T(indptr), T(indices), T(values))
x, gr = torch.empty((v, h), device=dev), torch.empty((v, h), device=dev)
d = torch.empty((v, k), device=dev)
s = torch.empty((v, k), dtype=torch.uint8, device=dev)
y, dx, gx = torch.empty((v, h), device=dev), torch.empty((v, k), device=dev), torch.empty((v, h), device=dev)


def step():
    if "topk" not in skip:
        S.topk_cbsr(x, k, data=d, sel=s)
    if "fwd" not in skip:
        g.forward(d, s, h, out=y)
    g.backward(gr, s, out=dx, algo=algo)
    if "scatter" not in skip:
        S.cbsr_scatter(dx, s, h, out=gx)


x.copy_(torch.rand((v, h), device=dev))
gr.copy_(torch.rand((v, h), device=dev))
S.topk_cbsr(x, k, data=d, sel=s)
step()
torch.cuda.synchronize()
graph = torch.cuda.CUDAGraph()
stream = torch.cuda.Stream()
stream.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(stream):
    with torch.cuda.graph(graph, stream=stream):
        step()
torch.cuda.current_stream().wait_stream(stream)
bad = 0
for it in range(20):
    x.copy_(torch.rand((v, h), device=dev))
    gr.copy_(torch.rand((v, h), device=dev))
    graph.replay()
    torch.cuda.synchronize()
    got = [t.clone() for t in (d, s, y, dx, gx)]
    step()
    torch.cuda.synchronize()
    ref = [d, s, y, dx, gx]
    diffs = []
    for name, a, b in zip(("data", "sel", "y", "dx", "gx"), got, ref):
        if not torch.allclose(a.float(), b.float(), rtol=1e-4, atol=1e-4):
            diffs.append(f"{name} maxdiff {float((a.float() - b.float()).abs().max()):.3e}")
    if diffs:
        bad += 1
        print(f"iter {it}: " + "; ".join(diffs), flush=True)
print(f"{algo_name} k={k} skip={sorted(skip)}: {bad}/20 replays differ", flush=True)
