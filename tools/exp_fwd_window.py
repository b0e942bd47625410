#!/usr/bin/env python3
"""Does the forward speed up when the gathered CBSR table is cache-resident?
Reddit-sized V and E, every edge's column drawn from [0, W): W = 2 K (L2),
32 K (Infinity Cache), V (the real case).  Development tool."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S  # noqa: E402


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps


dev = torch.device("cuda:0")
V, E, k, h = 232965, 114615892, 32, 256
gen = torch.Generator(device=dev)
gen.manual_seed(1)
X = torch.rand((V, h), generator=gen, device=dev)
data, sel = S.topk_cbsr(X, k)
for W in (2000, 8000, 32000, V):
    rows = torch.sort(torch.randint(0, V, (E,), generator=gen, device=dev)).values
    cols = torch.randint(0, W, (E,), generator=gen, device=dev)
    key = torch.sort(rows * V + cols).values
    rows, cols = key // V, key % V
    indptr = torch.zeros(V + 1, dtype=torch.int32, device=dev)
    indptr[1:] = torch.cumsum(torch.bincount(rows, minlength=V), 0).to(torch.int32)
    g = S.MaxKGraph(indptr, cols.to(torch.int32), torch.rand(E, generator=gen, device=dev))
    print(f"W={W}: fwd {timed(lambda: g.forward(data, sel, h)):.3f} ms", flush=True)
    del g, rows, cols, key, indptr
    torch.cuda.empty_cache()
