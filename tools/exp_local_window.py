#!/usr/bin/env python3
"""Experiment: does the LOCAL backward slow down because its G-row window leaves L2?
Same V, E and k as Reddit, but every edge's source row is drawn from [0, W).  Small W keeps the
whole G window L2-resident on every XCD.  Development tool; prints timings per W."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd import _lib  # noqa: E402
from spgemm_new_amd.models import cbsr_topk  # noqa: E402


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def window_csr(V, E, W, dev, gen):
    rows = torch.randint(0, W, (E,), generator=gen, device=dev, dtype=torch.int64)
    cols = torch.randint(0, V, (E,), generator=gen, device=dev, dtype=torch.int64)
    key = torch.sort(rows * V + cols).values
    rows, cols = key // V, key % V
    indptr = torch.zeros(V + 1, dtype=torch.int32, device=dev)
    indptr[1:] = torch.cumsum(torch.bincount(rows, minlength=V), 0).to(torch.int32)
    return indptr, cols.to(torch.int32)


def main():
    dev = torch.device("cuda:0")
    V, E, k, h = 232965, 114615892, 32, 256
    gen = torch.Generator(device=dev)
    gen.manual_seed(7)
    X = torch.rand((V, h), generator=gen, device=dev)
    G = torch.rand((V, h), generator=gen, device=dev)
    _, sel = cbsr_topk(X, k)
    for W in (2000, 8000, 32000, V):
        indptr, indices = window_csr(V, E, W, dev, gen)
        values = torch.rand(indices.numel(), generator=gen, device=dev)
        g = S.MaxKGraph(indptr, indices, values)
        out = []
        for algo, name in ((_lib.MAXK_BWD_LOCAL, "local"), (_lib.MAXK_BWD_STAGED, "staged"),
                           (_lib.MAXK_BWD_ATOMIC, "atomic")):
            out.append(f"{name} {timed(lambda: g.backward(G, sel, algo=algo)):.3f}")
        print(f"W={W}: " + "  ".join(out) + " ms", flush=True)
        del g, indptr, indices, values
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
