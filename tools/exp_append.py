#!/usr/bin/env python3
"""APPEND backward vs the deterministic algorithms on the BASELINE shapes
(round 6).  Development tool: per shape, forward (with
the edge selectors written when the backward reads them) and backward times,
median of `reps` HIP-event-timed calls, and each result's max relative
difference to STAGED.

usage: tools/exp_append.py [products|reddit|proteins|all|staged] [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd import _lib  # noqa: E402
from spgemm_new_amd.graphs import (CONFIGS, synthetic_columns, synthetic_indptr,  # noqa: E402
                                   synthetic_values)

ESEL = (_lib.MAXK_BWD_STAGED_EDGE, _lib.MAXK_BWD_EDGE_GATHER, _lib.MAXK_BWD_APPEND_EDGE)
NAMES = {_lib.MAXK_BWD_STAGED: "staged", _lib.MAXK_BWD_STAGED_EDGE: "staged_edge",
         _lib.MAXK_BWD_EDGE_GATHER: "edge_gather", _lib.MAXK_BWD_APPEND: "append",
         _lib.MAXK_BWD_APPEND_EDGE: "append_edge", _lib.MAXK_BWD_TILE: "tile",
         _lib.MAXK_BWD_MULTI_STAGED: "multi_staged", _lib.MAXK_BWD_MULTI_APPEND: "multi_append",
         _lib.MAXK_BWD_MULTI_EDGE_GATHER: "multi_edge_gather"}


def med(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def rel(a, b):
    return float(((a - b).abs() / b.abs().clamp_min(1)).max())


def graph(name, dev, seed=123):
    V, E = CONFIGS[name]
    indptr = synthetic_indptr(V, E, seed=seed, device=dev)
    indices = synthetic_columns(indptr, seed=seed)
    return V, indptr, indices


def single(name, ks, algos, reps, dev):
    V, indptr, indices = graph(name, dev)
    values = synthetic_values(123, 0, indices.numel(), device=dev)
    g = S.MaxKGraph(indptr, indices, values)
    gen = torch.Generator(device=dev)
    gen.manual_seed(124)
    h = 256
    X = torch.rand((V, h), generator=gen, device=dev)
    G = torch.rand((V, h), generator=gen, device=dev)
    y = torch.empty((V, h), device=dev)
    for k in ks:
        data, sel = S.topk_cbsr(X, k)
        dx = torch.empty((V, k), device=dev)
        ref = g.backward(G, sel, algo=_lib.MAXK_BWD_STAGED).clone()
        for a in algos:
            if a == _lib.MAXK_BWD_TILE and g.tile_plan(k) is None:
                continue
            es = a in ESEL
            tf = med(lambda: g.forward(data, sel, h, out=y, edge_sel=es), reps)
            g.forward(data, sel, h, out=y, edge_sel=es)
            tb = med(lambda: g.backward(G, sel, out=dx, algo=a), reps)
            bits = int(dx.view(torch.int32).to(torch.int64).sum())
            print(f"{name} k={k} {NAMES[a]:12s} fwd {tf:.3f} bwd {tb:.3f} step {tf + tb:.3f} ms"
                  f"  | vs staged {rel(dx, ref):.1e} bits {bits}", flush=True)
        del data, sel, dx, ref
        g._ws.clear()
        g._esel.clear()
        g._tile.clear()
        g._append.clear()
        torch.cuda.empty_cache()


def proteins(reps, dev):
    V, indptr, indices = graph("proteins", dev)
    R, k, h = 8, 32, 256
    vals = torch.stack([synthetic_values(130 + q, 0, indices.numel(), device=dev)
                        for q in range(R)], dim=1).contiguous()
    g = S.MaxKGraph(indptr, indices, vals[:, 0].contiguous())
    gen = torch.Generator(device=dev)
    gen.manual_seed(124)
    X = torch.rand((V, h), generator=gen, device=dev)
    G = torch.rand((R, V, h), generator=gen, device=dev)
    data, sel = S.topk_cbsr(X, k)
    dx = torch.empty((V, k), device=dev)
    ref = g.backward_multi(G, sel, vals, algo=_lib.MAXK_BWD_MULTI_STAGED).clone()
    for a in (_lib.MAXK_BWD_MULTI_STAGED, _lib.MAXK_BWD_MULTI_EDGE_GATHER, _lib.MAXK_BWD_MULTI_APPEND):
        tb = med(lambda: g.backward_multi(G, sel, vals, out=dx, algo=a), reps)
        bits = int(dx.view(torch.int32).to(torch.int64).sum())
        print(f"proteins R=8 k=32 {NAMES[a]:12s} bwd {tb:.3f} ms | vs multi_staged "
              f"{rel(dx, ref):.1e} bits {bits}", flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "one":   # one <graph> <k> <algo name> [reps]
        code = {v: k_ for k_, v in NAMES.items()}[sys.argv[4]]
        single(sys.argv[2], (int(sys.argv[3]),), (code,),
               int(sys.argv[5]) if len(sys.argv) > 5 else 5, torch.device("cuda:0"))
        return
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    dev = torch.device("cuda:0")
    if what in ("products", "all"):
        single("products", (8, 16, 32, 64),
               (_lib.MAXK_BWD_STAGED, _lib.MAXK_BWD_STAGED_EDGE, _lib.MAXK_BWD_EDGE_GATHER,
                _lib.MAXK_BWD_APPEND, _lib.MAXK_BWD_APPEND_EDGE, _lib.MAXK_BWD_TILE), reps, dev)
    if what == "staged":   # the deterministic push forms only
        single("products", (8, 16, 32),
               (_lib.MAXK_BWD_STAGED, _lib.MAXK_BWD_STAGED_EDGE, _lib.MAXK_BWD_EDGE_GATHER), reps, dev)
    if what in ("reddit", "all"):
        single("reddit", (32,), (_lib.MAXK_BWD_TILE, _lib.MAXK_BWD_APPEND,
                                 _lib.MAXK_BWD_APPEND_EDGE), reps, dev)
    if what in ("proteins", "all"):
        proteins(reps, dev)


if __name__ == "__main__":
    main()
