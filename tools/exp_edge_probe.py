#!/usr/bin/env python3
"""API edge cases on the GPU (development probe): empty graphs, empty rows,
zero columns, every forward form and backward algorithm on them.  Prints one
line per case: ok / the exception."""
import os
import sys
import traceback

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda:0")


def case(name, fn):
    try:
        r = fn()
        torch.cuda.synchronize()
        print(f"ok   {name}{'' if r is None else ': ' + str(r)}", flush=True)
    except Exception as e:  # noqa: BLE001
        print(f"FAIL {name}: {type(e).__name__}: {e}", flush=True)
        traceback.print_exc(limit=2)


def graph(V, C, E_per_row, seed=0):
    rng = np.random.default_rng(seed)
    deg = np.full(V, E_per_row, np.int64) if C > 0 else np.zeros(V, np.int64)
    deg = np.minimum(deg, C)
    indptr = np.zeros(V + 1, np.int32)
    indptr[1:] = np.cumsum(deg)
    idx = np.concatenate([np.sort(rng.choice(C, int(d), replace=False)) for d in deg]).astype(np.int32) \
        if deg.sum() else np.zeros(0, np.int32)
    vals = rng.random(len(idx)).astype(np.float32)
    T = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    return S.MaxKGraph(T(indptr), T(idx), T(vals), num_cols=C)


ALGOS = {"atomic": _lib.MAXK_BWD_ATOMIC, "staged": _lib.MAXK_BWD_STAGED, "local": _lib.MAXK_BWD_LOCAL,
         "tile": _lib.MAXK_BWD_TILE, "staged_edge": _lib.MAXK_BWD_STAGED_EDGE,
         "edge_gather": _lib.MAXK_BWD_EDGE_GATHER, "auto": _lib.MAXK_BWD_AUTO}
for (V, C, d) in [(0, 5, 0), (5, 0, 0), (5, 5, 0), (1, 1, 1), (3, 700, 2)]:
    for k in (8, 16, 32, 64):
        h = 256
        g = graph(V, C, d)
        X = torch.rand((C, h), device=dev)
        G = torch.rand((V, h), device=dev)
        tag = f"V={V} C={C} deg={d} k={k}"
        data, sel = S.topk_cbsr(X, k) if C > 0 else (torch.zeros((0, k), device=dev),
                                                     torch.zeros((0, k), dtype=torch.uint8, device=dev))
        case(f"{tag} forward", lambda: tuple(g.forward(data, sel, h).shape))
        case(f"{tag} forward esel", lambda: tuple(ops.spgemm_forward(g, data, sel, h, edge_sel=True).shape))
        if k >= 32:
            out = torch.empty((V, h), device=dev)
            case(f"{tag} forward blocked nb=3", lambda: tuple(ops._forward_blocked(g, 3, data, sel, h, out, g.values).shape))
        rec = S.cbsr_gather_records(data, sel) if C > 0 else torch.zeros((0, 5 * k), dtype=torch.uint8, device=dev)
        case(f"{tag} forward_records", lambda: tuple(g.forward_records(rec, k, h).shape))
        vals4 = torch.rand((g.num_edges, 4), device=dev)
        case(f"{tag} forward_multi R=4", lambda: tuple(g.forward_multi(data, sel, vals4, h).shape))
        G4 = torch.rand((4, V, h), device=dev)
        case(f"{tag} backward_multi R=4", lambda: tuple(g.backward_multi(G4, sel, vals4).shape))
        for an, a in ALGOS.items():
            def run(a=a):
                dx = g.backward(G, sel, algo=a)
                return (tuple(dx.shape), float(dx.abs().sum()) if dx.numel() else 0.0)
            case(f"{tag} backward {an}", run)
