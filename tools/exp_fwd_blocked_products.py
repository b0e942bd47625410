#!/usr/bin/env python3
"""Column-blocked forward on ogbn-products (round 6 experiment): the blocked form
(MaxKGraph.blocked_plan: the CSR restacked block-major, each pass gathering only
one block's CBSR rows, partial outputs summed in block order) is chosen on
long-row graphs only (mean degree >= 128, Reddit).  On products the CBSR table
(196 / 392 / 784 MB at k = 16 / 32 / 64) exceeds the 256 MB Infinity Cache, so
blocks of it would fit -- at the price of nb partial Y writes (2.5 GB each).
Median of 10 HIP-event calls per form, max rel. difference to the plain forward.

usage: tools/exp_fwd_blocked_products.py [k,...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd import ops  # noqa: E402
from spgemm_new_amd.graphs import (CONFIGS, synthetic_columns, synthetic_indptr,  # noqa: E402
                                   synthetic_values)


def med(fn, reps=10):
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
    return sorted(ts)[len(ts) // 2]


def main():
    ks = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "16,32,64").split(",")]
    dev = torch.device("cuda:0")
    V, E = CONFIGS["products"]
    indptr = synthetic_indptr(V, E, seed=123, device=dev)
    indices = synthetic_columns(indptr, seed=123)
    values = synthetic_values(123, 0, E, device=dev)
    g = S.MaxKGraph(indptr, indices, values)
    gen = torch.Generator(device=dev)
    gen.manual_seed(124)
    h = 256
    X = torch.rand((V, h), generator=gen, device=dev)
    y = torch.empty((V, h), device=dev)
    yb = torch.empty((V, h), device=dev)
    for k in ks:
        data, sel = S.topk_cbsr(X, k)
        t0 = med(lambda: g.forward(data, sel, h, out=y))
        print(f"products k={k} plain forward {t0:.3f} ms (blocks chosen {g._fwd_blocks})", flush=True)
        for nb in (2, 3, 4, 6):
            try:
                t = med(lambda: ops._forward_blocked(g, nb, data, sel, h, yb, g.values))
            except Exception as e:  # noqa: BLE001 -- report and go on
                print(f"  nb={nb}: {type(e).__name__}: {e}", flush=True)
                continue
            err = float(((yb - y).abs() / y.abs().clamp_min(1)).max())
            print(f"  nb={nb}: {t:.3f} ms  (vs plain {err:.1e})", flush=True)
            g._blocked.clear()
            for key in [kk for kk in g._ws if kk[0] in ("fwd_parts", "fwd_blocked")]:
                g._ws.pop(key)
            torch.cuda.empty_cache()
        del data, sel


if __name__ == "__main__":
    main()
