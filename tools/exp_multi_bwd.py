"""Proteins R=8 (BASELINE config 5) multi-relation backward: LOCAL rel8 vs the
relation-summing STAGED backward (CSC-order and edge-order staging rows), each
timed with HIP events (min / median of N), cross-checked against rel8 and the
adjoint identity.  Usage: python tools/exp_multi_bwd.py [--reps 10] [--k 32]"""
import argparse
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd import _lib  # noqa: E402
from spgemm_new_amd.graphs import synthetic_columns, synthetic_indptr, synthetic_values  # noqa: E402


def timed(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    return min(ts), statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--R", type=int, default=8)
    ap.add_argument("--algos", default="rel8,multi_staged,multi_edge_gather")
    ap.add_argument("--fwd", action="store_true", help="also time forward_multi")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    V, E, h, R, k = 132534, 79122504, 256, a.R, a.k
    t0 = time.time()
    indptr = synthetic_indptr(V, E, seed=123, device=dev)
    indices = synthetic_columns(indptr, seed=123)
    vals = torch.stack([synthetic_values(130 + q, 0, E, device=dev) for q in range(R)],
                       dim=1).contiguous()
    g = S.MaxKGraph(indptr, indices, vals[:, 0].contiguous())
    gen = torch.Generator(device=dev)
    gen.manual_seed(124)
    X = torch.rand((V, h), generator=gen, device=dev)
    G = torch.rand((R, V, h), generator=gen, device=dev)
    data, sel = S.topk_cbsr(X, k)
    print(f"graph built in {time.time() - t0:.1f}s", flush=True)
    algos = {"rel8": _lib.MAXK_BWD_LOCAL, "multi_staged": _lib.MAXK_BWD_MULTI_STAGED,
             "multi_edge_gather": _lib.MAXK_BWD_MULTI_EDGE_GATHER}
    res = {}
    for name in a.algos.split(","):
        out = torch.empty((V, k), device=dev)
        mn, md = timed(lambda: g.backward_multi(G, sel, vals, out=out, algo=algos[name]), a.reps)
        res[name] = out
        print(f"{name}: min {mn:.3f} ms  median {md:.3f} ms  ({g.last_bwd_algo})", flush=True)
    y = g.forward_multi(data, sel, vals, h)
    if a.fwd:
        mn, md = timed(lambda: g.forward_multi(data, sel, vals, h, out=y), a.reps)
        print(f"forward_multi: min {mn:.3f} ms  median {md:.3f} ms  checksum "
              f"{float(y.double().sum()):.6e}", flush=True)
    lhs = float((y.double() * G.double()).sum())
    del y
    for name, dx in res.items():
        rhs = float((data.double() * dx.double()).sum())
        ref = res[next(iter(res))]
        err = float(((dx - ref).abs() / ref.abs().clamp_min(1)).max())
        print(f"{name}: adjoint rel err {abs(lhs - rhs) / abs(lhs):.2e}, vs first {err:.2e}",
              flush=True)


if __name__ == "__main__":
    main()
