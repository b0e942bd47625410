#!/usr/bin/env python3
"""Experiment: split the backward's destinations between LOCAL (columns < a*V)
and STAGED (the rest) and run both concurrently on two HIP streams.
Development tool; prints timings for several splits."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd import _lib  # noqa: E402
from spgemm_new_amd.graphs import CONFIGS, synthetic_csr_gpu  # noqa: E402
from spgemm_new_amd.models import cbsr_topk  # noqa: E402


def column_split(indptr, indices, values, cut):
    """CSR of A[:, :cut] and A[:, cut:] (columns renumbered)."""
    V = indptr.numel() - 1
    rows = torch.repeat_interleave(torch.arange(V, device=indptr.device),
                                   (indptr[1:] - indptr[:-1]).long())
    out = []
    for m, off in ((indices < cut, 0), (indices >= cut, cut)):
        r = rows[m]
        ip = torch.zeros(V + 1, dtype=torch.int32, device=indptr.device)
        ip[1:] = torch.cumsum(torch.bincount(r, minlength=V), 0).to(torch.int32)
        out.append((ip, (indices[m] - off).to(torch.int32).contiguous(), values[m].contiguous()))
    return out


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    dev = torch.device("cuda:0")
    graph = sys.argv[1] if len(sys.argv) > 1 else "reddit"
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    V, E = CONFIGS[graph]
    h = 256
    indptr, indices = synthetic_csr_gpu(V, E, device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(124)
    values = torch.rand(E, generator=gen, device=dev)
    X = torch.rand((V, h), generator=gen, device=dev)
    G = torch.rand((V, h), generator=gen, device=dev)
    _, sel = cbsr_topk(X, k)
    full = S.MaxKGraph(indptr, indices, values)
    ref = full.backward(G, sel, algo=_lib.MAXK_BWD_STAGED)
    for algo, name in ((_lib.MAXK_BWD_STAGED, "staged"), (_lib.MAXK_BWD_LOCAL, "local")):
        print(f"{graph} k={k} full {name}: {timed(lambda: full.backward(G, sel, algo=algo)):.3f} ms",
              flush=True)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for a in (0.25, 0.35, 0.45, 0.55):
        cut = int(V * a)
        (ipL, ixL, vL), (ipS, ixS, vS) = column_split(indptr, indices, values, cut)
        gL = S.MaxKGraph(ipL, ixL, vL, num_cols=cut)
        gS = S.MaxKGraph(ipS, ixS, vS, num_cols=V - cut)
        selL, selS = sel[:cut].contiguous(), sel[cut:].contiguous()
        dxL = torch.empty((cut, k), device=dev)
        dxS = torch.empty((V - cut, k), device=dev)
        gL.backward(G, selL, out=dxL, algo=_lib.MAXK_BWD_LOCAL)
        gS.backward(G, selS, out=dxS, algo=_lib.MAXK_BWD_STAGED)
        torch.cuda.synchronize()

        def both():
            cur = torch.cuda.current_stream()
            s1.wait_stream(cur)
            s2.wait_stream(cur)
            with torch.cuda.stream(s1):
                gL.backward(G, selL, out=dxL, algo=_lib.MAXK_BWD_LOCAL)
            with torch.cuda.stream(s2):
                gS.backward(G, selS, out=dxS, algo=_lib.MAXK_BWD_STAGED)
            cur.wait_stream(s1)
            cur.wait_stream(s2)

        tl = timed(lambda: gL.backward(G, selL, out=dxL, algo=_lib.MAXK_BWD_LOCAL))
        ts = timed(lambda: gS.backward(G, selS, out=dxS, algo=_lib.MAXK_BWD_STAGED))
        tb = timed(both)
        err = float((torch.cat([dxL, dxS]) - ref).abs().max())
        print(f"a={a:.2f}: local {tl:.3f} staged {ts:.3f} concurrent {tb:.3f} ms  maxerr {err:.2e}",
              flush=True)
        del gL, gS


if __name__ == "__main__":
    main()
