#!/usr/bin/env python3
"""Experiment: effect of column-sorted CBSR rows on every kernel (dev tool)."""
import os, sys, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S
from spgemm_new_amd import _lib
from spgemm_new_amd.graphs import CONFIGS, synthetic_csr_gpu
from spgemm_new_amd.models import cbsr_topk


def timed(fn, reps=10):
    fn(); torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


dev = torch.device("cuda:0")
graph = sys.argv[1] if len(sys.argv) > 1 else "reddit"
for k in [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "32").split(",")]:
    V, E = CONFIGS[graph]
    indptr, indices = synthetic_csr_gpu(V, E, device=dev)
    gen = torch.Generator(device=dev); gen.manual_seed(124)
    values = torch.rand(E, generator=gen, device=dev)
    X = torch.rand((V, 256), generator=gen, device=dev)
    G = torch.rand((V, 256), generator=gen, device=dev)
    data, sel = cbsr_topk(X, k)
    ss, order = torch.sort(sel, dim=1)
    ds = torch.gather(data, 1, order).contiguous(); ss = ss.contiguous()
    g = S.MaxKGraph(indptr, indices, values)
    for name, (d, s) in (("topk-order", (data, sel)), ("col-sorted", (ds, ss))):
        tf = timed(lambda: g.forward(d, s, 256))
        tS = timed(lambda: g.backward(G, s, algo=_lib.MAXK_BWD_STAGED))
        tL = timed(lambda: g.backward(G, s, algo=_lib.MAXK_BWD_LOCAL))
        tA = timed(lambda: g.backward(G, s, algo=_lib.MAXK_BWD_ATOMIC), 3)
        print(f"{graph} k={k} {name}: fwd {tf:.3f}  staged {tS:.3f}  local {tL:.3f}  atomic {tA:.3f} ms", flush=True)
    del g
