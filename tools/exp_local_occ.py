#!/usr/bin/env python3
"""Experiment: LOCAL backward vs destinations-per-wave (occupancy) (dev tool)."""
import os, sys, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S
from spgemm_new_amd import _lib, ops
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
V, E = CONFIGS[graph]
indptr, indices = synthetic_csr_gpu(V, E, device=dev)
gen = torch.Generator(device=dev); gen.manual_seed(124)
values = torch.rand(E, generator=gen, device=dev)
X = torch.rand((V, 256), generator=gen, device=dev)
G = torch.rand((V, 256), generator=gen, device=dev)
for k in [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "32").split(",")]:
    _, sel = cbsr_topk(X, k)
    ref = None
    for lds_kb, wpc in ((20, 8), (10, 16), (8, 20), (6, 24), (5, 32), (4, 32)):
        ops.LOCAL_WAVE_LDS_BYTES = lds_kb * 1024
        ops.LOCAL_WAVES_PER_CU = wpc
        g = S.MaxKGraph(indptr, indices, values)
        plan = g.local_plan(k)
        out = g.backward(G, sel, algo=_lib.MAXK_BWD_LOCAL)
        if ref is None:
            ref = g.backward(G, sel, algo=_lib.MAXK_BWD_STAGED).clone()
        err = float((out - ref).abs().max())
        t = timed(lambda: g.backward(G, sel, algo=_lib.MAXK_BWD_LOCAL))
        print(f"{graph} k={k} lds/wave={lds_kb}KB dmax={plan['dmax']} waves={plan['num_waves']}: "
              f"{t:.3f} ms (err {err:.1e})", flush=True)
        del g
