#!/usr/bin/env python3
"""Backward algorithm timings on one shape: each algorithm alone (back-to-back
backward calls) and alternating with the forward (the bench step), to check
what MAXK_BWD_AUTO's measurement picks.  Development tool.

usage: tools/exp_autotune.py [graph] [k]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd import _lib  # noqa: E402
from spgemm_new_amd.graphs import CONFIGS, synthetic_csr_gpu  # noqa: E402


def ev(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps


graph = sys.argv[1] if len(sys.argv) > 1 else "products"
k = int(sys.argv[2]) if len(sys.argv) > 2 else 16
dev = torch.device("cuda:0")
V, E = CONFIGS[graph]
indptr, indices = synthetic_csr_gpu(V, E, device=dev)
gen = torch.Generator(device=dev)
gen.manual_seed(1)
values = torch.rand(E, generator=gen, device=dev)
X = torch.rand((V, 256), generator=gen, device=dev)
G = torch.rand((V, 256), generator=gen, device=dev)
data, sel = S.topk_cbsr(X, k)
g = S.MaxKGraph(indptr, indices, values)
y = torch.empty((V, 256), device=dev)
dx = torch.empty((V, k), device=dev)
g.backward(G, sel, out=dx)
print(f"{graph} k={k}: AUTO picked {g.last_bwd_algo}; autotune timings {g.bwd_timings}")
for name, a in (("staged", _lib.MAXK_BWD_STAGED), ("atomic", _lib.MAXK_BWD_ATOMIC),
                ("local", _lib.MAXK_BWD_LOCAL)):
    if a == _lib.MAXK_BWD_LOCAL and g.local_plan(k) is None:
        continue
    alone = ev(lambda: g.backward(G, sel, out=dx, algo=a))
    step = ev(lambda: (g.forward(data, sel, 256, out=y), g.backward(G, sel, out=dx, algo=a)))
    fwd = ev(lambda: g.forward(data, sel, 256, out=y))
    print(f"  {name:7s} alone {alone:.3f} ms   in step {step - fwd:.3f} ms (step {step:.3f}, fwd {fwd:.3f})",
          flush=True)
