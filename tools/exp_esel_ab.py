#!/usr/bin/env python3
"""Same-box A/B of the edge-selector backward forms on one shape: forward
(writing the edge selectors) + backward with EDGE_GATHER, STAGED_EDGE and plain
STAGED (whose forward writes none), alternated `rounds` times, mean ms over
`reps` calls per round.  Development tool behind MAXK_AUTO=fixed's k rule.

usage: tools/exp_esel_ab.py [graph] [k] [rounds] [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd import _lib  # noqa: E402
from spgemm_new_amd.graphs import CONFIGS, synthetic_csr_gpu  # noqa: E402

graph = sys.argv[1] if len(sys.argv) > 1 else "products"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 8
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
h = 256
dev = torch.device("cuda:0")
V, E = CONFIGS[graph]
indptr, indices = synthetic_csr_gpu(V, E, device=dev)
gen = torch.Generator(device=dev)
gen.manual_seed(1)
values = torch.rand(E, generator=gen, device=dev)
X = torch.rand((V, h), generator=gen, device=dev)
G = torch.rand((V, h), generator=gen, device=dev)
data, sel = S.topk_cbsr(X, K)
del X
g = S.MaxKGraph(indptr, indices, values)
y = torch.empty((V, h), device=dev)
dx = torch.empty((V, K), device=dev)
forms = {"edge_gather": _lib.MAXK_BWD_EDGE_GATHER, "staged_edge": _lib.MAXK_BWD_STAGED_EDGE,
         "staged": _lib.MAXK_BWD_STAGED}


def step(algo):
    if algo == _lib.MAXK_BWD_STAGED:
        g._esel_on.discard((K, h))
    else:
        g._esel_on.add((K, h))
    g.forward(data, sel, h, out=y)
    g.backward(G, sel, out=dx, algo=algo)


def ms(fn):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps


sums = {}
for name, algo in forms.items():
    step(algo)
    torch.cuda.synchronize()
    sums[name] = dx.double().sum().item()
res = {n: [] for n in forms}
for r in range(rounds):
    for name, algo in forms.items():
        res[name].append(ms(lambda: step(algo)))
for name, algo in forms.items():
    t = res[name]
    step(algo)
    f_ms = ms(lambda: g.forward(data, sel, h, out=y))
    b_ms = ms(lambda: g.backward(G, sel, out=dx, algo=algo))
    print(f"{graph} k={K} {name:12s} fwd+bwd ms per round {' '.join(f'{x:.3f}' for x in t)}  "
          f"min {min(t):.3f} (fwd {f_ms:.3f} + bwd {b_ms:.3f} alone)  checksum {sums[name]:.9e}",
          flush=True)
