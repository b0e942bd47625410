#!/usr/bin/env python3
"""ATOMIC backward run eagerly 50 times on one input vs the fp64 oracle (development tool)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd import _lib  # noqa: E402
from spgemm_new_amd.graphs import random_cbsr, small_csr  # noqa: E402
from oracle import oracle as O  # noqa: E402

dev = torch.device("cuda:0")
k = int(sys.argv[1]) if len(sys.argv) > 1 else 32
indptr, indices = small_csr(3000, seed=21)
values = np.random.default_rng(2).random(len(indices), dtype=np.float32)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
v, h = len(indptr) - 1, 256
_, sel = random_cbsr(v, k, h, seed=3)
grad = np.random.default_rng(4).random((v, h), dtype=np.float32)
g = S.MaxKGraph(T(indptr), T(indices), T(values))
ref = O.np_backward(indptr, indices, values, grad, sel)
bad = 0
dx = torch.empty((v, k), device=dev)
for it in range(50):
    dx.fill_(float("nan") if it % 2 else 1e30)
    g.backward(T(grad), T(sel), out=dx, algo=_lib.MAXK_BWD_ATOMIC)
    e = O.parity_error(dx.cpu().numpy(), ref)
    if e > 1e-4:
        bad += 1
        print(f"iter {it}: err {e:.3e}", flush=True)
print(f"eager ATOMIC k={k}: {bad}/50 wrong", flush=True)
