#!/usr/bin/env python3
"""Functional (warp4) API vs the panel path on the Reddit shape (development tool)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd import maxk_cuda_kernels as MCK  # noqa: E402
from spgemm_new_amd.graphs import CONFIGS, synthetic_csr_gpu  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps


dev = torch.device("cuda:0")
V, E = CONFIGS["reddit"]
indptr, indices = synthetic_csr_gpu(V, E, device=dev)
values = torch.rand(E, device=dev)
X = torch.rand((V, 256), device=dev)
G = torch.rand((V, 256), device=dev)
data, sel = S.topk_cbsr(X, 32)
w4 = MCK.build_warp4_metadata(indptr)
nw = w4.numel() // 4
g = S.MaxKGraph(indptr, indices, values)
print("warp4 fwd", timed(lambda: MCK.spmm_maxk_forward(w4, indices, values, data, sel, nw, 32)))
print("warp4 bwd", timed(lambda: MCK.spmm_maxk_backward(w4, indices, values, G, sel, nw, 32)))
print("panel fwd", timed(lambda: g.forward(data, sel, 256)))
print("panel bwd", timed(lambda: g.backward(G, sel)))
