#!/usr/bin/env python3
"""Column-blocked forward over row chunks (experiment): the graph cut into Q
row chunks, each run as its own blocked forward (nb blocks) into one shared
partial buffer, so a chunk's partial rows may still be in the Infinity Cache
when they are summed.  Development tool.

usage: tools/exp_fwd_chunks.py [graph] [k] [nb] [Q ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd import ops  # noqa: E402
from spgemm_new_amd.graphs import CONFIGS, synthetic_csr_gpu  # noqa: E402

graph = sys.argv[1] if len(sys.argv) > 1 else "reddit"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 32
NB = int(sys.argv[3]) if len(sys.argv) > 3 else 8
QS = [int(q) for q in sys.argv[4:]] or [1, 4, 8, 16]
dev = torch.device("cuda:0")
V, E = CONFIGS[graph]
indptr, indices = synthetic_csr_gpu(V, E, device=dev)
values = torch.rand(E, device=dev)
X = torch.rand((V, 256), device=dev)
data, sel = S.topk_cbsr(X, K)
g = S.MaxKGraph(indptr, indices, values)
ref = g.forward(data, sel, 256, edge_sel=False)
out = torch.empty_like(ref)


def ev(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) / reps)
    return best


for Q in QS:
    bounds = [V * q // Q for q in range(Q + 1)]
    shared = {}
    subs = []
    for q in range(Q):
        r0, r1 = bounds[q], bounds[q + 1]
        e0, e1 = int(indptr[r0]), int(indptr[r1])
        sg = S.MaxKGraph((indptr[r0:r1 + 1] - e0).contiguous(), indices[e0:e1], values[e0:e1],
                         num_cols=V)
        sg._ws = shared
        sg.blocked_plan(NB)
        subs.append((sg, r0, r1))

    def run():
        for sg, r0, r1 in subs:
            ops._forward_blocked(sg, NB, data, sel, 256, out[r0:r1], sg.values)
    t = ev(run)
    torch.cuda.synchronize()
    err = ((out - ref).abs().max() / ref.abs().max()).item()
    print(f"{graph} k={K} nb={NB} chunks={Q}: {t:.3f} ms (max rel diff {err:.1e})", flush=True)
    del subs, shared
    torch.cuda.empty_cache()
