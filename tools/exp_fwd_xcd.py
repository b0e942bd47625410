#!/usr/bin/env python3
"""Forward with source-column blocks pinned to XCDs (experiment): the CSR is
restacked block-major into NB x V rows (row b*V + r = row r's edges with
sources in block b), workgroup i runs the panels of block i % 8, and the NB
partial outputs are summed.  Needs a library built with -DFWD_XCD_EXP.
Development tool.

usage: tools/exp_fwd_xcd.py [graph] [k] [reps]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd import _lib  # noqa: E402
from spgemm_new_amd.graphs import CONFIGS, synthetic_csr_gpu  # noqa: E402

graph = sys.argv[1] if len(sys.argv) > 1 else "reddit"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 32
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
NB = int(sys.argv[4]) if len(sys.argv) > 4 else 8
dev = torch.device("cuda:0")
V, E = CONFIGS[graph]
indptr, indices = synthetic_csr_gpu(V, E, device=dev)
values = torch.rand(E, device=dev)
X = torch.rand((V, 256), device=dev)
data, sel = S.topk_cbsr(X, K)
g = S.MaxKGraph(indptr, indices, values)
L = _lib.load()
L.maxk_fwd_xmap_set.argtypes = [ctypes.POINTER(ctypes.c_int64)]
L.maxk_fwd_xmap_set.restype = ctypes.c_int


def xmap(vals):
    arr = (ctypes.c_int64 * 9)(*vals)
    assert L.maxk_fwd_xmap_set(arr) == 0


def ev(fn):
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


xmap([0] * 9)
y = g.forward(data, sel, 256, edge_sel=False)
print(f"{graph} k={K}: base forward {ev(lambda: g.forward(data, sel, 256, out=y, edge_sel=False)):.3f} ms",
      flush=True)
rows = torch.repeat_interleave(torch.arange(V, device=dev), indptr[1:] - indptr[:-1])
blk = (indices.long() * NB) // V
key = blk * V + rows
key, order = torch.sort(key, stable=True)
idx2 = indices[order].contiguous()
val2 = values[order].contiguous()
cnt = torch.bincount(key, minlength=NB * V)
indptr2 = torch.zeros(NB * V + 1, dtype=torch.int32, device=dev)
indptr2[1:] = torch.cumsum(cnt, 0).to(torch.int32)
g2 = S.MaxKGraph(indptr2, idx2, val2, num_cols=V)
y2 = torch.empty((NB * V, 256), device=dev)
srow = g2.sched.view(-1, 2)[:, 0].long()
P = g2.num_panels
xm = [int(torch.searchsorted(srow[:P].contiguous(), torch.tensor([b * V], device=dev)).item())
      for b in range(NB)] + [P]
print("  panels", P, flush=True)
for on in ((False, True) if NB == 8 else (False,)):
    xmap(xm if on else [0] * 9)
    t = ev(lambda: g2.forward(data, sel, 256, out=y2, edge_sel=False))
    print(f"  stacked forward, xcd map {on}: {t:.3f} ms", flush=True)
ysum = torch.empty_like(y)
tr = ev(lambda: torch.sum(y2.view(NB, V, 256), 0, out=ysum))
print(f"  reduction of {NB} partials: {tr:.3f} ms", flush=True)
xmap(xm if NB == 8 else [0] * 9)
g2.forward(data, sel, 256, out=y2, edge_sel=False)
torch.sum(y2.view(NB, V, 256), 0, out=ysum)
torch.cuda.synchronize()
print(f"  max rel diff vs base {((ysum - y).abs().max() / y.abs().max()).item():.2e}", flush=True)
xmap([0] * 9)
