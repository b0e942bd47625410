#!/usr/bin/env python3
"""Column-blocked forward with the blocks run as nb accumulating calls into Y
(no partial buffer) against the shipped partials + maxk_rows_sum form.
Development tool.

usage: tools/exp_fwd_acc.py [graph] [k] [nb ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd import _lib, ops  # noqa: E402
from spgemm_new_amd.graphs import CONFIGS, synthetic_csr_gpu  # noqa: E402

graph = sys.argv[1] if len(sys.argv) > 1 else "reddit"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 32
NBS = [int(x) for x in sys.argv[3:]] or [3, 4, 6]
dev = torch.device("cuda:0")
V, E = CONFIGS[graph]
indptr, indices = synthetic_csr_gpu(V, E, device=dev)
values = torch.rand(E, device=dev)
X = torch.rand((V, 256), device=dev)
data, sel = S.topk_cbsr(X, K)
g = S.MaxKGraph(indptr, indices, values)
ref = g.forward(data, sel, 256, edge_sel=False)
out = torch.empty_like(ref)
L = _lib.load()


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


for nb in NBS:
    plan = g.blocked_plan(nb)
    vals = g._blocked_values(plan, g.values)
    ip = plan["indptr"]
    subs = []
    for b in range(nb):
        e0, e1 = int(ip[b * V]), int(ip[(b + 1) * V])
        sub = S.MaxKGraph((ip[b * V:(b + 1) * V + 1] - e0).contiguous(), plan["indices"][e0:e1],
                          vals[e0:e1], num_cols=V)
        ws = sub._workspace(("fwd", 256), L.maxk_forward_workspace_bytes(sub.num_panels, 256))
        subs.append((sub, ws))

    def run():
        for b, (sub, ws) in enumerate(subs):
            flags = _lib.MAXK_FWD_CACHED_GATHER | (_lib.MAXK_FWD_ACCUMULATE if b else 0)
            _lib.check(L.maxk_spgemm_forward_ex(sub.sched.data_ptr(), sub.num_panels,
                                                sub.indptr.data_ptr(), sub.indices.data_ptr(),
                                                sub.values.data_ptr(), data.data_ptr(), sel.data_ptr(),
                                                V, 256, K, flags, out.data_ptr(), ws.data_ptr(),
                                                ws.numel(), None), "fwd")
    ta = ev(run)
    err = ((out - ref).abs().max() / ref.abs().max()).item()
    tp = ev(lambda: ops._forward_blocked(g, nb, data, sel, 256, out, g.values))
    print(f"{graph} k={K} nb={nb}: accumulate {ta:.3f} ms (rel diff {err:.1e}), partials {tp:.3f} ms",
          flush=True)
    del subs
    g._blocked.clear()
    g._ws.clear()
    torch.cuda.empty_cache()
