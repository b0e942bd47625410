#!/usr/bin/env python3
"""Forward as NC column classes (A = [A_0 | ... | A_{NC-1}], one launch per class
on its CBSR slice, outputs summed) on the Reddit shape.  Development tool."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd.graphs import CONFIGS, synthetic_csr_gpu  # noqa: E402


def timed(fn, reps=10):
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
h, k = 256, 32
indptr, indices = synthetic_csr_gpu(V, E, device=dev)
values = torch.rand(E, device=dev)
X = torch.rand((V, h), device=dev)
data, sel = S.topk_cbsr(X, k)
g = S.MaxKGraph(indptr, indices, values)
y = torch.empty((V, h), device=dev)
print(f"NC=1: {timed(lambda: g.forward(data, sel, h, out=y)):.3f} ms", flush=True)
rows = torch.repeat_interleave(torch.arange(V, device=dev), (indptr[1:] - indptr[:-1]).long())
for NC in (2, 4, 8):
    cuts = [V * x // NC for x in range(NC + 1)]
    parts = []
    for x in range(NC):
        m = (indices >= cuts[x]) & (indices < cuts[x + 1])
        ip = torch.zeros(V + 1, dtype=torch.int32, device=dev)
        ip[1:] = torch.cumsum(torch.bincount(rows[m], minlength=V), 0)
        gx = S.MaxKGraph(ip, (indices[m] - cuts[x]).to(torch.int32).contiguous(),
                         values[m].contiguous(), num_cols=cuts[x + 1] - cuts[x])
        parts.append((gx, data[cuts[x]:cuts[x + 1]].contiguous(), sel[cuts[x]:cuts[x + 1]].contiguous()))
    ys = [torch.empty((V, h), device=dev) for _ in range(NC)]

    def run():
        for (gx, dx, sx), yx in zip(parts, ys):
            gx.forward(dx, sx, h, out=yx)
    t_launch = timed(run)

    def run_sum():
        run()
        torch.sum(torch.stack(ys), 0, out=y)
    t_all = timed(run_sum)
    err = float((y - g.forward(data, sel, h)).abs().max())
    print(f"NC={NC}: class launches {t_launch:.3f} ms, + sum {t_all:.3f} ms  (max diff {err:.2e})",
          flush=True)
    del parts, ys
    torch.cuda.empty_cache()
