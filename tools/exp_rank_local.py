#!/usr/bin/env python3
"""Per-rank compute of the partitioned Reddit path at world sizes 2/4/8 on ONE GPU:
builds rank 0's local CSR (own rows, own + halo columns renumbered as HaloPlan does)
without collectives and times its local forward + backward.  Development tool."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd.distributed import row_partition  # noqa: E402
from spgemm_new_amd.graphs import CONFIGS, synthetic_csr_gpu  # noqa: E402
from spgemm_new_amd.ops import topk_cbsr  # noqa: E402


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


def main():
    dev = torch.device("cuda:0")
    V, E = CONFIGS["reddit"]
    h, k = 256, 32
    indptr, indices = synthetic_csr_gpu(V, E, device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(5)
    values = torch.rand(E, generator=gen, device=dev)
    X = torch.rand((V, h), generator=gen, device=dev)
    G = torch.rand((V, h), generator=gen, device=dev)
    data, sel = topk_cbsr(X, k)
    for world in (1, 2, 4, 8):
        b = row_partition(indptr, world)
        for rank in sorted({0, world - 1}):
            r0, r1 = b[rank], b[rank + 1]
            e0, e1 = int(indptr[r0]), int(indptr[r1])
            cols = indices[e0:e1].long()
            own = (cols >= r0) & (cols < r1)
            halo = torch.unique(cols[~own])
            local = torch.empty_like(cols)
            local[own] = cols[own] - r0
            local[~own] = (r1 - r0) + torch.searchsorted(halo, cols[~own])
            lip = (indptr[r0:r1 + 1] - e0).to(torch.int32).contiguous()
            g = S.MaxKGraph(lip, local.to(torch.int32).contiguous(), values[e0:e1].contiguous(),
                            num_cols=(r1 - r0) + halo.numel())
            ids = torch.cat([torch.arange(r0, r1, device=dev), halo])
            d_l, s_l = data[ids].contiguous(), sel[ids].contiguous()
            g_l = G[r0:r1].contiguous()
            y = torch.empty((r1 - r0, h), device=dev)
            dx = torch.empty((ids.numel(), k), device=dev)
            g.backward(g_l, s_l, out=dx)  # autotune
            tf = timed(lambda: g.forward(d_l, s_l, h, out=y))
            tb = timed(lambda: g.backward(g_l, s_l, out=dx))
            msg = ""
            if world > 1:  # the overlap split: own-column and halo-column blocks
                li = local
                rows = torch.repeat_interleave(torch.arange(r1 - r0, device=dev),
                                               (lip[1:] - lip[:-1]).long())
                lv = values[e0:e1]
                parts = []
                for m, shift, nc in ((li < (r1 - r0), 0, r1 - r0),
                                     (li >= (r1 - r0), r1 - r0, halo.numel())):
                    ip = torch.zeros(r1 - r0 + 1, dtype=torch.int32, device=dev)
                    ip[1:] = torch.cumsum(torch.bincount(rows[m], minlength=r1 - r0), 0)
                    parts.append(S.MaxKGraph(ip, (li[m] - shift).to(torch.int32).contiguous(),
                                             lv[m].contiguous(), num_cols=nc))
                go, gh = parts
                d_o, s_o = d_l[: r1 - r0].contiguous(), s_l[: r1 - r0].contiguous()
                d_h, s_h = d_l[r1 - r0:].contiguous(), s_l[r1 - r0:].contiguous()
                go.backward(g_l, s_o)
                gh.backward(g_l, s_h)
                tfo = timed(lambda: go.forward(d_o, s_o, h))
                tfh = timed(lambda: gh.forward(d_h, s_h, h))
                tbo = timed(lambda: go.backward(g_l, s_o))
                tbh = timed(lambda: gh.backward(g_l, s_h))
                msg = (f" | split fwd own {tfo:.3f} + halo {tfh:.3f}, bwd own {tbo:.3f} + halo "
                       f"{tbh:.3f} ms")
                del go, gh, parts
            print(f"world={world} rank={rank}: rows={r1 - r0} edges={e1 - e0} halo={halo.numel()} "
                  f"fwd {tf:.3f} ms bwd {tb:.3f} ms ({g.last_bwd_algo}) "
                  f"halo fwd {halo.numel() * 5 * k / 1e6:.1f} MB" + msg, flush=True)
            del g, d_l, s_l, g_l, y, dx
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
