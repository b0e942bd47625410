#!/usr/bin/env python3
"""A rank's single-block local forward / backward at world sizes 4 and 8 (Reddit,
k=32, h=256, loopback exchange): column-block counts, panel costs and TILE source
ranges, to tune the rank blocks toward the N=1 kernels' per-edge rate (VERDICT r3
item 3).  Development tool.

usage: tools/exp_rank_fwd.py [--worlds 4,8] [--graph reddit]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import spgemm_new_amd.distributed as D  # noqa: E402
from exp_rank_step import Loopback, timed  # noqa: E402
from spgemm_new_amd import _lib  # noqa: E402
from spgemm_new_amd.graphs import CONFIGS, synthetic_csr_gpu  # noqa: E402
from spgemm_new_amd.ops import topk_cbsr  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graph", default="reddit")
    ap.add_argument("--worlds", default="4,8")
    ap.add_argument("--k", type=int, default=32)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    V, E = CONFIGS[a.graph]
    h, k = 256, a.k
    indptr, indices = synthetic_csr_gpu(V, E, device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(5)
    values = torch.rand(E, generator=gen, device=dev)
    X = torch.rand((V, h), generator=gen, device=dev)
    G = torch.rand((V, h), generator=gen, device=dev)
    data, sel = topk_cbsr(X, k)
    for world in [int(w) for w in a.worlds.split(",")]:
        bounds = D.row_partition(indptr, world)
        for pc in (None, 512, 1024, 2048):
            D.a2a = Loopback(indptr, indices, bounds, 0, data, sel)
            kw = {} if pc is None else {"panel_cost": pc}
            m = D.PartitionedMaxK(indptr, indices, values, 0, world, dev, halo_mode="records",
                                  overlap=False, **kw)
            d_l, s_l, g_l = m.local_rows(data), m.local_rows(sel), m.local_rows(G)
            dall, sall = m.gather_halo_cbsr(d_l, s_l)
            e = m.local
            y = torch.empty((e.num_rows, h), device=dev)
            res = []
            for nb in (0, 2, 3, 4, 6, 8):
                e._fwd_blocks[(k, h)] = nb
                res.append(f"nb{nb} {timed(lambda: e.forward(dall, sall, h, out=y)):.3f}")
                e._blocked.clear()
                e._ws.clear()
            print(f"world={world} panel_cost={e.panel_cost} panels={e.num_panels} "
                  f"rows={e.num_rows} edges={e.num_edges}: fwd " + ", ".join(res), flush=True)
            del m, e
            torch.cuda.empty_cache()
        # TILE shapes: source ranges
        for splits in (None, 1, 2, 3, 4):
            D.a2a = Loopback(indptr, indices, bounds, 0, data, sel)
            kw = {} if splits is None else {"tile_splits": splits}
            m = D.PartitionedMaxK(indptr, indices, values, 0, world, dev, halo_mode="records",
                                  overlap=False, **kw)
            d_l, s_l, g_l = m.local_rows(data), m.local_rows(sel), m.local_rows(G)
            dall, sall = m.gather_halo_cbsr(d_l, s_l)
            e = m.local
            dx = torch.empty((e.num_cols, k), device=dev)
            t = timed(lambda: e.backward(g_l, sall, out=dx, algo=_lib.MAXK_BWD_TILE))
            p = e.tile_plan(k)
            tl = timed(lambda: e.backward(g_l, sall, out=dx, algo=_lib.MAXK_BWD_LOCAL))
            print(f"world={world} tile shape {(p['num_groups'], p['group_size'], p['num_workgroups'])}: "
                  f"bwd tile {t:.3f} ms (local {tl:.3f})", flush=True)
            del m, e
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
