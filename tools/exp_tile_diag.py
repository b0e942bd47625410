#!/usr/bin/env python3
"""Which destinations a TILE variant gets wrong (vs STAGED), by wave / slot /
half of the register layout.  Development tool."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd import _lib  # noqa: E402
from spgemm_new_amd.graphs import random_cbsr  # noqa: E402

dev = torch.device("cuda:0")
V, deg, k = 9000, 120, 32
rng = np.random.default_rng(18000)
d = rng.poisson(deg, V)
ip = np.zeros(V + 1, np.int64)
ip[1:] = np.cumsum(d)
idx = np.concatenate([np.sort(rng.choice(V, size=x, replace=False)) for x in d])
indptr = torch.from_numpy(ip.astype(np.int32)).to(dev)
indices = torch.from_numpy(idx.astype(np.int32)).to(dev)
values = torch.rand(indices.numel(), device=dev)
g = S.MaxKGraph(indptr, indices, values)
data, sel = random_cbsr(V, k, 256, seed=3)
sel = torch.from_numpy(sel).to(dev)
G = torch.rand((V, 256), device=dev)
plan = g.tile_plan(k)
print("plan", plan["num_groups"], plan["group_size"], plan["num_workgroups"])
dt = g.backward(G, sel, algo=_lib.MAXK_BWD_TILE)
ds = g.backward(G, sel, algo=_lib.MAXK_BWD_STAGED)
torch.cuda.synchronize()
err = (dt - ds).abs().max(1).values.cpu().numpy()
bad = np.nonzero(err > 1e-3 * max(1.0, ds.abs().max().item()))[0]
print("bad destinations", len(bad), "of", V)
gs = plan["group_size"]
j = bad % gs
wave = j % 16
pair = j // 16
half = pair % 2
slot = pair // 2
print("waves", np.bincount(wave, minlength=16).tolist())
print("halves", np.bincount(half, minlength=2).tolist())
print("slots", np.bincount(slot, minlength=64).tolist())
lanes = ((dt - ds).abs() > 1e-3).sum(0).cpu().numpy()
print("bad entries per lane l", lanes.tolist())
r = (dt - ds)[torch.from_numpy(bad[:5]).to(dev)]
print("sample diffs", r[:, :8].cpu().numpy())

# explain each bad destination's difference by one in-edge's contribution
ipc, ixc, vlc = indptr.cpu().numpy(), indices.cpu().numpy(), values.cpu().numpy()
Gc, selc = G.cpu().numpy(), sel.cpu().numpy()
dtc, dsc = dt.cpu().numpy(), ds.cpu().numpy()
rows_of = [[] for _ in range(V)]
for r in range(V):
    for e in range(ipc[r], ipc[r + 1]):
        rows_of[ixc[e]].append((r, vlc[e]))
for c in bad[:8]:
    d = dtc[c] - dsc[c]
    contrib = [(r, v, v * Gc[r, selc[c].astype(np.int64)]) for r, v in rows_of[c]]
    miss = min(contrib, key=lambda x: np.abs(d + x[2]).max())
    dbl = min(contrib, key=lambda x: np.abs(d - x[2]).max())
    # a record applied with the wrong source row: d = v * (G[r2] - G[r]) for some r2
    print(f"dest {c} (wave {(c % gs) % 16}, slot {(c % gs) // 32}, half {((c % gs) // 16) % 2}): "
          f"|d| {np.abs(d).max():.3f}, in-edges {len(contrib)}, "
          f"missing-one fit {np.abs(d + miss[2]).max():.2e} (row {miss[0]}), "
          f"double-one fit {np.abs(d - dbl[2]).max():.2e} (row {dbl[0]})")
    best = None
    for r, v, x in contrib:
        # solve d = v*G[r2, sel] - x for r2 over all rows
        want = (d + x) / v
        err = np.abs(Gc[:, selc[c].astype(np.int64)] - want).max(1)
        r2 = int(err.argmin())
        if best is None or err[r2] < best[0]:
            best = (err[r2], r, r2)
    print(f"    wrong-row fit {best[0]:.2e}: edge from row {best[1]} used row {best[2]} "
          f"(delta {best[2] - best[1]})")
