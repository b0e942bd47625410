"""Why TILE (splits = 1) and LOCAL differ in the last bit at k = 32 (products
full-size test) but not at k = 64: find mismatching dXs entries on a mid-size
graph with the TILE plan forced to one source range, and replay those entries'
sums on the host in source-row order with fp32 FMA (a*b + c exact in fp64,
rounded once to fp32) and with separate fp32 multiply and add."""
import sys

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__file__)))
import spgemm_new_amd as S  # noqa: E402
from spgemm_new_amd import _lib, ops, tile  # noqa: E402
from spgemm_new_amd.graphs import synthetic_csr_gpu  # noqa: E402

dev = torch.device("cuda")
V, E = 60000, 3_000_000
for k in (32, 64):
    indptr, indices = synthetic_csr_gpu(V, E, device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(3)
    vals = torch.rand(indices.numel(), generator=gen, device=dev)
    Gr = torch.rand((V, 256), generator=gen, device=dev)
    X = torch.rand((V, 256), generator=gen, device=dev)
    _, sel = S.topk_cbsr(X, k)
    g = S.MaxKGraph(indptr, indices, vals)
    mg = tile.max_group(k)
    ng = -(-V // mg)
    plan = tile.build(g.indptr, g.indices, g.values, V, V, shape=(ng, -(-V // ng), 1), k=k)
    plan["values_key"], plan["values_ref"] = ops._tensor_key(g.values), g.values
    plan["part"] = torch.empty(1, device=dev)
    g._tile[k] = plan
    t = g.backward(Gr, sel, algo=_lib.MAXK_BWD_TILE)
    for band_bytes in (1 << 40, 4 << 20):
        ops.LOCAL_BAND_BYTES = band_bytes
        g._local = {}
        loc = g.backward(Gr, sel, algo=_lib.MAXK_BWD_LOCAL)
        bad = (t != loc).nonzero()
        print(f"k={k} bands={g.local_bands(g.local_plan(k), 256)[1]} mismatches {bad.shape[0]} "
              f"of {t.numel()}")
    if bad.shape[0] == 0:
        continue
    ip, ix, vv = indptr.cpu().numpy(), indices.cpu().numpy(), vals.cpu().numpy()
    gn, sn = Gr.cpu().numpy(), sel.cpu().numpy()
    rows = np.repeat(np.arange(V), np.diff(ip))
    for c, l in bad[:5].tolist():
        es = np.nonzero(ix == c)[0]           # CSR order = source-row order
        col = sn[c, l]
        acc_fma, acc_sep = np.float32(0), np.float32(0)
        for e in es:
            a, b = np.float32(vv[e]), np.float32(gn[rows[e], col])
            acc_fma = np.float32(np.float64(a) * np.float64(b) + np.float64(acc_fma))
            acc_sep = np.float32(np.float32(a * b) + acc_sep)
        print(f"  ({c},{l}) deg {len(es)}: tile {t[c, l].item()!r} local {loc[c, l].item()!r} "
              f"seq-fma {float(acc_fma)!r} seq-mul-add {float(acc_sep)!r}")
