"""Randomised parity sweep (GPU): many small random problems, every kernel
against the fp64 oracle.

Each seed draws a graph (square or rectangular -- a multi-GPU rank's row block
with halo columns --, zero-heavy / uniform / hub degree mixes), a panel
schedule granularity, k and h, signed edge values, and checks the forward
SpGEMM, all three backward SSpMM algorithms, the top-k CBSR producer, the
dense SpMM baseline and (power-of-two k) the multi-relation forward and
backward.  Sizes are small so the oracle finishes in milliseconds; the seeds
are fixed so a failure is reproducible by its test id.
"""
import numpy as np
import pytest
import torch

import spgemm_new_amd as S
from spgemm_new_amd import _lib

pytestmark = pytest.mark.gpu
TOL = 1e-4
KS = [1, 2, 3, 4, 5, 8, 12, 16, 24, 32, 48, 64, 100, 128, 256]


def T(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def draw(seed):
    rng = np.random.default_rng(1000 + seed)
    V = int(rng.integers(1, 400))
    C = V if rng.random() < 0.6 else int(rng.integers(1, 600))
    mix = rng.integers(0, 3)
    if mix == 0:      # zero-heavy
        deg = np.where(rng.random(V) < 0.5, 0, rng.integers(1, 8, V))
    elif mix == 1:    # uniform
        deg = rng.integers(0, 40, V)
    else:             # a few hubs
        deg = rng.integers(0, 6, V)
        deg[rng.integers(0, V, 3)] = rng.integers(100, 800, 3)
    deg = np.minimum(deg, C)
    indptr = np.zeros(V + 1, np.int64)
    indptr[1:] = np.cumsum(deg)
    indices = np.empty(int(indptr[-1]), np.int32)
    for r in range(V):
        if deg[r]:
            indices[indptr[r]:indptr[r + 1]] = np.sort(rng.choice(C, int(deg[r]), replace=False))
    values = rng.standard_normal(len(indices)).astype(np.float32)
    k = int(rng.choice(KS))
    h = int(rng.integers(k, 257)) if rng.random() < 0.7 else 256
    panel_cost = int(rng.choice([8, 64, 300, 4096]))
    row_cost = int(rng.choice([1, 4, 16]))
    return rng, V, C, indptr.astype(np.int32), indices, values, k, h, panel_cost, row_cost


@pytest.mark.parametrize("seed", range(128))
def test_fuzz_parity(dev, oracle, seed):
    rng, V, C, indptr, indices, values, k, h, pc, rc = draw(seed)
    x = rng.standard_normal((C, h)).astype(np.float32)
    grad = rng.standard_normal((V, h)).astype(np.float32)
    g = S.MaxKGraph(T(indptr, dev), T(indices, dev), T(values, dev), num_cols=C,
                    panel_cost=pc, row_cost=rc)
    ctx = f"V={V} C={C} E={len(indices)} k={k} h={h} panel_cost={pc} row_cost={rc}"

    # CBSR producer: exact top-k sets (continuous inputs, no ties)
    data, sel = S.topk_cbsr(T(x, dev), k)
    sel_np, data_np = sel.cpu().numpy(), data.cpu().numpy()
    ref_idx = np.argsort(-x, axis=1, kind="stable")[:, :k]
    assert np.array_equal(np.sort(sel_np.astype(np.int64), 1), np.sort(ref_idx, 1)), ctx
    assert np.array_equal(data_np, np.take_along_axis(x, sel_np.astype(np.int64), 1)), ctx

    # forward SpGEMM (stale output must not leak)
    out = torch.full((V, h), float("nan"), device=dev)
    y = g.forward(data, sel, h, out=out)
    ref = oracle.np_forward(indptr, indices, values, data_np, sel_np, h)
    assert oracle.parity_error(y.cpu().numpy(), ref) <= TOL, ctx

    # backward SSpMM, every algorithm that supports the shape
    ref_b = oracle.np_backward(indptr, indices, values, grad, sel_np)
    algos = [_lib.MAXK_BWD_ATOMIC, _lib.MAXK_BWD_STAGED]
    if g.local_plan(k) is not None:
        algos.append(_lib.MAXK_BWD_LOCAL)
    for a in algos:
        dx = torch.full((C, k), float("nan"), device=dev)
        g.backward(T(grad, dev), sel, out=dx, algo=a)
        assert oracle.parity_error(dx.cpu().numpy(), ref_b) <= TOL, f"{ctx} algo={a}"

    # dense SpMM baseline
    if h % 4 == 0:
        yd = g.spmm_dense(T(x, dev))
        assert oracle.parity_error(yd.cpu().numpy(),
                                   oracle.np_spmm_dense(indptr, indices, values, x)) <= TOL, ctx

    # multi-relation forward / backward (R relations sharing CSR and CBSR)
    if k >= 4 and k & (k - 1) == 0 and len(indices) > 0:
        R = int(rng.integers(1, 17))
        vals = rng.standard_normal((len(indices), R)).astype(np.float32)
        ym = g.forward_multi(data, sel, T(vals, dev), h).cpu().numpy()
        gm = rng.standard_normal((R, V, h)).astype(np.float32)
        dxm = g.backward_multi(T(gm, dev), sel, T(vals, dev)).cpu().numpy()
        ref_m = np.zeros((C, k))
        for q in range(R):
            refq = oracle.np_forward(indptr, indices, vals[:, q], data_np, sel_np, h)
            assert oracle.parity_error(ym[q], refq) <= TOL, f"{ctx} R={R} q={q}"
            ref_m += oracle.np_backward(indptr, indices, vals[:, q], gm[q], sel_np)
        assert oracle.parity_error(dxm, ref_m) <= TOL, f"{ctx} R={R}"

    # halo-record forward (multi-GPU path), accumulating onto a random base
    if k >= 4 and k & (k - 1) == 0 and C > 0:
        rec = S.cbsr_gather_records(data, sel)
        base = rng.standard_normal((V, h)).astype(np.float32)
        yr = g.forward_records(rec, k, h, out=T(base, dev), accumulate=True)
        assert oracle.parity_error(yr.cpu().numpy(), ref + base) <= TOL, f"{ctx} records"

    # relation-interleaved multi-relation backward (R = 8, k = 32)
    if k == 32 and len(indices) > 0 and g.local_plan(32) is not None:
        vals8 = rng.standard_normal((len(indices), 8)).astype(np.float32)
        g8 = rng.standard_normal((8, V, h)).astype(np.float32)
        dx8 = torch.full((C, k), float("nan"), device=dev)
        g.backward_multi(T(g8, dev), sel, T(vals8, dev), out=dx8, algo=_lib.MAXK_BWD_LOCAL)
        ref8 = sum(oracle.np_backward(indptr, indices, vals8[:, q], g8[q], sel_np) for q in range(8))
        assert oracle.parity_error(dx8.cpu().numpy(), ref8) <= TOL, f"{ctx} rel8"


@pytest.mark.parametrize("seed", range(128, 224))
def test_fuzz_parity_fast_paths(dev, oracle, seed):
    """The same random problems through the forms the sweep above leaves to
    AUTO: the forward that also writes the edge selectors and the two
    backwards that read them (STAGED_EDGE, EDGE_GATHER; and APPEND on node and
    edge selectors, round 6), the column-blocked
    forward (random block count), and TILE (k = 32 / 64, h = 256) with a
    random number of source ranges per destination group; and the fused
    multi-relation forward with the fused multi-relation backwards (R = 4, 8, 16),
    MULTI_APPEND included."""
    from spgemm_new_amd import ops
    rng, V, C, indptr, indices, values, k, h, pc, rc = draw(seed)
    if rng.random() < 0.5 and k not in (32, 64):
        k = int(rng.choice([32, 64]))          # TILE / blocked shapes more often
        h = 256 if rng.random() < 0.7 else max(h, k)
    h = max(h, k)
    x = rng.standard_normal((C, h)).astype(np.float32)
    grad = rng.standard_normal((V, h)).astype(np.float32)
    splits = int(rng.integers(1, 5))
    g = S.MaxKGraph(T(indptr, dev), T(indices, dev), T(values, dev), num_cols=C,
                    panel_cost=pc, row_cost=rc, tile_splits=splits)
    ctx = f"V={V} C={C} E={len(indices)} k={k} h={h} panel_cost={pc} row_cost={rc} splits={splits}"
    data, sel = S.topk_cbsr(T(x, dev), k)
    sel_np, data_np = sel.cpu().numpy(), data.cpu().numpy()
    ref = oracle.np_forward(indptr, indices, values, data_np, sel_np, h)
    ref_b = oracle.np_backward(indptr, indices, values, grad, sel_np)
    G = T(grad, dev)

    # forward writing the edge selectors, then the backwards that read them
    out = torch.full((V, h), float("nan"), device=dev)
    y = ops.spgemm_forward(g, data, sel, h, out=out, edge_sel=True)
    assert oracle.parity_error(y.cpu().numpy(), ref) <= TOL, f"{ctx} esel forward"
    algos = [_lib.MAXK_BWD_STAGED_EDGE]
    if ops._edge_gather_ok(k):
        # round 6: the write-combined APPEND backward, both selector forms
        algos += [_lib.MAXK_BWD_EDGE_GATHER, _lib.MAXK_BWD_APPEND, _lib.MAXK_BWD_APPEND_EDGE]
    for a in algos:
        dx = torch.full((C, k), float("nan"), device=dev)
        g.backward(G, sel, out=dx, algo=a)
        assert oracle.parity_error(dx.cpu().numpy(), ref_b) <= TOL, f"{ctx} algo={a}"

    # column-blocked forward (the restacked CSR, partial outputs, fused last block)
    if len(indices) > 0:
        nb = int(rng.integers(1, 9))
        out = torch.full((V, h), float("nan"), device=dev)
        ops._forward_blocked(g, nb, data, sel, h, out, g.values)
        assert oracle.parity_error(out.cpu().numpy(), ref) <= TOL, f"{ctx} blocked nb={nb}"

    # TILE (its plan may decline a shape: the other algorithms serve it)
    if k in (32, 64) and h == 256 and len(indices) > 0 and g.tile_plan(k) is not None:
        dx = torch.full((C, k), float("nan"), device=dev)
        g.backward(G, sel, out=dx, algo=_lib.MAXK_BWD_TILE)
        assert oracle.parity_error(dx.cpu().numpy(), ref_b) <= TOL, f"{ctx} TILE"

    # fused multi-relation forward and both fused multi-relation backwards
    if k in (8, 16, 32, 64) and len(indices) > 0 and h % 4 == 0:
        R = int(rng.choice([4, 8, 16]))
        vals = rng.standard_normal((len(indices), R)).astype(np.float32)
        gm = rng.standard_normal((R, V, h)).astype(np.float32)
        ym = g.forward_multi(data, sel, T(vals, dev), h).cpu().numpy()
        ref_m = np.zeros((C, k))
        for q in range(R):
            refq = oracle.np_forward(indptr, indices, vals[:, q], data_np, sel_np, h)
            assert oracle.parity_error(ym[q], refq) <= TOL, f"{ctx} R={R} q={q}"
            ref_m += oracle.np_backward(indptr, indices, vals[:, q], gm[q], sel_np)
        for a in (_lib.MAXK_BWD_MULTI_STAGED, _lib.MAXK_BWD_MULTI_EDGE_GATHER,
                  _lib.MAXK_BWD_MULTI_APPEND):
            dxm = torch.full((C, k), float("nan"), device=dev)
            g.backward_multi(T(gm, dev), sel, T(vals, dev), out=dxm, algo=a)
            assert oracle.parity_error(dxm.cpu().numpy(), ref_m) <= TOL, f"{ctx} R={R} algo={a}"
