"""The APPEND backward (MAXK_BWD_APPEND / APPEND_EDGE / MULTI_APPEND; round 6,
VERDICT r5 items 3 and 4): write-combined propagation blocking.  Phase 1 appends
every edge's k products (and its destination) to the region of (destination
bin, XCD group) through an atomic cursor; phase 2 sums each bin in LDS.  The
order of a destination's sum follows arrival order, so the result is checked
per element against the fp64 oracle (1e-4, the north-star tolerance), not
bitwise; the plan's region table is checked exactly against a numpy
restatement of its definition.  Full size: tests/test_full_size.py (products
k = 8 ... 64 and Reddit vs rocSPARSE)."""
import numpy as np
import pytest
import torch

import spgemm_new_amd as S
from spgemm_new_amd import _lib
from spgemm_new_amd.graphs import random_cbsr, small_csr

TOL = 1e-4


def T(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _bins(num_cols, k):
    import ctypes
    L = _lib.load()
    nb, bs = ctypes.c_int(0), ctypes.c_int(0)
    _lib.check(L.maxk_append_bins(num_cols, k, ctypes.byref(nb), ctypes.byref(bs)), "bins")
    return nb.value, bs.value


def test_bins_rule():
    """(CPU: a host function of the library.)  Bins cover the columns, each
    bin's k-vectors fit 160 KB of LDS, whole rounds of 256 bins when there are
    more than 256."""
    for C in (1, 5, 64, 1000, 20_000, 232_965, 2_449_029):
        for k in (4, 8, 16, 32, 64, 128, 256):
            nb, bs = _bins(C, k)
            assert nb * bs >= C and (nb - 1) * bs < C, (C, k, nb, bs)
            assert bs * k * 4 <= 160 * 1024, (C, k, bs)
    nb, bs = _bins(2_449_029, 8)
    assert nb == 512 and bs == 4784       # products k = 8: two rounds of 256 workgroups


def _plan_ref(g, k, nb, bs):
    """region_base restated: edges counted per (bin of the destination, XCD group
    = (panel // 4) % 8) in panel order, exclusive prefix sum."""
    sched = g.bwd_sched.view(-1, 2).cpu().numpy()
    idx = g.indices[: g.num_edges].cpu().numpy().astype(np.int64)
    counts = np.zeros(nb * 8, np.int64)
    for w in range(g.bwd_num_panels):
        j0, j1 = sched[w, 1], sched[w + 1, 1]
        grp = (w // 4) % 8
        np.add.at(counts, (idx[j0:j1] // bs) * 8 + grp, 1)
    return np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)


@pytest.mark.gpu
@pytest.mark.parametrize("k", [8, 32])
def test_plan_equals_restatement(dev, k):
    indptr, indices = small_csr(2500, seed=4)
    g = S.MaxKGraph(T(indptr, dev), T(indices, dev), panel_cost=64)
    plan = g.append_plan(k)
    nb, bs = plan["num_bins"], plan["bin_size"]
    assert (nb, bs) == _bins(g.num_cols, k)
    got = plan["region_base"].cpu().numpy().astype(np.int64)
    assert np.array_equal(got, _plan_ref(g, k, nb, bs))
    assert got[-1] == len(indices)


_CASES = [(k, h, kind) for k in (4, 8, 16, 32, 64, 128, 256) for h, kind in
          ((256, "square"), (256, "rect"))] + [(8, 64, "square"), (16, 100, "rect"),
                                               (32, 256, "hub"), (8, 256, "hub"),
                                               (16, 256, "empty_rows")]


def _graph(kind, seed):
    rng = np.random.default_rng(seed)
    if kind == "square":
        indptr, indices = small_csr(1800, seed=seed)
        return indptr, indices, len(indptr) - 1
    if kind == "rect":      # a rank's block: fewer rows than columns
        indptr, indices = small_csr(700, seed=seed)
        C = 2300
        return indptr, (indices.astype(np.int64) * 3 % C).astype(np.int32), C
    if kind == "hub":       # one destination with thousands of in-edges (spans many chunks)
        indptr, indices = small_csr(1500, seed=seed)
        indices = indices.copy()
        indices[rng.random(len(indices)) < 0.4] = 7
        return indptr, indices, len(indptr) - 1
    if kind == "empty_rows":
        indptr = np.zeros(401, np.int32)
        indptr[200:] = 5
        indices = np.array([3, 9, 3, 0, 399], np.int32)
        return indptr, indices, 400
    raise ValueError(kind)


@pytest.mark.parametrize("k,h,kind", [c for c in _CASES if c[0] <= c[1]],
                         ids=[f"k{k}-h{h}-{kind}" for k, h, kind in _CASES if k <= h])
@pytest.mark.gpu
def test_append_matches_oracle(dev, oracle, k, h, kind):
    indptr, indices, C = _graph(kind, seed=10 + k)
    rng = np.random.default_rng(k + h)
    values = rng.standard_normal(len(indices)).astype(np.float32)
    g = S.MaxKGraph(T(indptr, dev), T(indices, dev), T(values, dev), num_cols=C, panel_cost=128)
    data, sel = random_cbsr(C, k, h, seed=k)
    grad = rng.standard_normal((len(indptr) - 1, h)).astype(np.float32)
    ref = oracle.np_backward(indptr, indices, values, grad, sel)
    sel_t, grad_t = T(sel, dev), T(grad, dev)
    for algo in (_lib.MAXK_BWD_APPEND, _lib.MAXK_BWD_APPEND_EDGE):
        if algo == _lib.MAXK_BWD_APPEND_EDGE:
            # the edge selectors come from a forward of this selector tensor
            g.forward(T(data, dev), sel_t, h, edge_sel=True)
        out = torch.full((C, k), float("nan"), device=dev)   # stale NaN: every row written
        g.backward(grad_t, sel_t, out=out, algo=algo)
        assert g.last_bwd_algo == ("append" if algo == _lib.MAXK_BWD_APPEND else "append_edge")
        assert oracle.parity_error(out.cpu().numpy(), ref) <= TOL, algo


@pytest.mark.gpu
def test_append_values_per_call(dev, oracle):
    """Per-call values (the plan depends on the graph's structure only)."""
    indptr, indices = small_csr(1200, seed=3)
    g = S.MaxKGraph(T(indptr, dev), T(indices, dev), panel_cost=256)
    rng = np.random.default_rng(5)
    data, sel = random_cbsr(1200, 16, 256, seed=1)
    grad = rng.standard_normal((1200, 256)).astype(np.float32)
    for _ in range(2):
        vals = rng.standard_normal(len(indices)).astype(np.float32)
        dx = S.sspmm_backward(g, T(grad, dev), T(sel, dev), values=T(vals, dev),
                              algo=_lib.MAXK_BWD_APPEND)
        ref = oracle.np_backward(indptr, indices, vals, grad, sel)
        assert oracle.parity_error(dx.cpu().numpy(), ref) <= TOL


@pytest.mark.gpu
def test_append_selectors_out_of_range(dev, oracle):
    """Selectors >= h read a zero gradient column, as in every algorithm."""
    indptr, indices = small_csr(900, seed=8)
    g = S.MaxKGraph(T(indptr, dev), T(indices, dev), panel_cost=128)
    rng = np.random.default_rng(2)
    h, k = 64, 8
    sel = rng.integers(0, 256, size=(900, k)).astype(np.uint8)
    grad = rng.standard_normal((900, h)).astype(np.float32)
    dx = g.backward(T(grad, dev), T(sel, dev), algo=_lib.MAXK_BWD_APPEND)
    gpad = np.zeros((900, 256), np.float32)
    gpad[:, :h] = grad
    ref = oracle.np_backward(indptr, indices, np.ones(len(indices), np.float32), gpad, sel)
    assert oracle.parity_error(dx.cpu().numpy(), ref) <= TOL


@pytest.mark.gpu
@pytest.mark.parametrize("R,k", [(4, 8), (8, 32), (16, 16), (8, 64)])
def test_multi_append_matches_oracle(dev, oracle, R, k):
    """The multi-relation APPEND (relations summed per edge in phase 1): equals
    sum_q (A_q^T G_q) gathered at sel."""
    indptr, indices = small_csr(1300, seed=R + k)
    v, h = len(indptr) - 1, 256
    rng = np.random.default_rng(R * k)
    values = rng.standard_normal((len(indices), R)).astype(np.float32)
    grad = rng.standard_normal((R, v, h)).astype(np.float32)
    _, sel = random_cbsr(v, k, h, seed=3)
    g = S.MaxKGraph(T(indptr, dev), T(indices, dev), T(np.ascontiguousarray(values[:, 0]), dev),
                    panel_cost=128)
    dx = g.backward_multi(T(grad, dev), T(sel, dev), T(values, dev), algo=_lib.MAXK_BWD_MULTI_APPEND)
    assert g.last_bwd_algo == "multi_append"
    ref = sum(oracle.np_backward(indptr, indices, np.ascontiguousarray(values[:, q]), grad[q], sel)
              for q in range(R))
    assert oracle.parity_error(dx.cpu().numpy(), ref) <= TOL


@pytest.mark.gpu
def test_append_degenerate(dev, oracle):
    """No edges / no rows: dXs = 0 (every element written); one edge."""
    for indptr, indices, C in ((np.zeros(11, np.int32), np.zeros(0, np.int32), 10),
                               (np.array([0, 1], np.int32), np.array([5], np.int32), 9)):
        g = S.MaxKGraph(T(indptr, dev), T(indices, dev), num_cols=C)
        sel = np.tile(np.arange(8, dtype=np.uint8), (C, 1))
        grad = np.ones((len(indptr) - 1, 256), np.float32)
        out = torch.full((C, 8), float("nan"), device=dev)
        g.backward(T(grad, dev), T(sel, dev), out=out, algo=_lib.MAXK_BWD_APPEND)
        ref = oracle.np_backward(indptr, indices, np.ones(len(indices), np.float32), grad, sel)
        assert oracle.parity_error(out.cpu().numpy(), ref) == 0.0
