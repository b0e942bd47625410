"""The ABLATION build (tools/variants_lib/libmaxk_variants.so):
kernels built, tested and measured slower on every BASELINE shape, kept out of
the product library.  Each is checked against the fp64 oracle and bitwise
against the product kernel it was an alternative to:
the register-accumulator R = 8 forward and backward phase 1, the bank-ordered
backward phase 1 and their CBSR preparations.  (BINNED: tests/test_binned.py.)"""
import os
import sys

import numpy as np
import pytest
import torch

import spgemm_new_amd as S
from spgemm_new_amd import _lib
from spgemm_new_amd.graphs import random_cbsr, small_csr

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "tools", "variants_lib"))
import variants as V  # noqa: E402

TOL = 1e-4
# the ablation library is built only on request (MAXK_BUILD_VARIANTS=1 or
# __graft_entry__.build_variants()); without it these tests skip
pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not os.path.exists(V.LIB_PATH),
                                 reason="ablation library not built (MAXK_BUILD_VARIANTS=1)")]


def T(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _edge_graph(kind):
    if kind == "empty_rows":
        return np.zeros(101, np.int32), np.zeros(0, np.int32)
    if kind == "single_row_hub":      # one row adjacent to every node, spans many panels
        v = 5000
        indptr = np.zeros(v + 1, np.int32)
        indptr[1:] = v
        indptr[0] = 0
        indptr[1:] = v
        return indptr, np.arange(v, dtype=np.int32)
    if kind == "one_node":
        return np.array([0, 1], np.int32), np.array([0], np.int32)
    if kind == "last_row_only":
        v = 300
        indptr = np.zeros(v + 1, np.int32)
        indptr[-1] = 70
        return indptr, np.sort(np.random.default_rng(0).choice(v, 70, replace=False)).astype(np.int32)
    raise KeyError(kind)


@pytest.mark.parametrize("k", [4, 8, 16, 32])
@pytest.mark.parametrize("order", ["column", "value"])
def test_cbsr_colmask(dev, k, order):
    """maxk_cbsr_colmask: each row's values in ascending column order and, per
    32-column word, the column bitmask and the count of selected columns below
    it -- whatever the CBSR entry order."""
    v, h = 700, 256
    x = torch.rand((v, h), device=dev)
    data, sel = S.topk_cbsr(x, k, order=order)
    L = V.load()
    sd = torch.empty((v, k), device=dev)
    mr = torch.empty((v, 16), dtype=torch.int32, device=dev)
    _lib.check(L.maxk_cbsr_colmask(data.data_ptr(), sel.data_ptr(), v, k, sd.data_ptr(),
                                   mr.data_ptr(), None), "colmask")
    torch.cuda.synchronize()
    s_np, d_np = sel.cpu().numpy().astype(np.int64), data.cpu().numpy()
    o = np.argsort(s_np, axis=1, kind="stable")
    np.testing.assert_array_equal(sd.cpu().numpy(), np.take_along_axis(d_np, o, 1))
    m = mr.cpu().numpy().view(np.uint32).reshape(v, 8, 2)
    for r in range(0, v, 7):
        cols = set(s_np[r].tolist())
        for w in range(8):
            bits = sum(1 << (c - 32 * w) for c in cols if 32 * w <= c < 32 * w + 32)
            assert m[r, w, 0] == bits and m[r, w, 1] == sum(c < 32 * w for c in cols)


@pytest.mark.parametrize("k", [4, 8, 16, 32])
@pytest.mark.parametrize("panel_cost", [100, 2048])
def test_forward_multi_gather_bitwise(dev, oracle, k, panel_cost):
    """The register-accumulator R = 8 forward (the ablation library) on a graph with hub
    rows split over many panels, empty rows and value-ordered (unsorted) CBSR
    entries equals the fp64 oracle, and gives the same bits as the LDS
    relation-vector kernel at k = 32 (both add every element's contributions in
    edge order; at k < 32 the LDS kernel sums per-edge-slot row copies, another
    fp32 order, so there it agrees to rounding)."""
    indptr, indices = small_csr(1200, seed=31)
    v, e, R = len(indptr) - 1, len(indices), 8
    vals = torch.rand((e, R), device=dev)
    x = torch.rand((v, 256), device=dev)
    data, sel = S.topk_cbsr(x, k, order="value")
    g = S.MaxKGraph(T(indptr, dev), T(indices, dev), panel_cost=panel_cost)
    y_g = V.forward_multi_gather(g, data, sel, vals, 256)
    y_l = g.forward_multi(data, sel, vals, 256)
    if k == 32:
        assert torch.equal(y_g, y_l)
    else:
        assert torch.allclose(y_g, y_l, rtol=1e-6, atol=1e-6)
    dn, sn, vn = data.cpu().numpy(), sel.cpu().numpy(), vals.cpu().numpy()
    for q in (0, 7):
        ref = oracle.np_forward(indptr, indices, vn[:, q].copy(), dn, sn, 256)
        assert oracle.parity_error(y_g[q].cpu().numpy(), ref) <= TOL


def test_forward_multi_gather_edge_cases(dev, oracle):
    """Gather form: empty edge list, a single hub row, the last row only; stale
    NaN outputs are overwritten; unsupported shapes refuse the explicit form."""
    for kind in ("single_row_hub", "empty_rows", "last_row_only"):
        indptr, indices = _edge_graph(kind)
        v, e = len(indptr) - 1, len(indices)
        vals = torch.rand((e, 8), device=dev)
        data, sel = random_cbsr(v, 32, 256, seed=5)
        g = S.MaxKGraph(T(indptr, dev), T(indices, dev), panel_cost=100)
        out = torch.full((8, v, 256), float("nan"), device=dev)
        V.forward_multi_gather(g, T(data, dev), T(sel, dev), vals, 256, out=out)
        for q in (0, 5):
            ref = oracle.np_forward(indptr, indices, vals[:, q].cpu().numpy(), data, sel, 256)
            assert oracle.parity_error(out[q].cpu().numpy(), ref) <= TOL, kind
    indptr, indices = small_csr(50, seed=2)
    g = S.MaxKGraph(T(indptr, dev), T(indices, dev))
    data, sel = random_cbsr(50, 64, 256, seed=1)
    with pytest.raises(RuntimeError, match="gather form"):
        V.forward_multi_gather(g, T(data, dev), T(sel, dev),
                               torch.rand((len(indices), 8), device=dev))


@pytest.mark.parametrize("k", [8, 16, 32])
@pytest.mark.parametrize("algo", [_lib.MAXK_BWD_MULTI_STAGED, _lib.MAXK_BWD_MULTI_EDGE_GATHER])
def test_backward_multi_gather_bitwise(dev, oracle, k, algo):
    """Phase 1 of the multi-relation STAGED backward in register form (R = 8,
    h = 256) writes the same staging rows as the LDS kernel (same FMAs, same
    relation order): dXs bitwise equal, and equal to sum_q of the fp64 oracle."""
    indptr, indices = small_csr(1100, seed=41)
    v, e, R = len(indptr) - 1, len(indices), 8
    vals = torch.rand((e, R), device=dev)
    grad = torch.rand((R, v, 256), device=dev)
    x = torch.rand((v, 256), device=dev)
    _, sel = S.topk_cbsr(x, k, order="value")
    g = S.MaxKGraph(T(indptr, dev), T(indices, dev), panel_cost=300)
    d_g = V.backward_multi_form(g, grad, sel, vals, "gather",
                              algo == _lib.MAXK_BWD_MULTI_EDGE_GATHER)
    d_l = g.backward_multi(grad, sel, vals, algo=algo)
    assert torch.equal(d_g, d_l)
    sn, vn, gn = sel.cpu().numpy(), vals.cpu().numpy(), grad.cpu().numpy()
    ref = sum(oracle.np_backward(indptr, indices, vn[:, q].copy(), gn[q], sn) for q in range(R))
    assert oracle.parity_error(d_g.cpu().numpy(), ref) <= TOL


@pytest.mark.parametrize("h,order", [(256, "value"), (256, "column"), (64, "value"), (36, "value")])
@pytest.mark.parametrize("algo", [_lib.MAXK_BWD_MULTI_STAGED, _lib.MAXK_BWD_MULTI_EDGE_GATHER])
def test_backward_multi_banked_bitwise(dev, oracle, h, order, algo):
    """R = 8, k = 32: phase 1 on bank-ordered selectors (one edge per
    wave-instruction, products stored at the columns' original entries) gives
    the LDS form's bits; h = 36 / 64 crowd the 32 columns into few residues mod 8
    (the bank order's overflow path)."""
    indptr, indices = small_csr(1300, seed=43)
    v, e, R = len(indptr) - 1, len(indices), 8
    vals = torch.rand((e, R), device=dev)
    grad = torch.rand((R, v, h), device=dev)
    x = torch.rand((v, h), device=dev)
    _, sel = S.topk_cbsr(x, 32, order=order)
    g = S.MaxKGraph(T(indptr, dev), T(indices, dev), panel_cost=300)
    d_b = V.backward_multi_form(g, grad, sel, vals, "banked",
                              algo == _lib.MAXK_BWD_MULTI_EDGE_GATHER)
    d_l = g.backward_multi(grad, sel, vals, algo=algo)
    assert torch.equal(d_b, d_l)
    sn, vn, gn = sel.cpu().numpy(), vals.cpu().numpy(), grad.cpu().numpy()
    ref = sum(oracle.np_backward(indptr, indices, vn[:, q].copy(), gn[q], sn) for q in range(R))
    assert oracle.parity_error(d_b.cpu().numpy(), ref) <= TOL


def test_bank_order_packed(dev):
    """maxk_cbsr_bank_order_ex's packed output: low byte = the reordered selector
    (== out_sel), high byte = its original entry; a permutation per row."""
    L = V.load()
    data, sel = random_cbsr(700, 32, 256, seed=5)
    sel[:40, :] = np.arange(0, 256, 8)[None, :]          # one residue only: all overflow
    d, s = T(data, dev), T(sel, dev)
    osel = torch.empty_like(s)
    sp = torch.empty(s.shape, dtype=torch.int16, device=dev)
    _lib.check(L.maxk_cbsr_bank_order_ex(d.data_ptr(), s.data_ptr(), 700, 32, 8, None,
                                         osel.data_ptr(), sp.data_ptr(), None), "bank_order_ex")
    torch.cuda.synchronize()
    p = sp.cpu().numpy().astype(np.int64) & 0xFFFF
    assert np.array_equal((p & 0xFF).astype(np.uint8), osel.cpu().numpy())
    orig = p >> 8
    assert (np.sort(orig, axis=1) == np.arange(32)[None, :]).all()
    assert np.array_equal(np.take_along_axis(sel, orig, axis=1), osel.cpu().numpy())
    assert L.maxk_cbsr_bank_order_ex(None, s.data_ptr(), 700, 32, 8, None, None, None,
                                     None) == _lib.MAXK_E_ARG
