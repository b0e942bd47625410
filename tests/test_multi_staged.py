"""Multi-relation STAGED backward (maxk_sspmm_backward_multi; config 5's
backward): dXs = sum_q (A_q^T G_q) sampled at sel, the relations summed per edge
inside phase 1.  Checked against the fp64 oracle (the sum of R single-relation
backward calls, oracle/oracle.py np_backward, which restates
kernels/spmm_maxk_backward.cu:15-115), tolerance 1e-4 per element."""
import numpy as np
import pytest
import torch

import spgemm_new_amd as S
from spgemm_new_amd import _lib
from spgemm_new_amd.graphs import random_cbsr, small_csr

pytestmark = pytest.mark.gpu
TOL = 1e-4
MULTI = (_lib.MAXK_BWD_MULTI_STAGED, _lib.MAXK_BWD_MULTI_EDGE_GATHER)
NAME = {_lib.MAXK_BWD_MULTI_STAGED: "multi_staged",
        _lib.MAXK_BWD_MULTI_EDGE_GATHER: "multi_edge_gather"}


def T(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def ref_multi(indptr, indices, vals, grad, sel):
    """sum_q A_q^T G_q at the selected columns, fp64; selectors >= h give 0 (the
    rule of every backward algorithm)."""
    indptr = np.asarray(indptr, np.int64)
    rows = np.repeat(np.arange(len(indptr) - 1), np.diff(indptr))
    cols = np.asarray(indices, np.int64)
    R, _, h = grad.shape
    agt = np.zeros((sel.shape[0], h + 1), np.float64)
    for q in range(R):
        np.add.at(agt[:, :h], cols, vals[:, q].astype(np.float64)[:, None] *
                  grad[q].astype(np.float64)[rows])
    s = np.minimum(sel.astype(np.int64), h)          # column h is the zero column
    return np.take_along_axis(agt, s, axis=1)


@pytest.mark.parametrize("algo", MULTI)
@pytest.mark.parametrize("R,k,h", [(8, 32, 256), (8, 8, 256), (8, 16, 256), (8, 64, 256),
                                   (4, 32, 256), (16, 32, 256), (8, 32, 64), (8, 16, 100),
                                   (4, 8, 12)])
def test_multi_staged_vs_oracle(dev, algo, R, k, h):
    indptr, indices = small_csr(900, seed=R + k + h)
    v, e = len(indptr) - 1, len(indices)
    vals = np.random.default_rng(9).random((e, R), dtype=np.float32)
    _, sel = random_cbsr(v, k, h, seed=6)
    grad = np.random.default_rng(10).random((R, v, h), dtype=np.float32)
    g = S.MaxKGraph(T(indptr, dev), T(indices, dev), panel_cost=300)
    out = torch.full((v, k), float("nan"), device=dev)       # every element is written
    dx = g.backward_multi(T(grad, dev), T(sel, dev), T(vals, dev), out=out, algo=algo)
    assert g.last_bwd_algo == NAME[algo]
    ref = ref_multi(indptr, indices, vals, grad, sel)
    from oracle import oracle as O
    assert O.parity_error(dx.cpu().numpy(), ref) <= TOL


@pytest.mark.parametrize("algo", MULTI)
def test_multi_staged_matches_composed_and_rel8(dev, algo):
    """Same result as R composed single-relation calls and as LOCAL rel8 (up to fp32
    order), run-to-run bitwise identical (no atomics)."""
    indptr, indices = small_csr(1200, seed=4)
    v, e, R, k = len(indptr) - 1, len(indices), 8, 32
    rng = np.random.default_rng(3)
    vals = T(rng.random((e, R), dtype=np.float32), dev)
    _, sel = random_cbsr(v, k, 256, seed=2)
    sel = T(sel, dev)
    grad = T(rng.random((R, v, 256), dtype=np.float32), dev)
    g = S.MaxKGraph(T(indptr, dev), T(indices, dev), panel_cost=256)
    a = g.backward_multi(grad, sel, vals, algo=algo).clone()
    b = g.backward_multi(grad, sel, vals, algo=algo).clone()
    assert torch.equal(a, b)
    comp = g.backward_multi(grad, sel, vals, algo=_lib.MAXK_BWD_STAGED)
    rel8 = g.backward_multi(grad, sel, vals, algo=_lib.MAXK_BWD_LOCAL)
    for other in (comp, rel8):
        err = ((a - other).abs() / other.abs().clamp_min(1)).max().item()
        assert err <= TOL


def test_multi_staged_edge_cases(dev):
    """Rectangular block (halo columns without rows), empty rows and columns, a hub
    row spanning many panels, out-of-range selectors (h = 64, selector bytes up to
    255 read as 0), and an empty edge list."""
    rng = np.random.default_rng(11)
    rows, cols, R, k, h = 300, 700, 8, 16, 64
    deg = rng.integers(0, 12, size=rows)
    deg[5] = 3000                       # hub: spans many panels of 256
    deg[6:20] = 0
    indptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    indices = np.concatenate([np.sort(rng.choice(cols, size=d, replace=d > cols))
                              for d in deg]).astype(np.int32)
    e = len(indices)
    vals = rng.random((e, R), dtype=np.float32)
    sel = np.stack([rng.choice(256, size=k, replace=False) for _ in range(cols)]).astype(np.uint8)
    grad = rng.random((R, rows, h), dtype=np.float32)
    g = S.MaxKGraph(T(indptr, dev), T(indices, dev), num_cols=cols, panel_cost=256)
    ref = ref_multi(indptr, indices, vals, grad, sel)
    from oracle import oracle as O
    for algo in MULTI:
        dx = g.backward_multi(T(grad, dev), T(sel, dev), T(vals, dev), algo=algo)
        assert O.parity_error(dx.cpu().numpy(), ref) <= TOL, algo
    # empty edge list: dXs = 0
    g0 = S.MaxKGraph(T(np.zeros(rows + 1, np.int32), dev), T(np.zeros(0, np.int32), dev),
                     num_cols=cols)
    out = torch.full((cols, k), float("nan"), device=dev)
    dx = g0.backward_multi(T(grad, dev), T(sel, dev), torch.zeros((0, R), device=dev), out=out)
    assert torch.count_nonzero(dx).item() == 0


def test_multi_auto_picks_fused(dev):
    """AUTO (measure) times the fused candidates and keeps one; the result is within
    tolerance of the oracle."""
    indptr, indices = small_csr(800, seed=12)
    v, e, R, k = len(indptr) - 1, len(indices), 8, 32
    rng = np.random.default_rng(5)
    vals = rng.random((e, R), dtype=np.float32)
    _, sel = random_cbsr(v, k, 256, seed=9)
    grad = rng.random((R, v, 256), dtype=np.float32)
    g = S.MaxKGraph(T(indptr, dev), T(indices, dev), panel_cost=256)
    dx = g.backward_multi(T(grad, dev), T(sel, dev), T(vals, dev))
    assert g.last_bwd_algo in ("multi_staged", "multi_edge_gather", "local_rel8")
    from oracle import oracle as O
    assert O.parity_error(dx.cpu().numpy(), ref_multi(indptr, indices, vals, grad, sel)) <= TOL


def test_multi_staged_abi_rejects(dev):
    """The C entry refuses shapes it does not serve (R, k, alignment)."""
    L = _lib.load()
    indptr, indices = small_csr(100, seed=1)
    g = S.MaxKGraph(T(indptr, dev), T(indices, dev))
    csc_pos, csc_indptr, csc_sched, CP = g.csc()
    v = g.num_rows
    out = torch.empty((v, 32), device=dev)
    grad = torch.zeros((8, v, 256), device=dev)
    sel = torch.zeros((v, 32), dtype=torch.uint8, device=dev)
    vals = torch.zeros((g.num_edges, 8), device=dev)
    ws = torch.empty(L.maxk_backward_workspace_bytes(_lib.MAXK_BWD_STAGED, g.num_edges, 32, CP),
                     dtype=torch.uint8, device=dev)

    def call(R=8, k=32, h=256, algo=_lib.MAXK_BWD_STAGED, vptr=None):
        return L.maxk_sspmm_backward_multi(
            algo, g.bwd_sched.data_ptr(), g.bwd_num_panels, g.indptr.data_ptr(),
            g.indices.data_ptr(), vptr or vals.data_ptr(), R, grad.data_ptr(), sel.data_ptr(),
            v, v, g.num_edges, h, k, out.data_ptr(), csc_pos.data_ptr(), csc_sched.data_ptr(),
            CP, csc_indptr.data_ptr(), ws.data_ptr(), ws.numel(), None)

    assert call() == _lib.MAXK_OK
    torch.cuda.synchronize()
    assert call(R=6) == _lib.MAXK_E_ARG
    assert call(k=24) == _lib.MAXK_E_DIM
    assert call(h=254) == _lib.MAXK_E_DIM
    assert call(algo=_lib.MAXK_BWD_ATOMIC) == _lib.MAXK_E_ARG
    assert call(vptr=vals.data_ptr() + 4) == _lib.MAXK_E_ARG


def test_multi_auto_misaligned_values_fall_back(dev):
    """AUTO's cached choice is the relation-summing kernel (16-B aligned inputs);
    a later call whose values are a contiguous but misaligned view takes rel8 /
    composed instead of failing, with the same result."""
    indptr, indices = small_csr(600, seed=14)
    v, e, R, k = len(indptr) - 1, len(indices), 8, 32
    rng = np.random.default_rng(6)
    vals = rng.random((e, R), dtype=np.float32)
    _, sel = random_cbsr(v, k, 256, seed=4)
    grad = T(rng.random((R, v, 256), dtype=np.float32), dev)
    g = S.MaxKGraph(T(indptr, dev), T(indices, dev), panel_cost=256)
    a = g.backward_multi(grad, T(sel, dev), T(vals, dev)).clone()
    flat = torch.empty(e * R + 1, device=dev)
    flat[1:] = T(vals, dev).reshape(-1)
    mis = flat[1:].view(e, R)
    assert mis.is_contiguous() and mis.data_ptr() % 16 != 0
    b = g.backward_multi(grad, T(sel, dev), mis)
    assert g.last_bwd_algo not in ("multi_staged", "multi_edge_gather")
    err = ((a - b).abs() / b.abs().clamp_min(1)).max().item()
    assert err <= TOL
