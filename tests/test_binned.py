"""BINNED backward (propagation blocking: products into destination bins, bins
summed in LDS).  Measured slower than STAGED / EDGE_GATHER at every k (DESIGN.md
§5), so it lives in the ablation build (tools/variants_lib, maxk_variants.h).

CPU: the plan restatement (tests/bin_ref.py) keeps its invariants -- every
edge in exactly one slot of its destination's bin, windows of 64 with distinct
destinations, slot order = (XCD, edge) up to the packing -- and its two-phase
emulation equals the oracle's backward (spmm_maxk_backward.cu:15-115 semantics).
GPU: the device plan is bit-identical to the restatement, the kernels
bit-identical to the emulation (same fp32 products, same slot-order sums), and
within 1e-4 of the oracle, node and edge selectors, k in {8, 16, 32}."""
import os
import sys

import numpy as np
import pytest
import torch

from spgemm_new_amd.graphs import random_cbsr, small_csr
from tests import bin_ref

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "tools", "variants_lib"))

TOL = 1e-4
# the GPU tests need the ablation library, built only on request
# (MAXK_BUILD_VARIANTS=1 or __graft_entry__.build_variants()); they skip without it
_VLIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools",
                     "variants_lib", "libmaxk_variants.so")
needs_vlib = pytest.mark.skipif(not os.path.exists(_VLIB),
                                reason="ablation library not built (MAXK_BUILD_VARIANTS=1)")


def _hub_csr(v=600, hub_every=15, seed=3):
    """Every hub_every-th row also points at column 7 (in-degree 40 at v=600)
    plus random edges: the windows must split the hub's in-edges, closing
    windows early (padding)."""
    rng = np.random.default_rng(seed)
    rows = []
    for r in range(v):
        cols = set(rng.choice(v, size=int(rng.integers(0, 12)), replace=False).tolist())
        if r % hub_every == 0:
            cols.add(7)
        rows.append(sorted(cols))
    indptr = np.zeros(v + 1, np.int32)
    indptr[1:] = np.cumsum([len(c) for c in rows])
    return indptr, np.array([c for r in rows for c in r], np.int32)


def _panels(E, step):
    return np.append(np.arange(0, E, step), E)


@pytest.mark.parametrize("graph", ["small", "hub"])
def test_bin_plan_invariants(graph):
    if graph == "small":
        indptr, indices = small_csr(1500, seed=5)
    else:
        indptr, indices = _hub_csr()
    V = len(indptr) - 1
    E = len(indices)
    pos, ptr, dst, slots = bin_ref.build(_panels(E, 97), indices, V)
    assert ptr[0] == 0 and ptr[-1] == slots and np.all(ptr % 64 == 0)
    assert np.all(np.diff(ptr) >= 0)
    assert len(np.unique(pos)) == E                      # one slot per edge
    b = indices // 255
    assert np.all(pos >= ptr[b]) and np.all(pos < ptr[b + 1])
    assert np.array_equal(dst[pos], (indices - b * 255).astype(np.uint8))
    assert np.count_nonzero(dst != 0xFF) == E
    for w0 in range(0, slots, 64):                       # distinct destinations per window
        d = dst[w0:w0 + 64]
        d = d[d != 0xFF]
        assert len(np.unique(d)) == len(d)


@pytest.mark.parametrize("k", [8, 16, 32])
@pytest.mark.parametrize("graph", ["small", "hub"])
def test_bin_emulation_matches_oracle(oracle, k, graph):
    if graph == "small":
        indptr, indices = small_csr(1200, seed=6)
    else:
        indptr, indices = _hub_csr()
    V = len(indptr) - 1
    values = np.random.default_rng(1).random(len(indices), dtype=np.float32)
    _, sel = random_cbsr(V, k, 256, seed=k)
    grad = np.random.default_rng(2).random((V, 256), dtype=np.float32)
    plan = bin_ref.build(_panels(len(indices), 50), indices, V)
    got = bin_ref.backward(indptr, indices, values, grad, sel, V, plan)
    ref = oracle.np_backward(indptr, indices, values, grad, sel)
    assert oracle.parity_error(got, ref) <= TOL


# ----------------------------------------------------------------------- GPU
def T(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _graph(dev, kind, num_cols=None):
    import spgemm_new_amd as S
    if kind == "small":
        indptr, indices = small_csr(3000, seed=21)
    elif kind == "hub":
        indptr, indices = _hub_csr()
    else:   # rectangular block: 700 rows, 1000 columns (a rank with halo columns)
        rng = np.random.default_rng(9)
        deg = rng.integers(0, 40, size=700)
        indptr = np.zeros(701, np.int32)
        indptr[1:] = np.cumsum(deg)
        indices = np.concatenate([np.sort(rng.choice(1000, d, replace=False)) for d in deg]
                                 ).astype(np.int32)
        num_cols = 1000
    values = np.random.default_rng(2).random(len(indices), dtype=np.float32)
    g = S.MaxKGraph(T(indptr, dev), T(indices, dev), T(values, dev), panel_cost=300,
                    num_cols=num_cols)
    return g, indptr, indices, values


@pytest.mark.gpu
@needs_vlib
@pytest.mark.parametrize("kind", ["small", "hub", "rect"])
def test_device_plan_equals_reference(dev, kind):
    import variants as V
    g, indptr, indices, values = _graph(dev, kind)
    plan = V.bin_plan(g)
    assert plan is not None
    starts = g.bwd_sched.view(-1, 2)[:, 1].cpu().numpy()
    pos, ptr, dst, slots = bin_ref.build(starts, indices, g.num_cols)
    assert plan["num_slots"] == slots
    assert np.array_equal(plan["bin_pos"].cpu().numpy(), pos)
    assert np.array_equal(plan["bin_ptr"].cpu().numpy(), ptr)
    assert np.array_equal(plan["bin_dst"].cpu().numpy(), dst)


@pytest.mark.gpu
@needs_vlib
@pytest.mark.parametrize("k", [8, 16, 32])
@pytest.mark.parametrize("kind", ["small", "hub", "rect"])
@pytest.mark.parametrize("h", [256, 100])
def test_binned_backward(dev, oracle, k, kind, h):
    import variants as V
    g, indptr, indices, values = _graph(dev, kind)
    C = g.num_cols
    _, sel = random_cbsr(C, k, h, seed=50 + k)
    grad = np.random.default_rng(k).random((g.num_rows, h), dtype=np.float32)
    plan = V.bin_plan(g)
    starts = g.bwd_sched.view(-1, 2)[:, 1].cpu().numpy()
    ref_plan = bin_ref.build(starts, indices, C)
    emu = bin_ref.backward(indptr, indices, values, grad, sel, C, ref_plan)
    ref = oracle.np_backward(indptr, indices, values, grad, sel) if kind != "rect" else \
        oracle.c_backward_csr(indptr, indices, values, grad, sel)
    G, Sel = T(grad, dev), T(sel, dev)
    for edge in (False, True):
        out = torch.full((C, k), float("nan"), device=dev)
        V.backward_binned(g, G, Sel, plan, edge=edge, out=out)
        got = out.cpu().numpy()
        assert np.array_equal(got, emu), (edge, np.abs(got - emu).max())
        assert oracle.parity_error(got, ref) <= TOL
        again = V.backward_binned(g, G, Sel, plan, edge=edge)
        assert torch.equal(again, out)                 # deterministic
    assert plan["num_slots"] >= g.num_edges


@pytest.mark.gpu
@needs_vlib
def test_binned_values_per_call(dev, oracle):
    """Per-call edge values."""
    import variants as V
    g, indptr, indices, values = _graph(dev, "small")
    k, h = 8, 256
    _, sel = random_cbsr(g.num_cols, k, h, seed=3)
    grad = np.random.default_rng(5).random((g.num_rows, h), dtype=np.float32)
    w = np.random.default_rng(6).random(len(indices), dtype=np.float32)
    out = V.backward_binned(g, T(grad, dev), T(sel, dev), V.bin_plan(g), values=T(w, dev))
    assert oracle.parity_error(out.cpu().numpy(),
                               oracle.np_backward(indptr, indices, w, grad, sel)) <= TOL


@pytest.mark.gpu
@needs_vlib
def test_binned_plan_refused_for_heavy_padding(dev):
    """A destination with a huge in-degree needs a window per in-edge: the plan
    is dropped (too many padding slots) and BINNED raises."""
    import spgemm_new_amd as S
    import variants as V
    v = 4000
    indptr = np.arange(v + 1, dtype=np.int32)            # every row -> column 0
    indices = np.zeros(v, np.int32)
    g = S.MaxKGraph(T(indptr, dev), T(indices, dev))
    assert V.bin_plan(g) is None
    _, sel = random_cbsr(v, 8, 256, seed=1)
    G = torch.rand((v, 256), device=dev)
    with pytest.raises(RuntimeError):
        V.backward_binned(g, G, T(sel, dev), None)
