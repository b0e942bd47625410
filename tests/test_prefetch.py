"""The edge-stream prefetch forms (maxk_spgemm.hip FWD_PF / BWD_PF): the
column-blocked forward (cacheable gathers) and the node-selector STAGED push at
k <= 16, h = 256, load the next batch's edges -- across row boundaries, up to
the panel's end -- and the push also the next row's gradient row, while the
current batch's gathers run.  Their edge cases are the panel shapes: a panel
that starts inside a row (split first row), one that ends inside a row (the
carry), rows of 0, 1, 63, 64, 65 and hundreds of edges, and panels of a few
edges.  Each case is checked against the fp64 oracle (1e-4, as test_gpu_parity);
the forward also against the plain forward of the same graph."""
import numpy as np
import pytest
import torch

import spgemm_new_amd as S
from spgemm_new_amd import _lib, ops
from spgemm_new_amd.graphs import random_cbsr

pytestmark = pytest.mark.gpu
TOL = 1e-4


def T(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _graph(V, C, seed):
    """Row lengths around the 64-edge batch: 0, 1, 63, 64, 65, 127, 128, 129 and
    long rows, in a shuffled order, plus a Poisson bulk."""
    rng = np.random.default_rng(seed)
    special = [0, 1, 63, 64, 65, 127, 128, 129, 0, 700, 2, 0, 1000]
    d = rng.poisson(40, V)
    d[rng.choice(V, len(special), replace=False)] = special
    d = np.minimum(d, C)
    indptr = np.zeros(V + 1, np.int64)
    indptr[1:] = np.cumsum(d)
    idx = np.concatenate([np.sort(rng.choice(C, size=x, replace=False)) for x in d])
    vals = rng.uniform(-1, 1, idx.size).astype(np.float32)
    return indptr.astype(np.int32), idx.astype(np.int32), vals


@pytest.mark.parametrize("panel_cost", [8, 64, 300, 4096])
@pytest.mark.parametrize("k", [4, 8, 16])
def test_staged_push_prefetch(dev, oracle, k, panel_cost):
    V = C = 1500
    indptr, idx, vals = _graph(V, C, seed=k * 7 + panel_cost)
    g = S.MaxKGraph(T(indptr, dev), T(idx, dev), T(vals, dev), panel_cost=panel_cost)
    data, sel = random_cbsr(V, k, 256, seed=k)
    sel_t, grad = T(sel, dev), np.random.default_rng(k).standard_normal((V, 256)).astype(np.float32)
    dx = torch.full((C, k), float("nan"), device=dev)
    g.backward(T(grad, dev), sel_t, out=dx, algo=_lib.MAXK_BWD_STAGED)
    ref = oracle.np_backward(indptr, idx, vals, grad, sel)
    assert oracle.parity_error(dx.cpu().numpy(), ref) <= TOL
    # the same sums as the edge-selector form, which has no prefetch (bitwise: one
    # staging row per edge at the same place, one segmented sum in the same order)
    y = torch.empty((V, 256), device=dev)
    g.forward(T(data, dev), sel_t, 256, out=y, edge_sel=True)
    dxe = torch.full((C, k), float("nan"), device=dev)
    g.backward(T(grad, dev), sel_t, out=dxe, algo=_lib.MAXK_BWD_STAGED_EDGE)
    assert torch.equal(dx, dxe)


@pytest.mark.parametrize("panel_cost", [8, 64, 300, 2048])
@pytest.mark.parametrize("k", [32, 64])
def test_blocked_forward_prefetch(dev, oracle, k, panel_cost):
    V = C = 1500
    indptr, idx, vals = _graph(V, C, seed=k + panel_cost)
    g = S.MaxKGraph(T(indptr, dev), T(idx, dev), T(vals, dev), panel_cost=panel_cost)
    data, sel = random_cbsr(V, k, 256, seed=k)
    ref = oracle.np_forward(indptr, idx, vals, data, sel, 256)
    for nb in (1, 3):
        out = torch.full((V, 256), float("nan"), device=dev)
        ops._forward_blocked(g, nb, T(data, dev), T(sel, dev), 256, out, g.values)
        assert oracle.parity_error(out.cpu().numpy(), ref) <= TOL, nb
