"""Golden vectors produced by the reference's own Python code
(tests/golden/make_golden.py: reference MaxK autograd + its CPU aggregation op).

CPU: the oracle reproduces them (pins the oracle).  GPU: the HIP path (top-k
CBSR producer + SpGEMM + SSpMM + autograd scatter) reproduces them: top-k index
sets bit-exact, fp32 values within 1e-4 (per element, relative to max(1,|ref|))."""
import os

import numpy as np
import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KS = (8, 16, 32, 64)
TOL = 1e-4


def load(k):
    inp = np.load(os.path.join(HERE, "inputs.npz"))
    g = np.load(os.path.join(HERE, f"kernel_k{k}.npz"))
    h = inp["x"].shape[1]
    mask = np.unpackbits(g["mask_bits"], axis=1)[:, :h].astype(bool)
    return inp, g, mask


def cbsr_from_mask(x, mask, k):
    sel = np.nonzero(mask)[1].reshape(x.shape[0], k).astype(np.uint8)
    data = np.take_along_axis(x, sel.astype(np.int64), axis=1).astype(np.float32)
    return data, sel


@pytest.mark.parametrize("k", KS)
def test_oracle_reproduces_reference(oracle, k):
    inp, g, mask = load(k)
    x, G = inp["x"], inp["G"]
    assert np.all(mask.sum(1) == k)
    # top-k index sets: oracle's CBSR producer == reference MaxK, bit-exact
    _, sel_o = oracle.np_cbsr(x, k)
    m_o = np.zeros_like(mask)
    np.put_along_axis(m_o, sel_o.astype(np.int64), True, axis=1)
    assert np.array_equal(m_o, mask)
    data, sel = cbsr_from_mask(x, mask, k)
    h = x.shape[1]
    y = oracle.np_forward(inp["indptr"], inp["indices"], inp["values"], data, sel, h)
    assert oracle.parity_error(y, g["Y"]) <= 1e-5
    w4 = oracle.c_warp4(inp["indptr"])
    yc = oracle.c_forward(w4, inp["indices"], inp["values"], data, sel, h)
    assert oracle.parity_error(yc, g["Y"]) <= TOL
    dxs = oracle.np_backward(inp["indptr"], inp["indices"], inp["values"], G, sel)
    dense = np.zeros_like(x, dtype=np.float64)
    np.put_along_axis(dense, sel.astype(np.int64), dxs, axis=1)
    assert oracle.parity_error(dense, g["grad_x"]) <= 1e-5
    dc = oracle.c_backward(w4, inp["indices"], inp["values"], G, sel)
    dense = np.zeros_like(x, dtype=np.float64)
    np.put_along_axis(dense, sel.astype(np.int64), dc, axis=1)
    assert oracle.parity_error(dense, g["grad_x"]) <= TOL


@pytest.mark.gpu
@pytest.mark.parametrize("k", KS)
def test_hip_reproduces_reference(dev, k):
    import torch

    from spgemm_new_amd import _lib
    from spgemm_new_amd.models import SpGEMMFunction, cbsr_topk
    import spgemm_new_amd as S
    inp, g, mask = load(k)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    x = t(inp["x"]).requires_grad_(True)
    gd = (t(inp["indptr"]), t(inp["indices"]), t(inp["values"]))
    # CBSR producer: index sets bit-exact vs the reference MaxK
    _, sel = cbsr_topk(x.detach(), k)
    m = torch.zeros_like(x, dtype=torch.bool)
    m.scatter_(1, sel.long(), True)
    assert torch.equal(m.cpu(), torch.from_numpy(mask))
    y = SpGEMMFunction.apply(x, gd, k)
    y.backward(t(inp["G"]))
    ey = np.max(np.abs(y.detach().cpu().numpy() - g["Y"]) / np.maximum(1, np.abs(g["Y"])))
    eg = np.max(np.abs(x.grad.cpu().numpy() - g["grad_x"]) / np.maximum(1, np.abs(g["grad_x"])))
    assert ey <= TOL and eg <= TOL, (ey, eg)
    # every backward algorithm agrees with the reference gradient
    graph = S.MaxKGraph(*gd)
    for algo in (_lib.MAXK_BWD_ATOMIC, _lib.MAXK_BWD_STAGED, _lib.MAXK_BWD_LOCAL):
        dxs = graph.backward(t(inp["G"]), sel, algo=algo)
        dense = torch.zeros_like(x).scatter_(1, sel.long(), dxs).cpu().numpy()
        e = np.max(np.abs(dense - g["grad_x"]) / np.maximum(1, np.abs(g["grad_x"])))
        assert e <= TOL, (algo, e)


# ---- SURVEY.md §8(c) shape: V=2048, h=256, k in {32, 64} (the TILE backward's
# shapes and the north-star config), from the same reference code
KS256 = (32, 64)


def load256(k):
    inp = np.load(os.path.join(HERE, "inputs_h256.npz"))
    g = np.load(os.path.join(HERE, f"kernel_h256_k{k}.npz"))
    h = inp["x"].shape[1]
    mask = np.unpackbits(g["mask_bits"], axis=1)[:, :h].astype(bool)
    grad_x = np.zeros(inp["x"].shape, np.float32)
    grad_x[mask] = g["grad_sel"].reshape(-1)
    return inp, g, mask, grad_x


def test_h256_fixture_shape():
    """The fixture covers what §8(c) asks for: V in 2-4 K, h = 256, degrees
    0/1/63/64/65/>200, at least 13 blocks of 12 warp4 chunks."""
    inp = np.load(os.path.join(HERE, "inputs_h256.npz"))
    deg = np.diff(inp["indptr"])
    assert 2000 <= len(deg) <= 4096 and inp["x"].shape[1] == 256
    for d in (0, 1, 63, 64, 65):
        assert (deg == d).any(), d
    assert (deg > 200).sum() >= 3
    assert int(np.sum((deg + 63) // 64)) >= 13 * 12


@pytest.mark.parametrize("k", KS256)
def test_oracle_reproduces_reference_h256(oracle, k):
    inp, g, mask, grad_x = load256(k)
    x, G = inp["x"], inp["G"]
    _, sel_o = oracle.np_cbsr(x, k)
    m_o = np.zeros_like(mask)
    np.put_along_axis(m_o, sel_o.astype(np.int64), True, axis=1)
    assert np.array_equal(m_o, mask)
    data, sel = cbsr_from_mask(x, mask, k)
    y = oracle.np_forward(inp["indptr"], inp["indices"], inp["values"], data, sel, 256)
    assert oracle.parity_error(y, g["Y"]) <= 1e-5
    dxs = oracle.np_backward(inp["indptr"], inp["indices"], inp["values"], G, sel)
    dense = np.zeros_like(x, dtype=np.float64)
    np.put_along_axis(dense, sel.astype(np.int64), dxs, axis=1)
    assert oracle.parity_error(dense, grad_x) <= 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("k", KS256)
def test_hip_reproduces_reference_h256(dev, k):
    """Top-k sets bit-exact; forward and every backward algorithm -- TILE
    included, which needs h = 256 -- within 1e-4 of the reference's vectors."""
    import torch

    import spgemm_new_amd as S
    from spgemm_new_amd import _lib
    from spgemm_new_amd.models import SpGEMMFunction, cbsr_topk
    inp, g, mask, grad_x = load256(k)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    x = t(inp["x"]).requires_grad_(True)
    gd = (t(inp["indptr"]), t(inp["indices"]), t(inp["values"]))
    _, sel = cbsr_topk(x.detach(), k)
    m = torch.zeros_like(x, dtype=torch.bool)
    m.scatter_(1, sel.long(), True)
    assert torch.equal(m.cpu(), torch.from_numpy(mask))
    y = SpGEMMFunction.apply(x, gd, k)
    y.backward(t(inp["G"]))
    rel = lambda a, b: np.max(np.abs(a - b) / np.maximum(1, np.abs(b)))  # noqa: E731
    assert rel(y.detach().cpu().numpy(), g["Y"]) <= TOL
    assert rel(x.grad.cpu().numpy(), grad_x) <= TOL
    graph = S.MaxKGraph(*gd)
    assert graph.tile_plan(k) is not None
    for algo in (_lib.MAXK_BWD_ATOMIC, _lib.MAXK_BWD_STAGED, _lib.MAXK_BWD_LOCAL,
                 _lib.MAXK_BWD_TILE):
        dxs = graph.backward(t(inp["G"]), sel, algo=algo)
        dense = torch.zeros_like(x).scatter_(1, sel.long(), dxs).cpu().numpy()
        assert rel(dense, grad_x) <= TOL, algo
