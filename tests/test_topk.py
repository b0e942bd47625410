"""CBSR producer (maxk_topk_cbsr), dense scatter and MaxK mask on the GPU.

Parity: the selected index set per row equals torch.topk's
(continuous random inputs, so no ties), data[r, j] == x[r, sel[r, j]] exactly;
in value order the (value, index) sequence equals torch.topk(sorted=True).
Ties, NaN and signed zero follow the documented rule (NaN largest, -0 == +0,
ties to the lower column), checked against a numpy restatement.
"""
import numpy as np
import pytest
import torch

import spgemm_new_amd as S
from spgemm_new_amd import _lib

pytestmark = pytest.mark.gpu


def _expected_sets(x: np.ndarray, k: int):
    """Reference rule on the host: order by (key desc, column asc)."""
    V, h = x.shape
    out = []
    for r in range(V):
        row = x[r].astype(np.float64)
        isnan = np.isnan(row)
        key = np.where(isnan, 0.0, row) + 0.0   # -0 == +0
        order = np.lexsort((np.arange(h), -key, ~isnan))  # NaN first, then value desc, col asc
        out.append(order[:k])
    return out


@pytest.mark.parametrize("h", [256, 64, 100, 4, 255])
@pytest.mark.parametrize("k", [1, 8, 16, 32, 64, 256])
def test_topk_sets_match_torch(dev, h, k):
    if k > h:
        pytest.skip("k > dim")
    g = torch.Generator(device=dev)
    g.manual_seed(h * 1000 + k)
    x = torch.randn((1537, h), generator=g, device=dev)
    data, sel = S.topk_cbsr(x, k, order="column")
    ref = torch.topk(x, k, dim=1).indices
    s_mine = torch.sort(sel.long(), dim=1).values
    s_ref = torch.sort(ref, dim=1).values
    assert torch.equal(s_mine, s_ref)
    assert torch.equal(sel.long(), s_mine)  # column order is ascending
    assert torch.equal(data, torch.gather(x, 1, sel.long()))


@pytest.mark.parametrize("h,k", [(256, 32), (256, 64), (64, 16), (256, 256), (100, 7)])
def test_topk_value_order_matches_torch(dev, h, k):
    g = torch.Generator(device=dev)
    g.manual_seed(7 + h + k)
    x = torch.rand((999, h), generator=g, device=dev)
    data, sel = S.topk_cbsr(x, k, order="value")
    ref_v, ref_i = torch.topk(x, k, dim=1)
    assert torch.equal(sel.long(), ref_i)
    assert torch.equal(data, ref_v)


def test_topk_ties_nan_signed_zero(dev):
    rng = np.random.default_rng(3)
    x = rng.integers(0, 4, size=(300, 256)).astype(np.float32)   # heavy ties
    x[::7, 5] = np.nan
    x[1::5, :40] = -0.0
    x[2::5, :40] = 0.0
    for k in (1, 3, 32, 200):
        data, sel = S.topk_cbsr(torch.from_numpy(x).to(dev), k, order="value")
        exp = _expected_sets(x, k)
        got = sel.cpu().numpy()
        for r in range(x.shape[0]):
            assert list(got[r]) == list(exp[r]), (k, r)
        d = data.cpu().numpy()
        np.testing.assert_array_equal(np.isnan(d), np.isnan(np.take_along_axis(x, got.astype(np.int64), 1)))
        dc, sc = S.topk_cbsr(torch.from_numpy(x).to(dev), k, order="column")
        assert np.array_equal(np.sort(got, 1), sc.cpu().numpy())


def test_topk_dense_and_mask(dev):
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    x = torch.randn((777, 256), generator=g, device=dev)
    data, sel, dense = S.topk_cbsr(x, 32, dense=True)
    mask = torch.zeros_like(x).scatter_(1, torch.topk(x, 32, dim=1).indices, 1.0)
    assert torch.equal(dense, x * mask)
    grad = torch.randn((777, 256), generator=g, device=dev)
    assert torch.equal(S.cbsr_mask(grad, sel), grad * mask)
    vals = torch.randn((777, 32), generator=g, device=dev)
    ref = torch.zeros_like(x).scatter_(1, sel.long(), vals)
    assert torch.equal(S.cbsr_scatter(vals, sel, 256), ref)
    # rectangular / odd widths
    vals7 = torch.randn((5, 7), generator=g, device=dev)
    _, sel7 = S.topk_cbsr(torch.randn((5, 100), generator=g, device=dev), 7)
    ref7 = torch.zeros((5, 100), device=dev).scatter_(1, sel7.long(), vals7)
    assert torch.equal(S.cbsr_scatter(vals7, sel7, 100), ref7)


def test_topk_errors_and_empty(dev):
    x = torch.rand((4, 300), device=dev)
    with pytest.raises(RuntimeError, match="dim <= 256"):
        S.topk_cbsr(x, 8)
    with pytest.raises(RuntimeError):
        S.topk_cbsr(torch.rand((4, 16), device=dev), 17)
    with pytest.raises(RuntimeError, match="must be CUDA"):
        S.topk_cbsr(torch.rand((4, 16)), 4)
    with pytest.raises(RuntimeError, match="order"):
        S.topk_cbsr(torch.rand((4, 16), device=dev), 4, order="random")
    d, s = S.topk_cbsr(torch.empty((0, 64), device=dev), 8)
    assert d.shape == (0, 8) and s.shape == (0, 8)
    L = _lib.load()
    assert L.maxk_topk_cbsr(None, 1, 64, 64, 8, 0, None, None, None, None) == _lib.MAXK_E_ARG


def test_maxk_autograd_matches_reference_semantics(dev):
    """utils/models.py:28-59: forward keeps the top-k, backward masks the gradient."""
    from spgemm_new_amd.models import MaxK
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    x = torch.randn((300, 256), generator=g, device=dev, requires_grad=True)
    y = MaxK.apply(x, 16)
    idx = torch.topk(x.detach(), 16, dim=1).indices
    mask = torch.zeros_like(x).scatter_(1, idx, 1.0)
    assert torch.equal(y, x.detach() * mask)
    gy = torch.randn_like(y)
    y.backward(gy)
    assert torch.equal(x.grad, gy * mask)


@pytest.mark.parametrize("k", [8, 16, 32, 64, 24])
def test_topk_lane_order_is_a_permutation(dev, k):
    """Lane order = column order with rank q at VEC*(q % LPE) + q // LPE."""
    g = torch.Generator(device=dev)
    g.manual_seed(k)
    x = torch.randn((500, 256), generator=g, device=dev)
    dc, sc = S.topk_cbsr(x, k, order="column")
    dl, sl = S.topk_cbsr(x, k, order="lane")
    vec = 4 if k >= 32 else (2 if k >= 16 else 1)
    if k % vec:
        pos = list(range(k))
    else:
        lpe = k // vec
        pos = [vec * (q % lpe) + q // lpe for q in range(k)]
    assert sorted(pos) == list(range(k))
    idx = torch.tensor(pos, device=dev)
    assert torch.equal(sl[:, idx], sc)
    assert torch.equal(dl[:, idx], dc)


def test_topk_abi_row_stride(dev):
    """C ABI: rows ld floats apart (a column slice of a wider matrix)."""
    g = torch.Generator(device=dev)
    g.manual_seed(21)
    big = torch.randn((300, 132), generator=g, device=dev)
    for dim, k in ((100, 16), (128, 32), (7, 3)):
        data = torch.empty((300, k), device=dev)
        sel = torch.empty((300, k), dtype=torch.uint8, device=dev)
        L = _lib.load()
        assert L.maxk_topk_cbsr(big.data_ptr(), 300, dim, 132, k, _lib.MAXK_TOPK_ORDER_VALUE,
                                data.data_ptr(), sel.data_ptr(), None, None) == 0
        torch.cuda.synchronize()
        ref_v, ref_i = torch.topk(big[:, :dim], k, dim=1)
        assert torch.equal(sel.long(), ref_i) and torch.equal(data, ref_v)
    assert L.maxk_topk_cbsr(big.data_ptr(), 300, 100, 99, 8, 0, data.data_ptr(), sel.data_ptr(),
                            None, None) == _lib.MAXK_E_DIM
