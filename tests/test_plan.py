"""Native plan builders (csrc/maxk_plan.hip) against numpy restatements (GPU).

The CSC transpose must be the stable one (edges of a column in CSR order); the
LOCAL plan must cover every destination with ranges of at most dmax columns
cut at the balanced in-degree points, list every edge exactly once, in
source-row order within its range, with (row, column) and value intact; the
band table must point at the first edge of each band.
"""
import ctypes

import numpy as np
import pytest
import torch

import spgemm_new_amd as S
from spgemm_new_amd import _lib
from spgemm_new_amd.graphs import small_csr

pytestmark = pytest.mark.gpu


def T(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def graphs():
    yield "mixed", *small_csr(3000, seed=31)


@pytest.mark.parametrize("name", ["mixed"])
def test_csc_build_stable(dev, name):
    _, indptr, indices = next(g for g in graphs() if g[0] == name)
    g = S.MaxKGraph(T(indptr, dev), T(indices, dev))
    csc_pos, csc_indptr, _, _ = g.csc()
    order = np.argsort(indices, kind="stable")
    pos = np.empty_like(order)
    pos[order] = np.arange(len(order))
    cnt = np.bincount(indices, minlength=len(indptr) - 1)
    ref_ptr = np.r_[0, np.cumsum(cnt)]
    assert np.array_equal(csc_indptr.cpu().numpy(), ref_ptr)
    assert np.array_equal(csc_pos.cpu().numpy()[: len(indices)], pos)


def ref_local_plan(indptr, indices, V, dmax, Tw):
    E = len(indices)
    csc_ptr = np.r_[0, np.cumsum(np.bincount(indices, minlength=V))].astype(np.int64)
    cuts = [0]
    for w in range(1, Tw):
        cuts.append(int(np.searchsorted(csc_ptr * Tw, w * E, side="left")))
    cuts.append(V)
    cuts = np.unique(cuts)
    dstart = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        dstart.extend(range(a, b, dmax))
    dstart = np.array(dstart + [V], np.int64)
    rows = np.repeat(np.arange(len(indptr) - 1), np.diff(indptr))
    owner = np.searchsorted(dstart, indices, side="right") - 1
    perm = np.argsort(owner, kind="stable")
    woff = np.r_[0, np.cumsum(np.bincount(owner, minlength=len(dstart) - 1))]
    erc = rows[perm] | ((indices[perm] - dstart[owner[perm]]) << 24)
    return dstart, woff, perm, erc


@pytest.mark.parametrize("k", [8, 32, 64])
def test_local_plan_build(dev, k):
    _, indptr, indices = next(graphs())
    V = len(indptr) - 1
    values = np.random.default_rng(k).random(len(indices), dtype=np.float32)
    g = S.MaxKGraph(T(indptr, dev), T(indices, dev), T(values, dev))
    plan = g.local_plan(k)
    dmax, W = plan["dmax"], plan["num_waves"]
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    from spgemm_new_amd.ops import LOCAL_WAVES_PER_CU
    Tw = max(-(-V // dmax), min(cus * LOCAL_WAVES_PER_CU, V))
    dstart, woff, perm, erc = ref_local_plan(indptr, indices.astype(np.int64), V, dmax, Tw)
    assert W == len(dstart) - 1
    assert np.array_equal(plan["dstart"].cpu().numpy(), dstart)
    assert np.all(np.diff(dstart) <= dmax) and np.all(np.diff(dstart) > 0)
    assert np.array_equal(plan["woff"].cpu().numpy(), woff)
    assert np.array_equal(plan["perm"].cpu().numpy(), perm)
    assert np.array_equal(plan["edge_rc"].cpu().numpy(), erc.astype(np.int32))
    assert np.array_equal(plan["edge_val"].cpu().numpy(), values[perm])
    # bands: first edge of each band per range; row NS = range ends
    for band_bytes in (1 << 16, 1 << 20):
        import spgemm_new_amd.ops as O
        old = O.LOCAL_BAND_BYTES
        O.LOCAL_BAND_BYTES = band_bytes
        try:
            seg, ns = g.local_bands(plan, 256)
        finally:
            O.LOCAL_BAND_BYTES = old
        seg = seg.cpu().numpy().reshape(ns + 1, W)
        rows = erc & 0xFFFFFF
        for s in range(ns):
            cut = s * (len(indptr) - 1) // ns
            ref = [woff[w] + np.searchsorted(rows[woff[w]:woff[w + 1]], cut) for w in range(W)]
            assert np.array_equal(seg[s], ref)
        assert np.array_equal(seg[ns], woff[1:])


def test_plan_abi_count_then_fill(dev):
    """The two-call protocol from C: count (dstart NULL) then fill; bad
    arguments return MAXK_E_ARG without launching."""
    _, indptr, indices = next(graphs())
    V, E = len(indptr) - 1, len(indices)
    L = _lib.load()
    ip, ix = T(indptr, dev), T(indices, dev)
    g = S.MaxKGraph(ip, ix)
    _, csc_indptr, _, _ = g.csc()
    ws = torch.empty(L.maxk_local_plan_workspace_bytes(E, V, 64), dtype=torch.uint8, device=dev)
    n = ctypes.c_int32(0)
    st = _lib.stream_ptr()
    rc = L.maxk_local_plan_build(ip.data_ptr(), ix.data_ptr(), None, V, V, E, csc_indptr.data_ptr(),
                                 64, 64, None, None, None, None, None, ctypes.byref(n),
                                 ws.data_ptr(), ws.numel(), st)
    assert rc == 0 and n.value >= 64 and n.value >= -(-V // 64)
    rc = L.maxk_local_plan_build(ip.data_ptr(), ix.data_ptr(), None, V, V, E, csc_indptr.data_ptr(),
                                 300, 64, None, None, None, None, None, ctypes.byref(n),
                                 ws.data_ptr(), ws.numel(), st)
    assert rc == _lib.MAXK_E_ARG   # dmax > 256
    rc = L.maxk_csc_build(ix.data_ptr(), E, V, None, None, None, 0, st)
    assert rc == _lib.MAXK_E_ARG
