"""Column-blocked forward (ops._forward_blocked, maxk_rows_sum, the
MAXK_FWD_CACHED_GATHER flag) against the CPU oracle: every block count, lanes
and shapes the plain forward covers, rectangular blocks, values that change
in place or arrive per call, hipGraph capture, and AUTO's choice.  Same
tolerance as test_gpu_parity (the blocks change the fp32 summation order)."""
import numpy as np
import pytest
import torch

import spgemm_new_amd as S
from spgemm_new_amd import _lib, ops
from spgemm_new_amd.graphs import random_cbsr, small_csr

pytestmark = pytest.mark.gpu
TOL = 1e-4


def T(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _dense_graph(V, C, deg, seed):
    rng = np.random.default_rng(seed)
    d = rng.poisson(deg, V)
    d[:3] = [0, C, 1]                                  # an empty row, a full row, a single edge
    indptr = np.zeros(V + 1, np.int64)
    indptr[1:] = np.cumsum(d)
    idx = np.concatenate([np.sort(rng.choice(C, size=x, replace=False)) for x in d])
    vals = rng.uniform(-1, 1, idx.size).astype(np.float32)
    return indptr.astype(np.int32), idx.astype(np.int32), vals


@pytest.mark.parametrize("nb", [1, 2, 3, 8, 16])
@pytest.mark.parametrize("k", [32, 64])
def test_blocked_forward_matches_oracle(dev, oracle, nb, k):
    indptr, idx, vals = _dense_graph(2000, 2000, 150, seed=nb + k)
    data, sel = random_cbsr(2000, k, 256, seed=k)
    g = S.MaxKGraph(T(indptr, dev), T(idx, dev), T(vals, dev))
    out = torch.full((2000, 256), float("nan"), device=dev)
    ops._forward_blocked(g, nb, T(data, dev), T(sel, dev), 256, out, g.values)
    ref = oracle.np_forward(indptr, idx, vals, data, sel, 256)
    assert oracle.parity_error(out.cpu().numpy(), ref) <= TOL


def test_blocked_forward_small_graph_and_narrow_rows(dev, oracle):
    """The degree-mix graph of the parity tests (degrees 0 .. 3000) and h < 256."""
    indptr, idx = small_csr(3000, seed=21)
    vals = np.random.default_rng(2).random(len(idx), dtype=np.float32)
    g = S.MaxKGraph(T(indptr, dev), T(idx, dev), T(vals, dev), panel_cost=300)
    for k, h in [(32, 256), (48, 100), (64, 64)]:
        data, sel = random_cbsr(3000, k, h, seed=k + h)
        out = torch.empty((3000, h), device=dev)
        ops._forward_blocked(g, 8, T(data, dev), T(sel, dev), h, out, g.values)
        ref = oracle.np_forward(indptr, idx, vals, data, sel, h)
        assert oracle.parity_error(out.cpu().numpy(), ref) <= TOL


def test_blocked_forward_rectangular(dev, oracle):
    """A rank's block: more columns than rows."""
    indptr, idx, vals = _dense_graph(700, 2500, 200, seed=4)
    data, sel = random_cbsr(2500, 32, 256, seed=9)
    g = S.MaxKGraph(T(indptr, dev), T(idx, dev), T(vals, dev), num_cols=2500)
    out = torch.empty((700, 256), device=dev)
    ops._forward_blocked(g, 8, T(data, dev), T(sel, dev), 256, out, g.values)
    ref = oracle.np_forward(indptr, idx, vals, data, sel, 256)
    assert oracle.parity_error(out.cpu().numpy(), ref) <= TOL


def test_blocked_forward_values_in_place_and_per_call(dev, oracle):
    indptr, idx, vals = _dense_graph(1500, 1500, 160, seed=5)
    data, sel = random_cbsr(1500, 32, 256, seed=2)
    g = S.MaxKGraph(T(indptr, dev), T(idx, dev), T(vals, dev))
    D, Sl = T(data, dev), T(sel, dev)
    out = torch.empty((1500, 256), device=dev)
    ops._forward_blocked(g, 4, D, Sl, 256, out, g.values)
    g.values.mul_(-2.0)                                # in place: the plan's copy must follow
    ops._forward_blocked(g, 4, D, Sl, 256, out, g.values)
    ref = oracle.np_forward(indptr, idx, -2.0 * vals, data, sel, 256)
    assert oracle.parity_error(out.cpu().numpy(), ref) <= TOL
    w = np.random.default_rng(3).random(len(idx), dtype=np.float32)
    ops._forward_blocked(g, 4, D, Sl, 256, out, T(w, dev))
    ref = oracle.np_forward(indptr, idx, w, data, sel, 256)
    assert oracle.parity_error(out.cpu().numpy(), ref) <= TOL


def test_blocked_forward_under_hipgraph(dev, oracle):
    indptr, idx, vals = _dense_graph(1500, 1500, 160, seed=6)
    data, sel = random_cbsr(1500, 32, 256, seed=3)
    g = S.MaxKGraph(T(indptr, dev), T(idx, dev), T(vals, dev))
    D, Sl = T(data, dev), T(sel, dev)
    out = torch.empty((1500, 256), device=dev)
    ops._forward_blocked(g, 8, D, Sl, 256, out, g.values)      # plan and buffers first
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s), torch.cuda.graph(graph, stream=s):
        ops._forward_blocked(g, 8, D, Sl, 256, out, g.values)
    torch.cuda.current_stream().wait_stream(s)
    g.values.mul_(0.5)
    out.zero_()
    graph.replay()
    torch.cuda.synchronize()
    ref = oracle.np_forward(indptr, idx, 0.5 * vals, data, sel, 256)
    assert oracle.parity_error(out.cpu().numpy(), ref) <= TOL


def test_rows_sum_order_and_tail(dev):
    L = _lib.load()
    for n in (1, 7, 1024, 4099):
        parts = torch.randn(5, n, device=dev)
        out = torch.empty(n, device=dev)
        _lib.check(L.maxk_rows_sum(parts.data_ptr(), 5, n, out.data_ptr(), None), "rows_sum")
        ref = parts[0].clone()
        for q in range(1, 5):
            ref += parts[q]
        torch.cuda.synchronize()
        assert torch.equal(out, ref)
    assert L.maxk_rows_sum(None, 0, 4, None, None) == _lib.MAXK_E_ARG


def test_auto_chooses_and_stays_correct(dev, oracle, monkeypatch):
    """AUTO (MAXK_FWD_BLOCKS=-1) measures the blocked forward against the plain
    one on a long-row graph, keeps its choice per (k, h), and is right either way;
    short-row graphs never try it."""
    monkeypatch.setattr(ops, "FWD_BLOCKS", -1)
    indptr, idx, vals = _dense_graph(2000, 2000, 300, seed=8)
    data, sel = random_cbsr(2000, 32, 256, seed=4)
    g = S.MaxKGraph(T(indptr, dev), T(idx, dev), T(vals, dev))
    y = g.forward(T(data, dev), T(sel, dev), 256)
    assert (32, 256) in g._fwd_blocks
    ref = oracle.np_forward(indptr, idx, vals, data, sel, 256)
    assert oracle.parity_error(y.cpu().numpy(), ref) <= TOL
    indptr2, idx2 = small_csr(3000, seed=21)           # mean degree < 128
    g2 = S.MaxKGraph(T(indptr2, dev), T(idx2, dev))
    g2.forward(T(random_cbsr(3000, 32, 256, seed=1)[0], dev),
               T(random_cbsr(3000, 32, 256, seed=1)[1], dev), 256)
    assert g2._fwd_blocks[(32, 256)] == 0 and not g2._blocked


@pytest.mark.parametrize("nb", [1, 3, 8])
def test_blocked_plan_builder_matches_torch_reference(dev, nb):
    """maxk_blocked_plan_build (device radix sort) == a stable torch sort of the
    (column block, row) keys; values permuted by the same order."""
    indptr, idx, vals = _dense_graph(1200, 3100, 40, seed=nb)
    g = S.MaxKGraph(T(indptr, dev), T(idx, dev), T(vals, dev), num_cols=3100)
    plan = g.blocked_plan(nb)
    V, C = 1200, 3100
    rows = torch.repeat_interleave(torch.arange(V, device=dev), (g.indptr[1:] - g.indptr[:-1]).long())
    key = (g.indices.long() * nb) // C * V + rows
    key, order = torch.sort(key, stable=True)
    ip = torch.zeros(nb * V + 1, dtype=torch.int32, device=dev)
    ip[1:] = torch.cumsum(torch.bincount(key, minlength=nb * V), 0).to(torch.int32)
    assert torch.equal(plan["indptr"], ip)
    assert torch.equal(plan["order"].long(), order)
    assert torch.equal(plan["indices"], g.indices[order])
    assert torch.equal(g._blocked_values(plan, g.values), g.values[order])


def _blocked_all_parts_then_sum(g, nb, data, sel, h, L):
    """The earlier form on the same panels: every block into its own partial
    (blocks 0..nb-2 on the head schedule, the last block on its own), then
    maxk_rows_sum over the nb parts."""
    plan = g.blocked_plan(nb)
    vals = g._blocked_values(plan, g.values)
    sp = ops._blocked_split(g, plan)
    V, k = g.num_rows, data.shape[1]
    P = max(sp["last_P"], sp.get("head_P", 1))
    ws = torch.empty(L.maxk_forward_workspace_bytes(P, h), dtype=torch.uint8, device=data.device)
    parts = torch.empty((nb, V, h), device=data.device)
    launches = [(sp["last_sched"], sp["last_P"], sp["last_indptr"], V, parts[nb - 1])]
    if nb > 1:
        launches.append((sp["head_sched"], sp["head_P"], plan["indptr"], sp["head_rows"], parts))
    for sched, np_, ip, rows, dst in launches:
        _lib.check(L.maxk_spgemm_forward_ex(sched.data_ptr(), np_, ip.data_ptr(),
                                            plan["indices"].data_ptr(), vals.data_ptr(),
                                            data.data_ptr(), sel.data_ptr(), rows, h, k,
                                            _lib.MAXK_FWD_CACHED_GATHER, dst.data_ptr(),
                                            ws.data_ptr(), ws.numel(), None), "fwd")
    out = torch.empty((V, h), device=data.device)
    _lib.check(L.maxk_rows_sum(parts.data_ptr(), nb, V * h, out.data_ptr(), None), "sum")
    return out


@pytest.mark.parametrize("nb", [1, 2, 4, 8])
def test_fused_last_block_sum_bitwise_equals_rows_sum(dev, nb):
    """maxk_spgemm_forward_sum_parts (the last block adds the partials in its
    row flush and in the split-row fixup) is bitwise the all-parts + rows_sum
    form: rows split over panels (panel_cost 300, degrees up to 3000), empty
    rows, h a multiple of 4 and not."""
    L = _lib.load()
    indptr, idx = small_csr(3000, seed=5)
    vals = np.random.default_rng(3).random(len(idx), dtype=np.float32)
    g = S.MaxKGraph(T(indptr, dev), T(idx, dev), T(vals, dev), panel_cost=300)
    for k, h in [(32, 256), (32, 98), (64, 256)]:
        data, sel = random_cbsr(3000, k, h, seed=k + h + nb)
        data, sel = T(data, dev), T(sel, dev)
        out = torch.full((3000, h), float("nan"), device=dev)
        ops._forward_blocked(g, nb, data, sel, h, out, g.values)
        ref = _blocked_all_parts_then_sum(g, nb, data, sel, h, L)
        assert torch.equal(out, ref), (nb, k, h)


def test_sum_parts_entry_arguments(dev):
    L = _lib.load()
    assert L.maxk_spgemm_forward_sum_parts(None, 1, None, None, None, None, None, 1, 256, 32, 0,
                                           None, 0, None, None, 0, None) == _lib.MAXK_E_ARG
    # accumulate is not a flag of this entry
    x = torch.zeros(16, device=dev)
    assert L.maxk_spgemm_forward_sum_parts(x.data_ptr(), 1, x.data_ptr(), None, None, None, None, 1,
                                           256, 32, _lib.MAXK_FWD_ACCUMULATE, None, 0, x.data_ptr(),
                                           None, 0, None) == _lib.MAXK_E_ARG
