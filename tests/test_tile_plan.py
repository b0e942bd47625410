"""TILE backward: the plan format (CPU: the torch reference builder's plan,
tests/tile_ref.py, replayed by spgemm_new_amd.tile.emulate against the float64
oracle), the device plan builder (GPU: maxk_tile_plan_build bit-identical to
the reference builder) and the kernel (GPU, against the oracle and the other
backward algorithms)."""
import ctypes

import numpy as np
import pytest
import torch

import tile_ref
from spgemm_new_amd import tile

TOL = 1e-4  # fp32 summation order vs the float64 oracle (north_star tolerance)


def _graph(V, C, avg_deg, seed, hub_rows=0):
    rng = np.random.default_rng(seed)
    deg = np.minimum(rng.poisson(avg_deg, V), C).astype(np.int64)
    if hub_rows:
        deg[:hub_rows] = min(C, avg_deg * 20)
    indptr = np.zeros(V + 1, np.int64)
    indptr[1:] = np.cumsum(deg)
    idx = np.concatenate([np.sort(rng.choice(C, size=d, replace=False)) for d in deg]) \
        if deg.sum() else np.zeros(0, np.int64)
    vals = rng.uniform(0, 1, idx.size).astype(np.float32)
    return indptr.astype(np.int32), idx.astype(np.int32), vals


def _inputs(V, C, seed, k=32, h=256):
    rng = np.random.default_rng(seed + 1)
    grad = rng.uniform(-1, 1, (V, h)).astype(np.float32)
    sel = np.stack([np.sort(rng.choice(h, k, replace=False)) for _ in range(C)]).astype(np.uint8)
    return grad, sel


@pytest.mark.parametrize("k", [32, 64])
@pytest.mark.parametrize("V,C,deg,shape,hubs", [
    (300, 300, 12, None, 0),           # one group, 8 source ranges, several chunks
    (800, 800, 6, None, 12),           # hub rows: chunks cut short where records pile up
    (500, 2600, 9, None, 0),           # groups > 2048 columns
    (700, 900, 20, (3, 300, 6), 0),    # forced: 3 groups of 300, 2 equal source ranges each
    (700, 900, 20, (3, 300, 4), 0),    # forced: 4 workgroups over 3 groups (pieces straddle)
    (900, 2500, 8, (3, 834, 7), 0),    # forced: 7 workgroups over 3 groups
    (200, 64, 4, (1, 64, 1), 0),       # few destinations, one range
    (5, 5, 2, None, 0),                # fewer source rows than ranges the CUs allow
    (3, 700, 40, None, 0),             # 3 source rows, many destinations
])
def test_plan_emulated_matches_oracle(oracle, V, C, deg, shape, hubs, k):
    """Both record formats (tile_format.h TILE_REC_WORDS 2 and 4) replayed on
    the CPU equal the oracle."""
    indptr, idx, vals = _graph(V, C, deg, seed=V + C, hub_rows=hubs)
    grad, sel = _inputs(V, C, seed=V, k=k)
    ref = oracle.np_backward(indptr, idx, vals, grad, sel)
    for rw in (2, 4):
        plan = tile_ref.build(torch.from_numpy(indptr), torch.from_numpy(idx),
                              torch.from_numpy(vals), V, C, cus=16, shape=shape, k=k,
                              record_words=rw)
        assert plan is not None and plan["records"].shape[1] == rw
        got = tile.emulate(plan, torch.from_numpy(grad), torch.from_numpy(sel)).numpy()
        assert oracle.parity_error(got, ref) < TOL


def test_plan_invariants():
    V, C = 400, 1000
    indptr, idx, vals = _graph(V, C, 15, seed=3)
    plan = tile_ref.build(torch.from_numpy(indptr), torch.from_numpy(idx), torch.from_numpy(vals),
                          V, C, cus=8)
    G, GS, P = plan["num_groups"], plan["group_size"], plan["num_workgroups"]
    assert G * GS >= C and GS <= tile.max_group(32)
    hdrs, recs = plan["headers"], plan["records"]
    hs, rs = plan["header_start"].tolist(), plan["record_start"].tolist()
    nch = plan["num_chunks"].tolist()
    NB, BR, _ = tile.ring_format()
    lead = NB - 1
    n_real = 0
    for b in range(G + P - 1):
        for wv in range(tile.WAVES):
            ro = rs[b * tile.WAVES + wv]
            for c in range(nch[b] + lead):
                e = hdrs[hs[b * tile.WAVES + wv] + c]
                assert all(int(r) == -1 or 0 <= int(r) < V for r in e[1:])
                if c >= lead:
                    n0, n1 = int(e[0]) & 0xFFFF, int(e[0]) >> 16
                    assert n0 % 4 == 0 and n1 % 4 == 0
                    seg = recs[ro: ro + n0 + n1]
                    real = seg[:, -1] != 0
                    n_real += int(real.sum())
                    # real records read rows of the chunk's own buffer
                    if seg.shape[1] == 2:
                        rowf = (seg[real][:, 0].long() & 0xFFFFFFFF) >> 24
                    else:
                        rowf = seg[real][:, 2].long() >> 10
                    assert bool(((rowf // BR) == (c - lead) % NB).all())
                    ro += n0 + n1
    assert n_real == int((torch.from_numpy(vals) != 0).sum())


@pytest.mark.parametrize("k", [32, 64])
@pytest.mark.parametrize("C", [1, 5, 63, 1000, 2048, 2049, 4096, 100_000, 232_965, 2_449_029])
@pytest.mark.parametrize("V", [1, 3, 5, 7, 40, 232_965])
@pytest.mark.parametrize("cus", [8, 256])
def test_shape_library_matches_reference(V, C, cus, k):
    """maxk_tile_plan_shape (C ABI, host code: no GPU needed) == the reference
    rule, and never asks for more workgroups than (group, source row) pairs:
    an empty workgroup range would leave a partial plane unwritten."""
    got = tile.choose_shape(V, C, cus, k)
    assert got == tile_ref.choose_shape(V, C, cus, k)
    G, GS, P = got
    assert P <= G * V and G * GS >= C


def test_oversubscribed_shape_refused_without_gpu():
    """num_workgroups > num_groups * num_rows is refused before any launch by the
    plan builder and the backward, and by tile.build."""
    from spgemm_new_amd import _lib
    L = _lib.load()
    a = 1 << 12   # aligned dummy pointers: validation fails before they are used
    rc = L.maxk_sspmm_backward_tile(a, a, a, a, a, 5, 40, 1, a, a, a, 5, 5, 256, 32, a, a, None)
    assert rc == _lib.MAXK_E_ARG
    rc = L.maxk_sspmm_backward_tile(a, a, a, a, a, 5, 25, 1, a, a, a, 5, 5, 1, 32, a, a, None)
    assert rc == _lib.MAXK_E_DIM          # the same call with P = G * V passes the shape check
    sizes = (ctypes.c_int64 * 3)()
    rc = L.maxk_tile_plan_build(a, a, a, 5, 5, 10, 32, 5, 1, 40, None, 0, None, None, 0, None, None,
                                None, sizes, a, 1 << 30, None)
    assert rc == _lib.MAXK_E_ARG
    idx = torch.zeros(3, dtype=torch.int32)
    with pytest.raises(ValueError):
        tile.build(torch.tensor([0, 3], dtype=torch.int32), idx, torch.ones(3), 1, 5,
                   shape=(5, 1, 6))


def test_emulator_leaves_unwritten_planes_nan():
    """The CPU replay starts its planes as NaN (the kernel's `part` is torch.empty),
    so a plan whose pieces missed a plane would fail test_plan_emulated_matches_oracle."""
    indptr, idx, vals = _graph(40, 300, 6, seed=3)
    plan = tile_ref.build(torch.from_numpy(indptr), torch.from_numpy(idx), torch.from_numpy(vals),
                          40, 300, shape=(2, 150, 8), k=32, record_words=4)
    grad, sel = _inputs(40, 300, seed=3)
    assert torch.isfinite(tile.emulate(plan, torch.from_numpy(grad), torch.from_numpy(sel))).all()


@pytest.mark.gpu
@pytest.mark.parametrize("k", [32, 64])
@pytest.mark.parametrize("V,C,splits", [(5, 5, None), (3, 700, None), (7, 7, 64), (2, 3000, 8)])
def test_tile_few_source_rows_nan_part(dev, oracle, V, C, splits, k):
    """Graphs with fewer source rows than the ranges the CUs would allow (and
    tile_splits > V): the shape must not create empty workgroup ranges, whose
    partial planes tile_combine_kernel would add unwritten.  `part` is filled
    with NaN first, so any plane the kernel skips shows up."""
    import spgemm_new_amd as S
    from spgemm_new_amd import _lib
    indptr, idx, vals = _graph(V, C, min(C // 2, 30), seed=V * 7 + C)
    grad, sel = _inputs(V, C, seed=V + C, k=k)
    g = S.MaxKGraph(torch.from_numpy(indptr).to(dev), torch.from_numpy(idx).to(dev),
                    torch.from_numpy(vals).to(dev), num_cols=C, tile_splits=splits)
    plan = g.tile_plan(k)
    assert plan is not None
    assert plan["num_workgroups"] <= plan["num_groups"] * V
    plan["part"].fill_(float("nan"))
    got = g.backward(torch.from_numpy(grad).to(dev), torch.from_numpy(sel).to(dev),
                     algo=_lib.MAXK_BWD_TILE)
    assert g.last_bwd_algo == "tile"
    ref = oracle.np_backward(indptr, idx, vals, grad, sel)
    assert oracle.parity_error(got.cpu().numpy(), ref) < TOL


@pytest.mark.parametrize("V,G,P", [(1, 1, 1), (300, 1, 8), (300, 3, 4), (900, 3, 7), (232_965, 128, 256),
                                   (232_965, 114, 256), (232_965, 128, 240), (2_449_029, 2392, 2392),
                                   (10, 7, 64)])
def test_part_planes_and_pieces(V, G, P):
    """maxk_tile_part_planes (C ABI, host code) == the Python piece formula, and
    the pieces of all workgroups tile the (group, row) space exactly once, each
    group's pieces in consecutive workgroups with planes 0, 1, ..."""
    from spgemm_new_amd import _lib
    assert _lib.load().maxk_tile_part_planes(V, G, P) == tile.part_planes(V, G, P)
    seen = {}
    for b in range(P):
        for pid, g, plane in tile.pieces_of(b, V, G, P):
            assert pid == g + b and 0 <= g < G
            seen.setdefault(g, []).append((b, plane))
    assert sorted(seen) == list(range(G))
    for g, lst in seen.items():
        assert [pl for _, pl in lst] == list(range(len(lst)))
        assert [b for b, _ in lst] == list(range(lst[0][0], lst[0][0] + len(lst)))
        assert len(lst) - 1 <= tile.part_planes(V, G, P)
    # rows: piece of (g, r) from the plan formula covers every row exactly once
    if V * G <= 5000:
        for g in range(G):
            pids = {g + (g * V + r) * P // (G * V) for r in range(V)}
            assert pids == {pid for b in range(P) for pid, gg, _ in tile.pieces_of(b, V, G, P) if gg == g}


_KEYS = ("headers", "header_start", "records", "record_start", "num_chunks")


@pytest.mark.gpu
@pytest.mark.parametrize("k", [32, 64])
@pytest.mark.parametrize("V,C,deg,shape,hubs", [
    (300, 300, 12, None, 0), (800, 800, 6, None, 12), (500, 2600, 9, None, 0),
    (700, 900, 20, (3, 300, 6), 0), (700, 900, 20, (3, 300, 4), 0), (200, 64, 4, (1, 64, 1), 0),
    (3000, 3000, 40, None, 0), (4000, 1500, 30, (2, 750, 10), 0),
    (4000, 1500, 30, (2, 750, 9), 0), (1, 5, 3, None, 0),
])
def test_device_plan_matches_reference_builder(dev, V, C, deg, shape, hubs, k):
    """maxk_tile_plan_build (device) == the torch reference builder, bit for
    bit, and edge_record points every CSR edge at its own record."""
    indptr, idx, vals = _graph(V, C, deg, seed=V + C, hub_rows=hubs)
    if idx.size == 0:
        pytest.skip("empty graph")
    args = [torch.from_numpy(a).to(dev) for a in (indptr, idx, vals)]
    got = tile.build(*args, V, C, cus=16, shape=shape, k=k)
    ref = tile_ref.build(*args, V, C, cus=16, shape=shape, k=k)
    assert (got is None) == (ref is None)
    if got is None:
        return
    for key in ("num_groups", "group_size", "num_workgroups", "part_planes"):
        assert got[key] == ref[key], key
    for key in _KEYS:
        a, b = got[key].cpu(), ref[key].cpu().to(got[key].dtype)
        assert a.shape == b.shape and torch.equal(a, b), key
    rec = got["records"].cpu()
    er = got["edge_record"].cpu().long()
    assert torch.equal(rec[er, -1], args[2].cpu().view(torch.int32))
    # set_values rewrites exactly the value words
    new = torch.rand(idx.size, device=dev)
    tile.set_values(got, new)
    rec2 = got["records"].cpu()
    assert torch.equal(rec2[er, -1], new.cpu().view(torch.int32))
    assert torch.equal(rec2[:, :-1], rec[:, :-1])


@pytest.mark.gpu
def test_tile_values_changed_in_place(dev, oracle):
    """The graph's values mutated in place after the TILE plan was built: TILE
    must see the new values (same as STAGED on the new values)."""
    import spgemm_new_amd as S
    from spgemm_new_amd import _lib
    V = 3000
    indptr, idx, vals = _graph(V, V, 40, seed=21)
    grad, sel = _inputs(V, V, seed=21)
    g = S.MaxKGraph(torch.from_numpy(indptr).to(dev), torch.from_numpy(idx).to(dev),
                    torch.from_numpy(vals).to(dev))
    G, sl = torch.from_numpy(grad).to(dev), torch.from_numpy(sel).to(dev)
    g.backward(G, sl, algo=_lib.MAXK_BWD_TILE)
    g.values.mul_(-2.0).add_(0.25)          # an optimizer step on the edge weights
    got = g.backward(G, sl, algo=_lib.MAXK_BWD_TILE)
    staged = g.backward(G, sl, algo=_lib.MAXK_BWD_STAGED)
    ref = oracle.np_backward(indptr, idx, g.values.cpu().numpy(), grad, sel)
    assert oracle.parity_error(got.cpu().numpy(), ref) < TOL
    assert (got - staged).abs().max().item() <= 1e-4 * max(1.0, staged.abs().max().item())


@pytest.mark.gpu
def test_tile_with_per_call_values(dev):
    """TILE with values other than the graph's own (its records are rewritten
    when the values they hold change): explicit and AUTO calls, alternating
    with own-values calls, all equal STAGED on the same values; AUTO keeps a
    separate choice for foreign values."""
    import spgemm_new_amd as S
    V = 3000
    indptr, idx, vals = _graph(V, V, 40, seed=5)
    grad, sel = _inputs(V, V, seed=5)
    g = S.MaxKGraph(torch.from_numpy(indptr).to(dev), torch.from_numpy(idx).to(dev),
                    torch.from_numpy(vals).to(dev))
    G, sl = torch.from_numpy(grad).to(dev), torch.from_numpy(sel).to(dev)
    w = torch.rand(idx.size, device=dev)

    def close(a, b):
        return (a - b).abs().max().item() <= 1e-4 * max(1.0, b.abs().max().item())
    ref_own = g.backward(G, sl, algo=S._lib.MAXK_BWD_STAGED)
    ref_w = g.backward(G, sl, values=w, algo=S._lib.MAXK_BWD_STAGED)
    for _ in range(2):   # own -> foreign -> own ...: the records follow
        own = g.backward(G, sl, algo=S._lib.MAXK_BWD_TILE)
        assert close(own, ref_own)
        other = g.backward(G, sl, values=w, algo=S._lib.MAXK_BWD_TILE)
        assert g.last_bwd_algo == "tile" and close(other, ref_w)
    w.mul_(0.5)          # foreign values changed in place: refreshed too
    assert close(g.backward(G, sl, values=w, algo=S._lib.MAXK_BWD_TILE), 0.5 * ref_w)
    a_own = g.backward(G, sl)
    a_w = g.backward(G, sl, values=w)
    assert close(a_own, ref_own) and close(a_w, 0.5 * ref_w)
    assert (32, 256, True) in g._bwd_choice and (32, 256, False) in g._bwd_choice


@pytest.mark.gpu
def test_tile_capture_sees_value_changes(dev):
    """A captured TILE backward records the records refresh, so edge values
    updated in place between replays are used."""
    import spgemm_new_amd as S
    V = 3000
    indptr, idx, vals = _graph(V, V, 40, seed=8)
    grad, sel = _inputs(V, V, seed=8)
    g = S.MaxKGraph(torch.from_numpy(indptr).to(dev), torch.from_numpy(idx).to(dev),
                    torch.from_numpy(vals).to(dev))
    G, sl = torch.from_numpy(grad).to(dev), torch.from_numpy(sel).to(dev)
    dx = torch.empty((V, 32), device=dev)
    g.backward(G, sl, out=dx, algo=S._lib.MAXK_BWD_TILE)     # plan built outside the capture
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    stream = torch.cuda.Stream()
    stream.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(stream):
        with torch.cuda.graph(graph, stream=stream):
            g.backward(G, sl, out=dx, algo=S._lib.MAXK_BWD_TILE)
    torch.cuda.current_stream().wait_stream(stream)
    g.values.mul_(3.0)
    graph.replay()
    torch.cuda.synchronize()
    ref = g.backward(G, sl, algo=S._lib.MAXK_BWD_STAGED)
    assert (dx - ref).abs().max().item() <= 1e-4 * max(1.0, ref.abs().max().item())


@pytest.mark.gpu
def test_tile_capture_then_foreign_values(dev):
    """a replay rewrites the TILE records with the graph's own values
    behind the Python state.  Sequence: capture with own values, eager with
    foreign values w, replay, eager with w again -- the last eager call must
    use w (the records are rewritten on every eager call once captured)."""
    import spgemm_new_amd as S
    V = 3000
    indptr, idx, vals = _graph(V, V, 40, seed=11)
    grad, sel = _inputs(V, V, seed=11)
    g = S.MaxKGraph(torch.from_numpy(indptr).to(dev), torch.from_numpy(idx).to(dev),
                    torch.from_numpy(vals).to(dev))
    G, sl = torch.from_numpy(grad).to(dev), torch.from_numpy(sel).to(dev)
    w = torch.rand(idx.size, device=dev)
    dx = torch.empty((V, 32), device=dev)
    g.backward(G, sl, out=dx, algo=S._lib.MAXK_BWD_TILE)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    stream = torch.cuda.Stream()
    stream.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(stream):
        with torch.cuda.graph(graph, stream=stream):
            g.backward(G, sl, out=dx, algo=S._lib.MAXK_BWD_TILE)
    torch.cuda.current_stream().wait_stream(stream)
    ref_own = g.backward(G, sl, algo=S._lib.MAXK_BWD_STAGED)
    ref_w = g.backward(G, sl, values=w, algo=S._lib.MAXK_BWD_STAGED)

    def close(a, b):
        return (a - b).abs().max().item() <= 1e-4 * max(1.0, b.abs().max().item())
    assert close(g.backward(G, sl, values=w, algo=S._lib.MAXK_BWD_TILE), ref_w)
    graph.replay()
    torch.cuda.synchronize()
    assert close(dx, ref_own)
    assert close(g.backward(G, sl, values=w, algo=S._lib.MAXK_BWD_TILE), ref_w)
    assert close(g.backward(G, sl, algo=S._lib.MAXK_BWD_TILE), ref_own)


@pytest.mark.gpu
def test_edge_selector_buffer_pinned_under_capture(dev):
    """an edge-selector buffer written under capture is never handed to
    another selector tensor (a replay would overwrite it between that tensor's
    eager forward and backward)."""
    import spgemm_new_amd as S
    from spgemm_new_amd import ops
    V = 3000
    indptr, idx, vals = _graph(V, V, 40, seed=12)
    g = S.MaxKGraph(torch.from_numpy(indptr).to(dev), torch.from_numpy(idx).to(dev),
                    torch.from_numpy(vals).to(dev))
    k, h = 16, 256
    gen = torch.Generator(device=dev)
    gen.manual_seed(3)
    sels = [torch.argsort(torch.rand((V, h), generator=gen, device=dev), 1)[:, :k].sort(1)
            .values.to(torch.uint8).contiguous() for _ in range(ops.ESEL_CACHE + 2)]
    data = torch.rand((V, k), generator=gen, device=dev)
    y = torch.empty((V, h), device=dev)
    g.forward(data, sels[0], h, out=y, edge_sel=True)    # outside: a plain slot
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    stream = torch.cuda.Stream()
    stream.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(stream):
        with torch.cuda.graph(graph, stream=stream):
            g.forward(data, sels[1], h, out=y, edge_sel=True)
    torch.cuda.current_stream().wait_stream(stream)
    pinned = g.edge_selectors(sels[1])
    assert pinned is not None
    for s in sels[2:]:                                    # more than the cache holds
        g.forward(data, s, h, out=y, edge_sel=True)
        assert g.edge_selectors(s).data_ptr() != pinned.data_ptr()
    assert g.edge_selectors(sels[1]) is pinned
    graph.replay()
    torch.cuda.synchronize()
    es = g.edge_selectors(sels[-1]).view(-1)[: idx.size * k].view(idx.size, k)
    ref = sels[-1][torch.from_numpy(idx).to(dev).long()]
    assert torch.equal(es, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("V,C,deg,k", [(3000, 3000, 40, 32), (9000, 9000, 120, 32),
                                       (3000, 5000, 60, 32), (4000, 1500, 30, 32),
                                       (3000, 3000, 40, 64), (5000, 2500, 50, 64)])
def test_tile_backward_gpu_matches_oracle(dev, oracle, V, C, deg, k):
    """Square and rectangular (a multi-GPU rank's block with halo columns), k = 32 and 64."""
    import spgemm_new_amd as S
    from spgemm_new_amd import _lib
    indptr, idx, vals = _graph(V, C, deg, seed=V + C)
    grad, sel = _inputs(V, C, seed=V, k=k)
    g = S.MaxKGraph(torch.from_numpy(indptr).to(dev), torch.from_numpy(idx).to(dev),
                    torch.from_numpy(vals).to(dev), num_cols=C)
    assert g.tile_plan(k) is not None
    G = torch.from_numpy(grad).to(dev)
    sl = torch.from_numpy(sel).to(dev)
    got = g.backward(G, sl, algo=_lib.MAXK_BWD_TILE)
    torch.cuda.synchronize()
    assert g.last_bwd_algo == "tile"
    ref = oracle.np_backward(indptr, idx, vals, grad, sel)
    assert oracle.parity_error(got.cpu().numpy(), ref) < TOL
    # deterministic, and equal (to fp32 order) to the other algorithms
    again = g.backward(G, sl, algo=_lib.MAXK_BWD_TILE)
    assert torch.equal(got, again)
    loc = g.backward(G, sl, algo=_lib.MAXK_BWD_LOCAL)
    assert (got - loc).abs().max().item() <= 1e-4 * max(1.0, loc.abs().max().item())
    if g.tile_plan(k)["part_planes"] == 0:
        # one piece per group: TILE adds each destination's edges in source-row
        # order, one FMA per edge, as LOCAL does -> bit-identical.  With more
        # pieces their partial sums are added at the end instead.
        assert torch.equal(got, loc)


@pytest.mark.gpu
def test_tile_backward_gpu_groups_and_zero_rows(dev, oracle):
    """Several destination groups (> 2048 columns), columns without in-edges,
    rows without out-edges, and G holding inf/NaN only in rows with no edges."""
    import spgemm_new_amd as S
    from spgemm_new_amd import _lib
    V = 5000
    indptr, idx, vals = _graph(V, V, 25, seed=7)
    deg = np.diff(indptr)
    grad, sel = _inputs(V, V, seed=7)
    empty_rows = np.nonzero(deg == 0)[0]
    if empty_rows.size:
        grad[empty_rows[0], :] = np.inf
    g = S.MaxKGraph(torch.from_numpy(indptr).to(dev), torch.from_numpy(idx).to(dev),
                    torch.from_numpy(vals).to(dev))
    got = g.backward(torch.from_numpy(grad).to(dev), torch.from_numpy(sel).to(dev),
                     algo=_lib.MAXK_BWD_TILE).cpu().numpy()
    ref = oracle.np_backward(indptr, idx, vals, grad, sel)
    assert np.isfinite(got).all()
    assert oracle.parity_error(got, ref) < TOL


@pytest.mark.gpu
@pytest.mark.parametrize("k", [32, 64])
def test_tile_one_range_is_sequential_fma(dev, k):
    """With one source range TILE adds each destination's edges in source-row
    order, one fp32 FMA per edge, so every dXs entry equals the host replay
    acc = fma(val, G[row, sel], acc) in CSR order bit for bit (fma emulated as
    the exact fp64 product plus acc, rounded once).  LOCAL matches it at k = 64;
    at k = 32 LOCAL rounds the product before the add in some entries
    (tools/exp_tile_local_bits.py), a last-bit difference."""
    import spgemm_new_amd as S
    from spgemm_new_amd import _lib, ops
    V = 2000
    indptr, idx, vals = _graph(V, V, 30, seed=41)
    grad, sel = _inputs(V, V, seed=41, k=k)
    g = S.MaxKGraph(torch.from_numpy(indptr).to(dev), torch.from_numpy(idx).to(dev),
                    torch.from_numpy(vals).to(dev))
    ng = -(-V // tile.max_group(k))
    plan = tile.build(g.indptr, g.indices, g.values, V, V, shape=(ng, -(-V // ng), 1), k=k)
    plan["values_key"], plan["values_ref"] = ops._tensor_key(g.values), g.values
    plan["part"] = torch.empty(1, device=dev)
    g._tile[k] = plan
    got = g.backward(torch.from_numpy(grad).to(dev), torch.from_numpy(sel).to(dev),
                     algo=_lib.MAXK_BWD_TILE).cpu().numpy()
    rows = np.repeat(np.arange(V), np.diff(indptr))
    acc = np.zeros((V, k), np.float32)
    for e in range(idx.size):          # CSR order = source-row order per destination
        c = idx[e]
        prod = np.float64(vals[e]) * grad[rows[e], sel[c].astype(np.int64)].astype(np.float64)
        acc[c] = (prod + acc[c].astype(np.float64)).astype(np.float32)
    assert np.array_equal(got, acc)


@pytest.mark.gpu
@pytest.mark.parametrize("k", [32, 64])
@pytest.mark.parametrize("V,C,deg,P", [(3000, 3000, 40, 5), (3000, 5000, 30, 7), (2000, 4500, 25, 4),
                                       (1500, 1500, 20, 63)])
def test_tile_backward_straddling_pieces(dev, oracle, V, C, deg, P, k):
    """Workgroup ranges that straddle destination groups (P not a multiple of
    the group count): a workgroup runs two or more pieces, each group's later
    pieces go to partial planes summed per group -- equal to the oracle, and
    bitwise reproducible."""
    import spgemm_new_amd as S
    from spgemm_new_amd import _lib, ops
    indptr, idx, vals = _graph(V, C, deg, seed=V + C + P)
    grad, sel = _inputs(V, C, seed=V + P, k=k)
    g = S.MaxKGraph(torch.from_numpy(indptr).to(dev), torch.from_numpy(idx).to(dev),
                    torch.from_numpy(vals).to(dev), num_cols=C)
    G = -(-C // tile.max_group(k))
    G = max(G, 2)
    plan = tile.build(g.indptr, g.indices, g.values, V, C, shape=(G, -(-C // G), P), k=k)
    assert plan is not None and plan["num_workgroups"] == P
    assert any(len(tile.pieces_of(b, V, G, P)) > 1 for b in range(P))
    plan["values_key"], plan["values_ref"] = ops._tensor_key(g.values), g.values
    plan["part"] = torch.empty(max(1, plan["part_planes"] * C * k), device=dev)
    g._tile[k] = plan
    Gt, sl = torch.from_numpy(grad).to(dev), torch.from_numpy(sel).to(dev)
    got = g.backward(Gt, sl, algo=_lib.MAXK_BWD_TILE)
    assert g.last_bwd_algo == "tile"
    ref = oracle.np_backward(indptr, idx, vals, grad, sel)
    assert oracle.parity_error(got.cpu().numpy(), ref) < TOL
    assert torch.equal(got, g.backward(Gt, sl, algo=_lib.MAXK_BWD_TILE))


@pytest.mark.gpu
def test_tile_repeat_calls_with_empty_wave_chunks(dev, oracle):
    """A sparse graph (most wave-chunks hold no records): every step must wait for
    its record loads even when it has nothing to do, or the next step's loads race
    into the same registers (stale records; seen on products k=32).  Ten repeat
    calls must be bit-identical and right."""
    import spgemm_new_amd as S
    from spgemm_new_amd import _lib
    V, C = 20000, 20000
    indptr, idx, vals = _graph(V, C, 3, seed=77)
    grad, sel = _inputs(V, C, seed=78, k=32)
    g = S.MaxKGraph(torch.from_numpy(indptr).to(dev), torch.from_numpy(idx).to(dev),
                    torch.from_numpy(vals).to(dev))
    assert g.tile_plan(32) is not None
    G, sl = torch.from_numpy(grad).to(dev), torch.from_numpy(sel).to(dev)
    first = g.backward(G, sl, algo=_lib.MAXK_BWD_TILE)
    for _ in range(10):
        assert torch.equal(first, g.backward(G, sl, algo=_lib.MAXK_BWD_TILE))
    ref = oracle.np_backward(indptr, idx, vals, grad, sel)
    assert oracle.parity_error(first.cpu().numpy(), ref) < TOL
