"""The row-partitioned HIP path pinned against the unpartitioned one at the
BASELINE shapes and rank counts.

BASELINE config 4 (ogbn-products-shaped, k = 32) at world 2, 4 and 8 and
config 5 (ogbn-proteins-shaped, R = 8 relations) at world 8, every rank on
cuda:0 (world 2 / 4: gloo stands in for RCCL, the exchange staged through host
memory; world 8: the ranks are threads of one process and tools/wire_model.py's
ThreadFabric exchanges their tensors on side streams).
The parent process generates the graph's CSR once (power-law indptr and
columns take many synchronising passes, and N processes time-share the one
card) and each rank maps only its rows' slice of it; edge values, features and
gradient rows are hashes of global ids (graphs.synthetic_*) that a rank
generates for its own rows.  Every rank runs forward + backward through
PartitionedMaxK, and its own rows of Y and dXs are compared per element with a
single MaxKGraph over the whole graph (per row: spmm_maxk.cu:17-106 and
spmm_maxk_backward.cu:15-115 semantics), within 1e-4 relative.  A consistent
halo-renumbering error (a permuted send list, a wrong owner) changes rows and
fails here, which the adjoint identity alone could not see.  Also checked:
with the local backward pinned to TILE with one source range (per destination
one sequential FMA chain over its in-edges in source-row order, whatever other
columns the block holds), dXs with the overlapped backward (own / halo parts)
is bitwise the single block's.  (The defaults are not bitwise across blocks:
STAGED's merge-path panels split destinations at places that depend on the
block's other columns, LOCAL rounds some products in its tail rounds, TILE's
source-range count follows the block's column count.)"""
import multiprocessing as mp
import os
import socket

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOL = 1e-4
H, K, SEED = 256, 32, 123
SEED_X, SEED_G = 1001, 2002


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _values(R, e0, e1, dev):
    from spgemm_new_amd.graphs import synthetic_values
    if R == 1:
        return synthetic_values(SEED, e0, e1, device=dev)
    return torch.stack([synthetic_values(SEED + 7 + q, e0, e1, device=dev) for q in range(R)],
                       1).contiguous()


def _grad(R, r0, r1, dev):
    from spgemm_new_amd.graphs import synthetic_features
    if R == 1:
        return synthetic_features(SEED_G, r0, r1, H, dev)
    return torch.stack([synthetic_features(SEED_G + q, r0, r1, H, dev) for q in range(R)])


def _worker(rank, world, port, graph, R, graphdir, outdir, q, rounds=1):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    # up to 8 ranks share the box's CPU share: keep each one's host thread pool small
    torch.set_num_threads(2)
    import faulthandler
    faulthandler.dump_traceback_later(45, repeat=True)   # where a slow rank is, every 45 s
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from spgemm_new_amd import _lib
        from spgemm_new_amd.distributed import PartitionedMaxK, row_partition
        from spgemm_new_amd.graphs import synthetic_features
        from spgemm_new_amd.ops import topk_cbsr
        import numpy as np
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        log = lambda msg: print(f"[pin {graph} N={world} rank {rank}] {msg}", flush=True)
        indptr = torch.from_numpy(np.load(os.path.join(graphdir, "indptr.npy"))).to(dev)
        b = row_partition(indptr, world)
        r0, r1 = b[rank], b[rank + 1]
        e0, e1 = int(indptr[r0]), int(indptr[r1])
        log(f"rows [{r0}, {r1}) edges [{e0}, {e1})")
        cols_all = np.load(os.path.join(graphdir, "indices.npy"), mmap_mode="r")
        cols = torch.from_numpy(np.ascontiguousarray(cols_all[e0:e1])).to(dev)
        vals = _values(R, e0, e1, dev)
        data, sel = topk_cbsr(synthetic_features(SEED_X, r0, r1, H, dev), K)
        G = _grad(R, r0, r1, dev)
        tile = _lib.MAXK_BWD_TILE
        log("block generated")
        kw = {"rounds": rounds} if R > 1 else {"bwd_algo": tile, "tile_splits": 1,
                                               "rounds": rounds}
        m = PartitionedMaxK(indptr, cols, vals, rank, world, dev, local_block=True, **kw)
        log(f"partition built (halo {m.plan.num_halo}, mode {m.halo_mode}, rounds {m.rounds})")
        assert m.rounds == rounds
        if R == 1:
            y = m.forward(data, sel, H)
            dx = m.backward(G, sel)
            assert m.overlap_backward
            # the single-block backward (no own / halo split), same local algorithm
            m1 = PartitionedMaxK(indptr, cols, vals, rank, world, dev, local_block=True,
                                 overlap=False, **kw)
            y1 = m1.forward(data, sel, H)
            dx1 = m1.backward(G, sel)
            bitwise = bool(torch.equal(dx, dx1))
            fwd_split = float(((y - y1).abs() / y1.abs().clamp_min(1)).max())
        else:
            y = m.forward_multi(data, sel, H)
            dx = m.backward_multi(G, sel)
            bitwise, fwd_split = True, 0.0
        torch.cuda.synchronize()
        log("forward + backward done")
        torch.save({"r0": r0, "r1": r1, "y": y.cpu(), "dx": dx.cpu(), "halo": m.plan.num_halo},
                   os.path.join(outdir, f"rank{rank}.pt"))
        flags = torch.tensor([float(not bitwise), fwd_split])
        dist.all_reduce(flags, op=dist.ReduceOp.MAX)
        if rank == 0:
            q.put(flags.tolist())
    finally:
        dist.destroy_process_group()


_REF = {}


def _reference(graph, R, graphdir):
    """Y and dXs of the whole graph on one GPU (single MaxKGraph), cached per graph;
    the graph's indptr / indices are written to `graphdir` for the ranks."""
    key = (graph, R)
    if key not in _REF:
        import numpy as np
        import spgemm_new_amd as S
        from spgemm_new_amd import _lib
        from spgemm_new_amd.graphs import (CONFIGS, synthetic_columns, synthetic_features,
                                           synthetic_indptr)
        from spgemm_new_amd.ops import topk_cbsr
        dev = torch.device("cuda", 0)
        V, E = CONFIGS[graph]
        indptr = synthetic_indptr(V, E, seed=SEED, device=dev)
        indices = synthetic_columns(indptr, seed=SEED)
        np.save(os.path.join(graphdir, "indptr.npy"), indptr.cpu().numpy())
        np.save(os.path.join(graphdir, "indices.npy"), indices.cpu().numpy())
        vals = _values(R, 0, E, dev)
        data, sel = topk_cbsr(synthetic_features(SEED_X, 0, V, H, dev), K)
        G = _grad(R, 0, V, dev)
        if R == 1:
            g = S.MaxKGraph(indptr, indices, vals)
            y = g.forward(data, sel, H)
            dx = g.backward(G, sel, algo=_lib.MAXK_BWD_STAGED)
        else:
            g = S.MaxKGraph(indptr, indices, vals[:, 0].contiguous())
            y = g.forward_multi(data, sel, vals, H)
            dx = g.backward_multi(G, sel, vals)
        torch.cuda.synchronize()
        _REF.clear()
        _REF[key] = (y.cpu(), dx.cpu(), graphdir)
        del g, y, dx, G, data, sel, vals, indices, indptr
        torch.cuda.empty_cache()
    return _REF[key]


def _rel_err(a, b):
    return float(((a - b).abs() / b.abs().clamp_min(1)).max()) if b.numel() else 0.0


def _thread_ranks(graph, world, R, rounds, graphdir):
    """World 8 as threads of this process (tools/wire_model.ThreadFabric: every
    collective a real exchange between the ranks' tensors, delivered on side
    streams with RCCL's ordering): eight processes time-sharing the one card spent
    minutes in context switches at every synchronising step, one process does not.
    Returns per rank (r0, r1, y, dx, halo, bitwise, fwd_split, rounds)."""
    import sys

    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import spgemm_new_amd.distributed as D
    from spgemm_new_amd import _lib
    from spgemm_new_amd.graphs import synthetic_features
    from spgemm_new_amd.ops import topk_cbsr
    from wire_model import ThreadFabric, install
    dev = torch.device("cuda", 0)
    indptr = torch.from_numpy(np.load(os.path.join(graphdir, "indptr.npy"))).to(dev)
    cols_all = np.load(os.path.join(graphdir, "indices.npy"), mmap_mode="r")
    b = D.row_partition(indptr, world)
    fabric = ThreadFabric(world, dev, fixed_us=0.0, timeout_s=600.0)
    restore = install(fabric, D)

    def rank_fn(rank):
        r0, r1 = b[rank], b[rank + 1]
        e0, e1 = int(indptr[r0]), int(indptr[r1])
        cols = torch.from_numpy(np.ascontiguousarray(cols_all[e0:e1])).to(dev)
        vals = _values(R, e0, e1, dev)
        data, sel = topk_cbsr(synthetic_features(SEED_X, r0, r1, H, dev), K)
        G = _grad(R, r0, r1, dev)
        kw = {"rounds": rounds} if R > 1 else {"bwd_algo": _lib.MAXK_BWD_TILE, "tile_splits": 1,
                                               "rounds": rounds}
        m = D.PartitionedMaxK(indptr, cols, vals, rank, world, dev, local_block=True, **kw)
        if R == 1:
            y = m.forward(data, sel, H)
            dx = m.backward(G, sel)
            m1 = D.PartitionedMaxK(indptr, cols, vals, rank, world, dev, local_block=True,
                                   overlap=False, **kw)
            y1 = m1.forward(data, sel, H)
            dx1 = m1.backward(G, sel)
            bitwise = bool(torch.equal(dx, dx1))
            fwd_split = _rel_err(y, y1)
        else:
            y = m.forward_multi(data, sel, H)
            dx = m.backward_multi(G, sel)
            bitwise, fwd_split = True, 0.0
        return r0, r1, y.cpu(), dx.cpu(), m.plan.num_halo, bitwise, fwd_split, m.rounds

    try:
        return fabric.run(rank_fn)
    finally:
        restore()


@pytest.mark.gpu
@pytest.mark.timeout(900)   # up to 8 spawned ranks time-share one card: minutes on a busy box
@pytest.mark.parametrize("graph,world,R,rounds", [("products", 2, 1, 1), ("products", 4, 1, 1),
                                                  ("products", 8, 1, 1), ("proteins", 8, 8, 1),
                                                  ("products", 2, 1, 2), ("products", 8, 1, 2)])
def test_partitioned_rows_match_single_gpu(graph, world, R, rounds, tmp_path, tmp_path_factory):
    """World 2 / 4: one gloo process per rank; world 8: the ranks as threads of
    this process exchanging through tools/wire_model.ThreadFabric.  rounds = 1 and
    the round-pipelined exchange (rounds = 2: products N = 8's default)."""
    y_ref, dx_ref, graphdir = _reference(graph, R, str(tmp_path_factory.mktemp(graph)))
    if world >= 8:
        res = _thread_ranks(graph, world, R, rounds, graphdir)
        assert all(r[7] == rounds for r in res)
        assert all(r[5] for r in res), "overlapped backward differs bitwise from the single block"
        assert max(r[6] for r in res) <= TOL
        rows = 0
        for r0, r1, y, dx, halo, _, _, _ in res:
            rows += r1 - r0
            assert halo > 0
            yr = y_ref[r0:r1] if R == 1 else y_ref[:, r0:r1]
            assert y.shape == yr.shape
            assert _rel_err(y, yr) <= TOL, (r0, _rel_err(y, yr))
            assert _rel_err(dx, dx_ref[r0:r1]) <= TOL, (r0, _rel_err(dx, dx_ref[r0:r1]))
        assert rows == y_ref.shape[-2]
        return
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker,
                         args=(r, world, port, graph, R, graphdir, str(tmp_path), q, rounds))
             for r in range(world)]
    # the children's OpenMP pools, and one hardware queue per rank: N processes time-share
    # the one card, and more queues than the scheduler maps at once stall every sync
    child_env = {"OMP_NUM_THREADS": "2", "GPU_MAX_HW_QUEUES": "1"}
    saved = {k: os.environ.get(k) for k in child_env}
    os.environ.update(child_env)
    try:
        for p in procs:
            p.start()
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    for p in procs:
        p.join(timeout=600)
        if p.exitcode is None:
            p.kill()
            p.join()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    not_bitwise, fwd_split = q.get(timeout=5)
    assert not_bitwise == 0.0, "overlapped backward differs bitwise from the single block"
    assert fwd_split <= TOL
    rows = 0
    for r in range(world):
        part = torch.load(os.path.join(str(tmp_path), f"rank{r}.pt"), weights_only=True)
        r0, r1 = part["r0"], part["r1"]
        rows += r1 - r0
        assert part["halo"] > 0
        yr = y_ref[r0:r1] if R == 1 else y_ref[:, r0:r1]
        assert part["y"].shape == yr.shape
        assert _rel_err(part["y"], yr) <= TOL, (r, _rel_err(part["y"], yr))
        assert _rel_err(part["dx"], dx_ref[r0:r1]) <= TOL, (r, _rel_err(part["dx"], dx_ref[r0:r1]))
    assert rows == y_ref.shape[-2]
