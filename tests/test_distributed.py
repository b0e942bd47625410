"""Multi-process (world_size 2 and 3, gloo, CPU) tests of the 1-D row partition
+ all-to-all-v halo exchange (spgemm_new_amd.distributed).  The local compute
is the CPU oracle injected as the engine (test-only), so the partitioning,
renumbering and both exchange directions are checked without a GPU; the GPU
engine is exercised by the -m gpu tests and bench.py --gpus N."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from spgemm_new_amd.graphs import random_cbsr, small_csr


class OracleEngine:
    """Test-only local engine: numpy oracle on a rectangular local block."""

    def __init__(self, indptr, indices, values, num_cols, **_):
        from oracle import oracle as O
        self.O = O
        self.indptr = indptr.numpy()
        self.indices = indices.numpy()
        self.values = values.numpy()
        self.num_cols = num_cols

    def forward(self, data, sel, dim):
        assert data.shape[0] == self.num_cols
        y = self.O.np_forward(self.indptr, self.indices, self.values, data.numpy(), sel.numpy(), dim)
        return torch.from_numpy(y.astype(np.float32))

    def backward(self, grad, sel, values=None):
        assert sel.shape[0] == self.num_cols
        vals = self.values if values is None else values.numpy()
        d = self.O.np_backward(self.indptr, self.indices, vals, grad.numpy(), sel.numpy())
        return torch.from_numpy(d.astype(np.float32))

    def forward_records(self, records, k, dim, out=None, accumulate=False):
        assert records.shape == (self.num_cols, 5 * k) and records.dtype == torch.uint8
        data = records[:, : 4 * k].contiguous().view(torch.float32)
        y = self.forward(data, records[:, 4 * k:].contiguous(), dim)
        if out is None:
            return y
        if accumulate:
            out += y
        else:
            out.copy_(y)
        return out

    def forward_multi(self, data, sel, values, dim):
        ys = []
        for q in range(values.shape[1]):
            y = self.O.np_forward(self.indptr, self.indices, values[:, q].numpy(), data.numpy(),
                                  sel.numpy(), dim)
            ys.append(torch.from_numpy(y.astype(np.float32)))
        return torch.stack(ys)

    def backward_multi(self, grad, sel, values):
        out = None
        for q in range(values.shape[1]):
            d = self.backward(grad[q], sel, values[:, q].contiguous())
            out = d if out is None else out + d
        return out


class RowsOnlyEngine(OracleEngine):
    """An engine without forward_records: the halo rows are unpacked and concatenated."""

    def __getattribute__(self, name):
        if name == "forward_records":
            raise AttributeError(name)
        return object.__getattribute__(self, name)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, overlap=True, engine="records", k=8):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from spgemm_new_amd.distributed import PartitionedMaxK
        indptr, indices = small_csr(900, seed=4)
        v, h = len(indptr) - 1, 64
        values = np.random.default_rng(1).random(len(indices), dtype=np.float32)
        data, sel = random_cbsr(v, k, h, seed=2)
        grad = np.random.default_rng(3).random((v, h), dtype=np.float32)
        eng = OracleEngine if engine == "records" else RowsOnlyEngine
        m = PartitionedMaxK(torch.from_numpy(indptr), torch.from_numpy(indices),
                            torch.from_numpy(values), rank, world, "cpu", engine=eng,
                            overlap=overlap)
        assert m.overlap == (overlap and m.plan.num_halo > 0)
        sel_l = m.local_rows(torch.from_numpy(sel))
        y = m.forward(m.local_rows(torch.from_numpy(data)), sel_l, h)
        hs = m.last_halo_selectors()
        # the forward's selectors are reused; a different tensor is exchanged again
        dx = m.backward(m.local_rows(torch.from_numpy(grad)), sel_l)
        dx2 = m.backward(m.local_rows(torch.from_numpy(grad)), sel_l.clone())
        assert torch.equal(dx, dx2)
        # after another forward (other selectors) the saved halo selectors still
        # give the first forward's backward (what PartitionedSpGEMMFunction does)
        d2, s2 = random_cbsr(v, k, h, seed=9)
        m.forward(m.local_rows(torch.from_numpy(d2)), m.local_rows(torch.from_numpy(s2)), h)
        dx3 = m.backward(m.local_rows(torch.from_numpy(grad)), sel_l, halo_sel=hs)
        assert torch.equal(dx, dx3)
        # gather to rank 0
        ys = [None] * world
        dxs = [None] * world
        dist.all_gather_object(ys, y.numpy())
        dist.all_gather_object(dxs, dx.numpy())
        if rank == 0:
            from oracle import oracle as O
            yr = O.np_forward(indptr, indices, values, data, sel, h)
            dr = O.np_backward(indptr, indices, values, grad, sel)
            ey = O.parity_error(np.concatenate(ys), yr)
            ed = O.parity_error(np.concatenate(dxs), dr)
            q.put((ey, ed, m.plan.num_halo, m.bounds))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,overlap,engine,k", [
    (2, True, "records", 8), (3, True, "records", 8), (2, False, "records", 8),
    (3, False, "records", 8), (2, True, "rows", 8), (3, False, "rows", 8),
    (2, True, "records", 5), (3, False, "records", 5), (8, True, "records", 8)])
def test_partitioned_matches_single(world, overlap, engine, k):
    """overlap=True splits each block into own | halo column parts and runs the
    exchange asynchronously; overlap=False is the single-block path.  The halo
    travels as records read in place ("records"; k = 5 has none and takes the
    rows path) or is unpacked into rows ("rows")."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, overlap, engine, k))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    ey, ed, nh, bounds = q.get(timeout=5)
    assert nh > 0 and bounds[0] == 0 and bounds[-1] == 900
    assert ey <= 1e-5 and ed <= 1e-5, (ey, ed)


def _multi_worker(rank, world, port, q, R):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from spgemm_new_amd.distributed import PartitionedMaxK
        indptr, indices = small_csr(700, seed=9)
        v, h, k = len(indptr) - 1, 64, 16
        values = np.random.default_rng(5).random((len(indices), R), dtype=np.float32)
        data, sel = random_cbsr(v, k, h, seed=6)
        grad = np.random.default_rng(7).random((R, v, h), dtype=np.float32)
        m = PartitionedMaxK(torch.from_numpy(indptr), torch.from_numpy(indices),
                            torch.from_numpy(values), rank, world, "cpu", engine=OracleEngine)
        sel_l = m.local_rows(torch.from_numpy(sel))
        y = m.forward_multi(m.local_rows(torch.from_numpy(data)), sel_l, h)
        r0, r1 = m.bounds[rank], m.bounds[rank + 1]
        dx = m.backward_multi(torch.from_numpy(grad[:, r0:r1]).contiguous(), sel_l)
        ys, dxs = [None] * world, [None] * world
        dist.all_gather_object(ys, y.numpy())
        dist.all_gather_object(dxs, dx.numpy())
        if rank == 0:
            from oracle import oracle as O
            yr = np.stack([O.np_forward(indptr, indices, values[:, j].copy(), data, sel, h)
                           for j in range(R)])
            dr = sum(O.np_backward(indptr, indices, values[:, j].copy(), grad[j], sel)
                     for j in range(R))
            q.put((O.parity_error(np.concatenate(ys, axis=1), yr),
                   O.parity_error(np.concatenate(dxs), dr)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,R", [(2, 8), (3, 3)])
def test_partitioned_multi_relation(world, R):
    """Config 5 on N ranks: one halo exchange shared by R relations, fused local
    forward, composed backward with one reverse exchange."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_multi_worker, args=(r, world, port, q, R)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    ey, ed = q.get(timeout=5)
    assert ey <= 1e-5 and ed <= 1e-5, (ey, ed)


def test_row_partition_balance():
    from spgemm_new_amd.distributed import row_partition
    indptr, _ = small_csr(2000, seed=8)
    t = torch.from_numpy(indptr)
    for world in (1, 2, 4, 8):
        b = row_partition(t, world)
        assert b[0] == 0 and b[-1] == 2000 and all(b[i] <= b[i + 1] for i in range(world))
        cost = [int(indptr[b[i + 1]] - indptr[b[i]]) + 16 * (b[i + 1] - b[i]) for i in range(world)]
        assert max(cost) - min(cost) <= int(np.diff(indptr).max()) + 16 + 1


def _gpu_worker(rank, world, port, q, overlap=True, records=True, R=1):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from spgemm_new_amd.distributed import PartitionedMaxK
        dev = torch.device("cuda:0")
        indptr, indices = small_csr(2500, seed=6)
        v, h, k = len(indptr) - 1, 256, 32
        shape = (len(indices),) if R == 1 else (len(indices), R)
        values = np.random.default_rng(1).random(shape, dtype=np.float32)
        data, sel = random_cbsr(v, k, h, seed=2)
        gshape = (v, h) if R == 1 else (R, v, h)
        grad = np.random.default_rng(3).random(gshape, dtype=np.float32)
        m = PartitionedMaxK(torch.from_numpy(indptr).to(dev), torch.from_numpy(indices).to(dev),
                            torch.from_numpy(values).to(dev), rank, world, dev, panel_cost=256,
                            overlap=overlap, records=records)
        td = lambda a: m.local_rows(torch.from_numpy(a).to(dev))  # noqa: E731
        r0, r1 = m.bounds[rank], m.bounds[rank + 1]
        sel_l = td(sel)
        if R == 1:
            for _ in range(2):   # the second step reuses the exchange buffers
                y = m.forward(td(data), sel_l, h)
                dx = m.backward(td(grad), sel_l)
        else:
            y = m.forward_multi(td(data), sel_l, h)
            dx = m.backward_multi(torch.from_numpy(grad[:, r0:r1]).contiguous().to(dev), sel_l)
        torch.cuda.synchronize()
        ys, dxs = [None] * world, [None] * world
        dist.all_gather_object(ys, y.cpu().numpy())
        dist.all_gather_object(dxs, dx.cpu().numpy())
        if rank == 0:
            from oracle import oracle as O
            if R == 1:
                yr = O.np_forward(indptr, indices, values, data, sel, h)
                dr = O.np_backward(indptr, indices, values, grad, sel)
                ey = O.parity_error(np.concatenate(ys), yr)
            else:
                yr = np.stack([O.np_forward(indptr, indices, values[:, j].copy(), data, sel, h)
                               for j in range(R)])
                dr = sum(O.np_backward(indptr, indices, values[:, j].copy(), grad[j], sel)
                         for j in range(R))
                ey = O.parity_error(np.concatenate(ys, axis=1), yr)
            ed = O.parity_error(np.concatenate(dxs), dr)
            q.put((ey, ed))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("overlap,records,R", [(True, True, 1), (False, True, 1),
                                               (True, False, 1), (False, False, 1),
                                               (True, True, 8)])
def test_partitioned_hip_engine_two_ranks_one_gpu(overlap, records, R):
    """2 ranks share cuda:0; HIP kernels on rectangular row blocks with halo columns
    (halo records read in place, or unpacked rows; R = 8: the multi-relation path);
    exchange over gloo (staged through host)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, 2, port, q, overlap, records, R))
             for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    ey, ed = q.get(timeout=5)
    assert ey <= 1e-4 and ed <= 1e-4, (ey, ed)


def _autograd_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from spgemm_new_amd.distributed import PartitionedMaxK
        from spgemm_new_amd.models import PartitionedSpGEMMFunction
        dev = torch.device("cuda:0")
        indptr, indices = small_csr(1200, seed=12)
        v, h, k = len(indptr) - 1, 64, 8
        values = np.random.default_rng(2).random(len(indices), dtype=np.float32)
        x = np.random.default_rng(3).random((v, h), dtype=np.float32)
        G = np.random.default_rng(4).random((v, h), dtype=np.float32)
        m = PartitionedMaxK(torch.from_numpy(indptr).to(dev), torch.from_numpy(indices).to(dev),
                            torch.from_numpy(values).to(dev), rank, world, dev, panel_cost=128)
        xo = m.local_rows(torch.from_numpy(x).to(dev)).requires_grad_(True)
        # two layers through one partitioned graph: the second forward reuses the
        # exchange buffers before the first layer's backward runs
        y1 = PartitionedSpGEMMFunction.apply(xo, m, k)
        y2 = PartitionedSpGEMMFunction.apply(0.5 * y1 + xo, m, k)
        (y2 * m.local_rows(torch.from_numpy(G).to(dev))).sum().backward()
        torch.cuda.synchronize()
        ys, gs = [None] * world, [None] * world
        dist.all_gather_object(ys, y2.detach().cpu().numpy())
        dist.all_gather_object(gs, xo.grad.cpu().numpy())
        if rank == 0:
            q.put((np.concatenate(ys), np.concatenate(gs)))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_partitioned_autograd_two_layers():
    """PartitionedSpGEMMFunction (2 ranks on cuda:0, gloo) through two layers
    equals SpGEMMFunction on the whole graph: outputs and input gradients."""
    from spgemm_new_amd.models import SpGEMMFunction
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_autograd_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    # read before joining: rank 0 cannot exit until its (large) result has left the queue
    y_part, g_part = q.get(timeout=300)
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    dev = torch.device("cuda:0")
    indptr, indices = small_csr(1200, seed=12)
    v, h, k = len(indptr) - 1, 64, 8
    values = np.random.default_rng(2).random(len(indices), dtype=np.float32)
    x = torch.from_numpy(np.random.default_rng(3).random((v, h), dtype=np.float32)).to(dev)
    G = torch.from_numpy(np.random.default_rng(4).random((v, h), dtype=np.float32)).to(dev)
    graph = tuple(torch.from_numpy(a).to(dev) for a in (indptr, indices, values))
    xg = x.clone().requires_grad_(True)
    y2 = SpGEMMFunction.apply(0.5 * SpGEMMFunction.apply(xg, graph, k) + xg, graph, k)
    (y2 * G).sum().backward()
    ey = np.abs(y_part - y2.detach().cpu().numpy()) / np.maximum(1, np.abs(y2.detach().cpu().numpy()))
    eg = np.abs(g_part - xg.grad.cpu().numpy()) / np.maximum(1, np.abs(xg.grad.cpu().numpy()))
    assert ey.max() <= 1e-4 and eg.max() <= 1e-4, (ey.max(), eg.max())


def _local_block_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from spgemm_new_amd.distributed import PartitionedMaxK, row_partition
        from spgemm_new_amd.graphs import synthetic_columns, synthetic_indptr, synthetic_values
        V, E, h, k = 1500, 40000, 64, 8
        indptr = synthetic_indptr(V, E, seed=7, device="cpu")
        b = row_partition(indptr, world)
        r0, r1 = b[rank], b[rank + 1]
        e0, e1 = int(indptr[r0]), int(indptr[r1])
        # this rank generates only its rows (and their edge values)
        cols = synthetic_columns(indptr, seed=7, rows=(r0, r1))
        vals = synthetic_values(7, e0, e1, device="cpu")
        m = PartitionedMaxK(indptr, cols, vals, rank, world, "cpu", engine=OracleEngine,
                            local_block=True)
        m_sync = PartitionedMaxK(indptr, cols, vals, rank, world, "cpu", engine=OracleEngine,
                                 local_block=True, overlap_backward=False)
        assert m.overlap_backward and not m_sync.overlap_backward
        data, sel = random_cbsr(V, k, h, seed=3)
        grad = np.random.default_rng(4).random((V, h), dtype=np.float32)
        sel_l = m.local_rows(torch.from_numpy(sel))
        d_l, g_l = m.local_rows(torch.from_numpy(data)), m.local_rows(torch.from_numpy(grad))
        y = m.forward(d_l, sel_l, h)
        dx = m.backward(g_l, sel_l)
        m_sync.forward(d_l, sel_l, h)
        assert torch.equal(dx, m_sync.backward(g_l, sel_l))   # overlap changes no sum order
        ys, dxs = [None] * world, [None] * world
        dist.all_gather_object(ys, y.numpy())
        dist.all_gather_object(dxs, dx.numpy())
        if rank == 0:
            from oracle import oracle as O
            from spgemm_new_amd.graphs import synthetic_csr_gpu
            ip, ix = synthetic_csr_gpu(V, E, seed=7, device="cpu")   # the whole graph, once
            vv = synthetic_values(7, 0, E, device="cpu").numpy()
            ipn, ixn = ip.numpy(), ix.numpy()
            q.put((O.parity_error(np.concatenate(ys), O.np_forward(ipn, ixn, vv, data, sel, h)),
                   O.parity_error(np.concatenate(dxs), O.np_backward(ipn, ixn, vv, grad, sel))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_partitioned_local_block_generation(world):
    """Each rank generates only its own rows of the synthetic graph
    (synthetic_columns / synthetic_values by row range, local_block=True) and
    the partitioned forward / backward -- with and without the overlapped
    reverse exchange -- equal the oracle on the whole graph."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_local_block_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    ey, ed = q.get(timeout=5)
    assert ey <= 1e-5 and ed <= 1e-5, (ey, ed)


def test_synthetic_row_range_equals_whole_graph():
    """synthetic_columns over a row range == the same rows of the whole graph
    (columns distinct and ascending per row), self loops included."""
    from spgemm_new_amd.graphs import synthetic_columns, synthetic_csr_gpu, synthetic_values
    ip, ix = synthetic_csr_gpu(3000, 90000, seed=5, device="cpu", self_loops=True)
    for r0, r1 in ((0, 1), (17, 1234), (2999, 3000), (0, 3000)):
        e0, e1 = int(ip[r0]), int(ip[r1])
        assert torch.equal(synthetic_columns(ip, 5, rows=(r0, r1), self_loops=True), ix[e0:e1])
    ipn, ixn = ip.numpy(), ix.numpy()
    for r in range(3000):
        seg = ixn[ipn[r]:ipn[r + 1]]
        assert np.all(np.diff(seg) > 0) and (seg.size == 0 or r in seg)
    assert torch.equal(synthetic_values(5, 100, 200, "cpu"), synthetic_values(5, 0, 300, "cpu")[100:200])


def _fullsize_worker(rank, world, port, q, graph, R):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from spgemm_new_amd.distributed import PartitionedMaxK, row_partition
        from spgemm_new_amd.graphs import (CONFIGS, synthetic_columns, synthetic_indptr,
                                           synthetic_values)
        from spgemm_new_amd.ops import topk_cbsr
        dev = torch.device("cuda:0")
        V, E = CONFIGS[graph]
        h, k = 256, 32
        indptr = synthetic_indptr(V, E, device=dev)
        b = row_partition(indptr, world)
        r0, r1 = b[rank], b[rank + 1]
        e0, e1 = int(indptr[r0]), int(indptr[r1])
        cols = synthetic_columns(indptr, rows=(r0, r1))          # this rank's rows only
        if R == 1:
            vals = synthetic_values(123, e0, e1, device=dev)
        else:
            vals = torch.stack([synthetic_values(130 + q, e0, e1, device=dev) for q in range(R)],
                               1).contiguous()
        m = PartitionedMaxK(indptr, cols, vals, rank, world, dev, local_block=True)
        gen = torch.Generator(device=dev)
        gen.manual_seed(7 + rank)
        x = torch.rand((r1 - r0, h), generator=gen, device=dev)
        data, sel = topk_cbsr(x, k)
        if R == 1:
            G = torch.rand((r1 - r0, h), generator=gen, device=dev)
            y = m.forward(data, sel, h)
            dx = m.backward(G, sel)
        else:
            G = torch.rand((R, r1 - r0, h), generator=gen, device=dev)
            y = m.forward_multi(data, sel, h)
            dx = m.backward_multi(G, sel)
        # adjoint identity over the whole graph: sum_ranks <Y_own, G_own> = sum_ranks <X^_own, dXs_own>
        s = torch.tensor([float((y.double() * G.double()).sum()),
                          float((data.double() * dx.double()).sum()),
                          float(m.plan.num_halo)], dtype=torch.float64)
        dist.all_reduce(s)
        if rank == 0:
            q.put(s.tolist())
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("graph,R", [("products", 1), ("proteins", 8)])
def test_partitioned_full_size_two_ranks_one_gpu(graph, R):
    """BASELINE config 4 (ogbn-products row-partitioned) and config 5 (proteins,
    8 relations) at full size, 2 ranks sharing cuda:0 (gloo stands in for RCCL):
    each rank generates only its block, the halo exchange runs both ways, and
    the whole-graph adjoint identity holds to 1e-6."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fullsize_worker, args=(r, 2, port, q, graph, R))
             for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=600)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    lhs, rhs, halo = q.get(timeout=5)
    assert halo > 0
    assert abs(lhs - rhs) / abs(lhs) <= 1e-6, (lhs, rhs)


def _allgather_worker(rank, world, port, q, k):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from spgemm_new_amd.distributed import PartitionedMaxK
        indptr, indices = small_csr(900, seed=4)
        v, h = len(indptr) - 1, 64
        values = np.random.default_rng(1).random(len(indices), dtype=np.float32)
        data, sel = random_cbsr(v, k, h, seed=2)
        grad = np.random.default_rng(3).random((v, h), dtype=np.float32)
        args = (torch.from_numpy(indptr), torch.from_numpy(indices), torch.from_numpy(values),
                rank, world, "cpu")
        m_rec = PartitionedMaxK(*args, engine=OracleEngine, halo_mode="records")
        m_ag = PartitionedMaxK(*args, engine=OracleEngine, halo_mode="allgather")
        m_auto = PartitionedMaxK(*args, engine=OracleEngine)
        # overlap="auto": a few KB of halo records -> single block; threshold 0 -> split
        import spgemm_new_amd.distributed as Dm
        m_ov_auto = PartitionedMaxK(*args, engine=OracleEngine, overlap="auto")
        saved = Dm.OVERLAP_MIN_HALO_BYTES
        Dm.OVERLAP_MIN_HALO_BYTES = 0
        try:
            m_ov_zero = PartitionedMaxK(*args, engine=OracleEngine, overlap="auto")
        finally:
            Dm.OVERLAP_MIN_HALO_BYTES = saved
        assert m_ov_auto.overlap is False and m_ov_zero.overlap is True
        d_l, s_l = m_rec.local_rows(torch.from_numpy(data)), m_rec.local_rows(torch.from_numpy(sel))
        g_l = m_rec.local_rows(torch.from_numpy(grad))
        y_r, y_a = m_rec.forward(d_l, s_l, h), m_ag.forward(d_l, s_l, h)
        dx_r, dx_a = m_rec.backward(g_l, s_l), m_ag.backward(g_l, s_l)
        same = torch.equal(y_r, y_a) and torch.equal(dx_r, dx_a) and \
            torch.equal(m_rec.last_halo_selectors(), m_ag.last_halo_selectors())
        ys, dxs = [None] * world, [None] * world
        dist.all_gather_object(ys, y_a.numpy())
        dist.all_gather_object(dxs, dx_a.numpy())
        flags = [None] * world
        dist.all_gather_object(flags, (same, m_auto.halo_mode, m_ag.halo_bytes(k)))
        if rank == 0:
            from oracle import oracle as O
            ey = O.parity_error(np.concatenate(ys), O.np_forward(indptr, indices, values, data, sel, h))
            ed = O.parity_error(np.concatenate(dxs),
                                O.np_backward(indptr, indices, values, grad, sel))
            q.put((ey, ed, flags))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_allgather_halo_mode_bitwise_equals_records(world):
    """SURVEY.md §8e's all-gather fallback: the forward all-gathers the whole CBSR
    (records) instead of the halo all-to-all-v and the halo part reads it in
    place -- Y, dXs and the saved halo selectors bitwise equal to the records
    path, and both equal the oracle; "auto" picks it when a halo covers more
    than 75 % of V, the same choice on every rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    k = 8
    procs = [ctx.Process(target=_allgather_worker, args=(r, world, port, q, k))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    ey, ed, flags = q.get(timeout=5)
    assert ey <= 1e-4 and ed <= 1e-4
    assert all(f[0] for f in flags), flags
    assert len({f[1] for f in flags}) == 1          # one collective on every rank
    for same, mode, nbytes in flags:
        assert nbytes["allgather_fwd"] >= nbytes["records_fwd"] > 0


def _mixed_worker(rank, world, port, q, isolated):
    """Ranks with different halo sizes (and, with `isolated`, rank 0 without any
    halo) under overlap="auto" + halo_mode "allgather"/"auto": the choices must be
    the same on every rank, the collectives must match (no hang) and the result
    must equal the oracle."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import spgemm_new_amd.distributed as Dm
        from spgemm_new_amd.distributed import PartitionedMaxK, row_partition
        indptr, indices = small_csr(900, seed=4)
        v, h, k = len(indptr) - 1, 64, 8
        if isolated:
            # rank 0's rows reference only rank 0's own columns: its halo is empty
            b = row_partition(torch.from_numpy(indptr), world)
            rng = np.random.default_rng(11)
            indices = indices.copy()
            for r in range(b[0], b[1]):
                e0, e1 = indptr[r], indptr[r + 1]
                indices[e0:e1] = np.sort(rng.integers(b[0], b[1], e1 - e0))
        values = np.random.default_rng(1).random(len(indices), dtype=np.float32)
        data, sel = random_cbsr(v, k, h, seed=2)
        grad = np.random.default_rng(3).random((v, h), dtype=np.float32)
        args = (torch.from_numpy(indptr), torch.from_numpy(indices), torch.from_numpy(values),
                rank, world, "cpu")
        probe = PartitionedMaxK(*args, engine=OracleEngine, overlap=False, halo_mode="records")
        halos = [None] * world
        dist.all_gather_object(halos, probe.plan.num_halo)
        saved = Dm.OVERLAP_MIN_HALO_BYTES
        # between the smallest and the largest rank's halo records
        Dm.OVERLAP_MIN_HALO_BYTES = (min(halos) + max(halos)) // 2 * Dm.OVERLAP_BYTES_PER_HALO_NODE
        try:
            res = []
            for mode in ("allgather", "auto"):
                m = PartitionedMaxK(*args, engine=OracleEngine, overlap="auto", halo_mode=mode)
                d_l = m.local_rows(torch.from_numpy(data))
                s_l = m.local_rows(torch.from_numpy(sel))
                y = m.forward(d_l, s_l, h)
                dx = m.backward(m.local_rows(torch.from_numpy(grad)), s_l)
                res.append((y.numpy(), dx.numpy(), m.overlap, m.halo_mode, m.plan.num_halo))
        finally:
            Dm.OVERLAP_MIN_HALO_BYTES = saved
        allres = [None] * world
        dist.all_gather_object(allres, res)
        if rank == 0:
            from oracle import oracle as O
            yr = O.np_forward(indptr, indices, values, data, sel, h)
            dr = O.np_backward(indptr, indices, values, grad, sel)
            errs = []
            for i in range(2):
                errs.append((O.parity_error(np.concatenate([a[i][0] for a in allres]), yr),
                             O.parity_error(np.concatenate([a[i][1] for a in allres]), dr)))
            q.put((errs, [[(r[2], r[3], r[4]) for r in a] for a in allres], halos))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,isolated", [(3, False), (3, True), (4, True)])
def test_overlap_and_halo_mode_decided_collectively(world, isolated):
    """OVERLAP_MIN_HALO_BYTES between two ranks' halo sizes, halo_mode "allgather"
    and "auto": every rank takes the same split decision (on the largest halo)
    and the same collective; a rank with no halo at all (isolated) cannot be
    split, so the all-gather mode falls back to records on every rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mixed_worker, args=(r, world, port, q, isolated))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    errs, flags, halos = q.get(timeout=5)
    assert all(ey <= 1e-4 and ed <= 1e-4 for ey, ed in errs), errs
    if isolated:
        assert halos[0] == 0 and max(halos) > 0
    else:
        assert min(halos) < max(halos)
    for i in range(2):
        modes = {r[i][1] for r in flags}
        assert len(modes) == 1, flags              # one collective on every rank
        # the split decision is the same wherever a rank has a halo to split off
        assert len({r[i][0] for r in flags if r[i][2] > 0}) == 1, flags
        if isolated:
            assert modes == {"records"}, flags
    if not isolated:
        assert flags[0][0][1] == "allgather"


@pytest.mark.gpu
@pytest.mark.parametrize("k", [4, 8, 16, 32, 64])
def test_records_sel_gather(k):
    """maxk_records_sel_gather (the all-gather halo mode's selector gather) equals
    the selector rows of the records it reads."""
    from spgemm_new_amd import _lib
    from spgemm_new_amd.ops import cbsr_gather_records
    dev = torch.device("cuda:0")
    n_rows = 3001
    data = torch.rand((n_rows, k), device=dev)
    sel = torch.randint(0, 256, (n_rows, k), dtype=torch.uint8, device=dev)
    rec = cbsr_gather_records(data, sel)
    rows = torch.randint(0, n_rows, (777,), dtype=torch.int32, device=dev)
    out = torch.empty((777, k), dtype=torch.uint8, device=dev)
    _lib.check(_lib.load().maxk_records_sel_gather(rec.data_ptr(), k, rows.data_ptr(), 777,
                                                    out.data_ptr(), _lib.stream_ptr(dev)),
               "maxk_records_sel_gather")
    assert torch.equal(out, sel[rows.long()])


# Seeded random configurations of the row-partitioned HIP path (ranks share
# cuda:0, gloo exchange): world, k, overlap, halo mode, relations, panel cost.
_SWEEP = [dict(world=2, k=8, overlap=True, halo="records", R=1, pc=128, seed=31),
          dict(world=3, k=16, overlap=True, halo="allgather", R=1, pc=64, seed=32),
          dict(world=2, k=64, overlap=False, halo="records", R=1, pc=256, seed=33),
          dict(world=3, k=32, overlap=True, halo="allgather", R=4, pc=256, seed=34),
          dict(world=2, k=16, overlap=True, halo="auto", R=8, pc=512, seed=35),
          dict(world=3, k=64, overlap=True, halo="records", R=1, pc=32, seed=36)]


def _sweep_worker(rank, world, port, q, cfg):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from spgemm_new_amd.distributed import PartitionedMaxK
        dev = torch.device("cuda:0")
        rng = np.random.default_rng(cfg["seed"])
        indptr, indices = small_csr(int(rng.integers(600, 1600)), seed=cfg["seed"])
        v, k, R = len(indptr) - 1, cfg["k"], cfg["R"]
        h = 256 if rng.random() < 0.5 else int(rng.choice([64, 128]))
        h = max(h, k)
        shape = (len(indices),) if R == 1 else (len(indices), R)
        values = rng.standard_normal(shape).astype(np.float32)
        data, sel = random_cbsr(v, k, h, seed=cfg["seed"] + 1)
        gshape = (v, h) if R == 1 else (R, v, h)
        grad = rng.standard_normal(gshape).astype(np.float32)
        m = PartitionedMaxK(torch.from_numpy(indptr).to(dev), torch.from_numpy(indices).to(dev),
                            torch.from_numpy(values).to(dev), rank, world, dev,
                            panel_cost=cfg["pc"], overlap=cfg["overlap"], halo_mode=cfg["halo"])
        td = lambda a: m.local_rows(torch.from_numpy(a).to(dev))  # noqa: E731
        r0, r1 = m.bounds[rank], m.bounds[rank + 1]
        sel_l = td(sel)
        if R == 1:
            for _ in range(2):   # the second step reuses the exchange buffers
                y = m.forward(td(data), sel_l, h)
                dx = m.backward(td(grad), sel_l)
        else:
            y = m.forward_multi(td(data), sel_l, h)
            dx = m.backward_multi(torch.from_numpy(grad[:, r0:r1]).contiguous().to(dev), sel_l)
        torch.cuda.synchronize()
        ys, dxs = [None] * world, [None] * world
        dist.all_gather_object(ys, y.cpu().numpy())
        dist.all_gather_object(dxs, dx.cpu().numpy())
        if rank == 0:
            from oracle import oracle as O
            if R == 1:
                yr = O.np_forward(indptr, indices, values, data, sel, h)
                dr = O.np_backward(indptr, indices, values, grad, sel)
                ey = O.parity_error(np.concatenate(ys), yr)
            else:
                yr = np.stack([O.np_forward(indptr, indices, values[:, j].copy(), data, sel, h)
                               for j in range(R)])
                dr = sum(O.np_backward(indptr, indices, values[:, j].copy(), grad[j], sel)
                         for j in range(R))
                ey = O.parity_error(np.concatenate(ys, axis=1), yr)
            ed = O.parity_error(np.concatenate(dxs), dr)
            q.put((ey, ed, m.halo_mode, m.overlap))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", _SWEEP, ids=[f"N{c['world']}-k{c['k']}-{c['halo']}-R{c['R']}"
                                             for c in _SWEEP])
def test_partitioned_hip_engine_sweep(cfg):
    """The row-partitioned HIP path on seeded random graphs: world 2 / 3, k 8 to 64,
    signed values, overlap on / off, records and all-gather halo modes, single and
    multi-relation (R = 4, 8), narrow h; every rank's rows of Y and dXs gathered and
    checked per element against the fp64 oracle of the whole graph."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = cfg["world"]
    procs = [ctx.Process(target=_sweep_worker, args=(r, world, port, q, cfg)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    ey, ed, mode, overlap = q.get(timeout=5)
    if cfg["halo"] == "allgather" and cfg["overlap"]:
        assert mode == "allgather"
    assert ey <= 1e-4 and ed <= 1e-4, (ey, ed, mode, overlap)


def _tiny_worker(rank, world, port, q, V, overlap):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from spgemm_new_amd.distributed import PartitionedMaxK
        dev = torch.device("cuda:0")
        rng = np.random.default_rng(5)
        deg = rng.integers(0, V + 1, V)
        deg[0] = V                                   # one full row
        indptr = np.zeros(V + 1, np.int64)
        indptr[1:] = np.cumsum(deg)
        indices = np.concatenate([np.sort(rng.choice(V, d, replace=False)) for d in deg]
                                 ).astype(np.int32)
        values = rng.random(len(indices)).astype(np.float32)
        k, h = 8, 64
        data, sel = random_cbsr(V, k, h, seed=2)
        grad = rng.random((V, h)).astype(np.float32)
        m = PartitionedMaxK(torch.from_numpy(indptr.astype(np.int32)).to(dev),
                            torch.from_numpy(indices).to(dev), torch.from_numpy(values).to(dev),
                            rank, world, dev, overlap=overlap)
        td = lambda a: m.local_rows(torch.from_numpy(a).to(dev))  # noqa: E731
        sel_l = td(sel)
        y = m.forward(td(data), sel_l, h)
        dx = m.backward(td(grad), sel_l)
        torch.cuda.synchronize()
        ys, dxs = [None] * world, [None] * world
        dist.all_gather_object(ys, y.cpu().numpy())
        dist.all_gather_object(dxs, dx.cpu().numpy())
        if rank == 0:
            from oracle import oracle as O
            ip = indptr.astype(np.int32)
            ey = O.parity_error(np.concatenate(ys), O.np_forward(ip, indices, values, data, sel, h))
            ed = O.parity_error(np.concatenate(dxs), O.np_backward(ip, indices, values, grad, sel))
            q.put((ey, ed, m.bounds))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("V,world,overlap", [(3, 4, True), (3, 4, False), (1, 2, True)])
def test_partitioned_hip_engine_empty_ranks(V, world, overlap):
    """More ranks than rows: some ranks own no row (an empty block on the HIP
    engine, still taking part in every collective)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tiny_worker, args=(r, world, port, q, V, overlap))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    ey, ed, bounds = q.get(timeout=5)
    assert bounds[-1] == V and any(bounds[i] == bounds[i + 1] for i in range(world))
    assert ey <= 1e-4 and ed <= 1e-4, (ey, ed)


def _rounds_worker(rank, world, port, q, halo_mode, k):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from spgemm_new_amd.distributed import PartitionedMaxK
        indptr, indices = small_csr(1100, seed=6)
        v, h = len(indptr) - 1, 64
        rng = np.random.default_rng(4)
        values = rng.standard_normal(len(indices)).astype(np.float32)
        data, sel = random_cbsr(v, k, h, seed=5)
        grad = rng.standard_normal((v, h)).astype(np.float32)
        res = {}
        for R in (1, 2, 3):
            m = PartitionedMaxK(torch.from_numpy(indptr), torch.from_numpy(indices),
                                torch.from_numpy(values), rank, world, "cpu", engine=OracleEngine,
                                overlap=True, halo_mode=halo_mode, rounds=R)
            assert m.rounds == R and (R == 1 or len(m.halo_rounds) == R)
            tab = m._round_tab
            assert tab[0][0] == 0 and tab[-1][1] == m.plan.num_halo
            assert tab[-1][4] == sum(m.plan.send_counts)
            sel_l = m.local_rows(torch.from_numpy(sel))
            y = m.forward(m.local_rows(torch.from_numpy(data)), sel_l, h)
            dx = m.backward(m.local_rows(torch.from_numpy(grad)), sel_l)
            # a selector tensor other than the forward's goes through the round exchange
            dx2 = m.backward(m.local_rows(torch.from_numpy(grad)), sel_l.clone())
            assert torch.equal(dx, dx2)
            res[R] = (y.numpy(), dx.numpy(), m.halo_mode)
        for R in (2, 3):
            # backward: the same column sums, returns added in peer order -> bitwise
            assert np.array_equal(res[R][1], res[1][1]), R
            assert np.max(np.abs(res[R][0] - res[1][0]) / np.maximum(1, np.abs(res[1][0]))) <= 1e-5
        ys, dxs = [None] * world, [None] * world
        dist.all_gather_object(ys, res[3][0])
        dist.all_gather_object(dxs, res[3][1])
        if rank == 0:
            from oracle import oracle as O
            ey = O.parity_error(np.concatenate(ys), O.np_forward(indptr, indices, values, data, sel, h))
            ed = O.parity_error(np.concatenate(dxs), O.np_backward(indptr, indices, values, grad, sel))
            q.put((ey, ed, res[3][2]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,halo_mode,k", [(2, "records", 8), (3, "records", 16),
                                               (3, "allgather", 8), (8, "records", 8),
                                               (8, "allgather", 32)])
def test_round_pipelined_exchange(world, halo_mode, k):
    """rounds = 2 / 3: the halo numbered round-major, every
    exchange in R all-to-all-v rounds, the records forward and the overlapped
    backward one engine per round: dXs bitwise the rounds = 1 result, Y within
    fp32 regrouping (1e-5), both against the fp64 oracle of the whole graph."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rounds_worker, args=(r, world, port, q, halo_mode, k))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    ey, ed, mode = q.get(timeout=5)
    assert mode == halo_mode
    assert ey <= 1e-4 and ed <= 1e-4, (ey, ed)


class _FakePlan:
    """The fields of HaloPlan that _round_major reads and rewrites."""

    def __init__(self, rng, world, num_own):
        self.num_own = num_own
        self.recv_counts = [int(x) for x in rng.integers(0, 40, size=world)]
        self.send_counts = [int(x) for x in rng.integers(0, 40, size=world)]
        self.num_halo = sum(self.recv_counts)
        self.halo_global = torch.arange(self.num_halo, dtype=torch.int64) * 7 + 1000
        n_send = sum(self.send_counts)
        self.send_local = torch.from_numpy(rng.integers(0, num_own, size=n_send)).long()
        cols = rng.integers(0, num_own + self.num_halo, size=500)
        self.local_indices = torch.from_numpy(cols).to(torch.int32)


@pytest.mark.parametrize("world,R", [(2, 2), (3, 3), (8, 2), (5, 4), (4, 1)])
def test_round_major_renumbering(world, R):
    """_round_major: round j carries the j-th equal-count slice
    of every peer's rows, in peer order; the halo renumbering is a permutation that
    keeps every edge on the same global node; the send list is the same multiset in
    the round-major order; the round table tiles both sides exactly."""
    from spgemm_new_amd.distributed import PartitionedMaxK
    rng = np.random.default_rng(world * 10 + R)
    p = _FakePlan(rng, world, num_own=60)
    old_global, old_send = p.halo_global.clone(), p.send_local.clone()
    old_li = p.local_indices.clone().long()
    self = PartitionedMaxK.__new__(PartitionedMaxK)
    self.world, self.device = world, torch.device("cpu")
    tab = self._round_major(p, R)
    assert len(tab) == R and tab[0][0] == 0 and tab[0][3] == 0
    assert tab[-1][1] == p.num_halo and tab[-1][4] == sum(p.send_counts)
    for j in range(1, R):
        assert tab[j][0] == tab[j - 1][1] and tab[j][3] == tab[j - 1][4]
    roff = np.concatenate([[0], np.cumsum(p.recv_counts)])
    soff = np.concatenate([[0], np.cumsum(p.send_counts)])
    pos_r = pos_s = 0
    for j, (r0, r1, rc, s0, s1, sc) in enumerate(tab):
        assert r1 - r0 == sum(rc) and s1 - s0 == sum(sc)
        for q in range(world):
            a, b = p.recv_counts[q] * j // R, p.recv_counts[q] * (j + 1) // R
            assert rc[q] == b - a
            assert torch.equal(p.halo_global[pos_r:pos_r + rc[q]], old_global[roff[q] + a:roff[q] + b])
            pos_r += rc[q]
            a, b = p.send_counts[q] * j // R, p.send_counts[q] * (j + 1) // R
            assert sc[q] == b - a
            assert torch.equal(p.send_local[pos_s:pos_s + sc[q]], old_send[soff[q] + a:soff[q] + b])
            assert bool((self._send_peer[pos_s:pos_s + sc[q]] == q).all())
            pos_s += sc[q]
    # every edge still points at the same global node
    li = p.local_indices.long()
    own = li < p.num_own
    assert torch.equal(li[own], old_li[own])
    assert torch.equal(p.halo_global[li[~own] - p.num_own], old_global[old_li[~own] - p.num_own])
