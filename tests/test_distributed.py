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

    def backward(self, grad, sel):
        assert sel.shape[0] == self.num_cols
        d = self.O.np_backward(self.indptr, self.indices, self.values, grad.numpy(), sel.numpy())
        return torch.from_numpy(d.astype(np.float32))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, overlap=True):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from spgemm_new_amd.distributed import PartitionedMaxK
        indptr, indices = small_csr(900, seed=4)
        v, h, k = len(indptr) - 1, 64, 8
        values = np.random.default_rng(1).random(len(indices), dtype=np.float32)
        data, sel = random_cbsr(v, k, h, seed=2)
        grad = np.random.default_rng(3).random((v, h), dtype=np.float32)
        m = PartitionedMaxK(torch.from_numpy(indptr), torch.from_numpy(indices),
                            torch.from_numpy(values), rank, world, "cpu", engine=OracleEngine,
                            overlap=overlap)
        assert m.overlap == (overlap and m.plan.num_halo > 0)
        y = m.forward(m.local_rows(torch.from_numpy(data)), m.local_rows(torch.from_numpy(sel)), h)
        dx = m.backward(m.local_rows(torch.from_numpy(grad)), m.local_rows(torch.from_numpy(sel)))
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


@pytest.mark.parametrize("world,overlap", [(2, True), (3, True), (2, False), (3, False)])
def test_partitioned_matches_single(world, overlap):
    """overlap=True splits each block into own | halo column parts and runs the
    exchange asynchronously; overlap=False is the single-block path."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, overlap)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    ey, ed, nh, bounds = q.get(timeout=5)
    assert nh > 0 and bounds[0] == 0 and bounds[-1] == 900
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


def _gpu_worker(rank, world, port, q, overlap=True):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from spgemm_new_amd.distributed import PartitionedMaxK
        dev = torch.device("cuda:0")
        indptr, indices = small_csr(2500, seed=6)
        v, h, k = len(indptr) - 1, 256, 32
        values = np.random.default_rng(1).random(len(indices), dtype=np.float32)
        data, sel = random_cbsr(v, k, h, seed=2)
        grad = np.random.default_rng(3).random((v, h), dtype=np.float32)
        m = PartitionedMaxK(torch.from_numpy(indptr).to(dev), torch.from_numpy(indices).to(dev),
                            torch.from_numpy(values).to(dev), rank, world, dev, panel_cost=256,
                            overlap=overlap)
        td = lambda a: m.local_rows(torch.from_numpy(a).to(dev))  # noqa: E731
        y = m.forward(td(data), td(sel), h)
        dx = m.backward(td(grad), td(sel))
        torch.cuda.synchronize()
        ys, dxs = [None] * world, [None] * world
        dist.all_gather_object(ys, y.cpu().numpy())
        dist.all_gather_object(dxs, dx.cpu().numpy())
        if rank == 0:
            from oracle import oracle as O
            ey = O.parity_error(np.concatenate(ys), O.np_forward(indptr, indices, values, data, sel, h))
            ed = O.parity_error(np.concatenate(dxs), O.np_backward(indptr, indices, values, grad, sel))
            q.put((ey, ed))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("overlap", [True, False])
def test_partitioned_hip_engine_two_ranks_one_gpu(overlap):
    """2 ranks share cuda:0; HIP kernels on rectangular row blocks with halo columns;
    exchange over gloo (staged through host)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, 2, port, q, overlap)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    ey, ed = q.get(timeout=5)
    assert ey <= 1e-4 and ed <= 1e-4, (ey, ed)
