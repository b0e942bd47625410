"""Multi-GPU MaxK aggregation: 1-D row partition + all-to-all-v halo exchange.

The reference is single-GPU (SURVEY.md §2.2 "Collectives: none"); this is the
distribution the north star asks for:

* rank p owns a contiguous block of rows [r_p, r_{p+1}) of A, balanced on
  edges + rows (the same cost model as the panel schedule), together with its
  nodes' CBSR rows, gradient rows and dXs rows;
* its block of A is stored as a num_own x (num_own + num_halo) CSR whose
  columns are renumbered once: own nodes first, then the remote ("halo") nodes
  it references, grouped by owner rank;
* forward: one all-to-all-v of packed CBSR rows (k fp32 + k uint8 = 5k bytes
  per halo node) brings the halo rows in, then the local SpGEMM runs;
* backward: the local SSpMM produces dXs for own AND halo columns; one reverse
  all-to-all-v returns the halo partial sums (4k bytes per node) to their
  owners, which add them in.

One process per GPU; torch.distributed (RCCL over xGMI with the "nccl"
backend; gloo for CPU tests).  RCCL's all_to_all_single is a grouped
send/recv across all peers, so every xGMI link is used at once.

The local compute is pluggable (``engine``) so the partition / exchange logic
can be tested on CPU with gloo; the default engine is the HIP MaxKGraph.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .ops import MaxKGraph


class _Done:
    def wait(self):
        return None


def a2a(out: torch.Tensor, inp: torch.Tensor, out_split=None, in_split=None,
        async_op: bool = False):
    """all_to_all_single; with the gloo backend, device tensors are staged
    through host memory (tests on one GPU) and the call completes before it
    returns.  RCCL ("nccl") runs in place; with async_op the collective is
    ordered after the work already on the current stream and the returned
    handle's wait() orders later work after it, so kernels launched in
    between overlap the transfer."""
    if out.is_cuda and dist.get_backend() == "gloo":
        o = out.cpu()
        dist.all_to_all_single(o, inp.cpu(), out_split, in_split)
        out.copy_(o)
        return _Done() if async_op else out
    if async_op:
        return dist.all_to_all_single(out, inp, out_split, in_split, async_op=True)
    dist.all_to_all_single(out, inp, out_split, in_split)
    return out


def row_partition(indptr: torch.Tensor, world: int, row_cost: int = 16) -> list[int]:
    """Contiguous row bounds [b_0=0, ..., b_world=V] balancing edges + row_cost*rows."""
    V = indptr.numel() - 1
    cost = indptr.long() - int(indptr[0]) + torch.arange(V + 1, device=indptr.device) * row_cost
    total = int(cost[-1])
    tgt = torch.tensor([total * p / world for p in range(world + 1)], device=indptr.device,
                       dtype=torch.float64)
    b = torch.searchsorted(cost.double(), tgt).clamp_(0, V).tolist()
    b[0], b[-1] = 0, V
    for i in range(1, world + 1):
        b[i] = max(b[i], b[i - 1])
    return b


class HaloPlan:
    """Static exchange plan of one rank (built once per graph)."""

    def __init__(self, indptr, indices, bounds, rank, world, device):
        self.rank, self.world, self.bounds = rank, world, bounds
        r0, r1 = bounds[rank], bounds[rank + 1]
        e0, e1 = int(indptr[r0]), int(indptr[r1])
        self.num_own = r1 - r0
        cols = indices[e0:e1].to(device).long()
        own = (cols >= r0) & (cols < r1)
        halo = torch.unique(cols[~own])                        # sorted global ids
        self.num_halo = halo.numel()
        b = torch.tensor(bounds, device=device)
        owner = torch.searchsorted(b, halo, right=True) - 1     # ascending: grouped by owner
        self.recv_counts = torch.bincount(owner, minlength=world).tolist()
        local = torch.empty_like(cols)
        local[own] = cols[own] - r0
        local[~own] = self.num_own + torch.searchsorted(halo, cols[~own])
        self.local_indptr = (indptr[r0:r1 + 1].to(device) - e0).to(torch.int32).contiguous()
        self.local_indices = local.to(torch.int32).contiguous()
        self.halo_global = halo
        # who needs which of my nodes: exchange the requested id lists once
        send_counts = torch.zeros(world, dtype=torch.int64, device=device)
        a2a(send_counts, torch.tensor(self.recv_counts, dtype=torch.int64, device=device))
        self.send_counts = send_counts.tolist()
        req = torch.empty(sum(self.send_counts), dtype=torch.int64, device=device)
        a2a(req, halo.contiguous(), self.send_counts, self.recv_counts)
        self.send_local = (req - r0).contiguous()               # my local ids to send, per peer
        self.edge_range = (e0, e1)

    @property
    def halo_bytes_fwd_per_k(self):
        return self.num_halo * 5


def _default_engine(local_indptr, local_indices, local_values, num_cols, **kw):
    return MaxKGraph(local_indptr, local_indices, local_values, num_cols=num_cols, **kw)


class PartitionedMaxK:
    """A rank's share of the graph + its halo exchange.

    ``forward(data_own, sel_own, dim)`` returns Y for own rows;
    ``backward(G_own, sel_own)`` returns dXs for own nodes (halo sums added).
    ``engine(indptr, indices, values, num_cols, **kw)`` builds the local compute
    object (must provide ``forward(data, sel, dim)`` / ``backward(grad, sel)``).
    """

    def __init__(self, indptr, indices, values, rank: int, world: int, device,
                 engine=None, row_cost: int = 16, overlap: bool = True, **engine_kw):
        self.rank, self.world, self.device = rank, world, torch.device(device)
        self.bounds = row_partition(indptr, world, row_cost)
        self.plan = HaloPlan(indptr, indices, self.bounds, rank, world, self.device)
        p = self.plan
        e0, e1 = p.edge_range
        lv = values[e0:e1].to(self.device).contiguous()
        make = engine or _default_engine
        # overlap (forward): the block is also split by column into own | halo
        # parts, so the own part computes while the halo CBSR is in flight.  The
        # backward keeps the single block: split, each part's LOCAL sweep visits
        # every source band and the pair cost +0.05 ms (N=8) to +0.31 ms (N=2)
        # more than the block, more than the exchange they would hide
        # (tools/exp_rank_local.py).
        self.overlap = overlap and p.num_halo > 0
        if self.overlap:
            li = p.local_indices.long()
            is_own = li < p.num_own
            rows = torch.repeat_interleave(
                torch.arange(p.num_own, device=self.device),
                (p.local_indptr[1:] - p.local_indptr[:-1]).long(), output_size=li.numel())

            def part(mask, col_shift, ncols):
                ip = torch.zeros(p.num_own + 1, dtype=torch.int32, device=self.device)
                ip[1:] = torch.cumsum(torch.bincount(rows[mask], minlength=p.num_own), 0)
                return make(ip, (li[mask] - col_shift).to(torch.int32).contiguous(),
                            lv[mask].contiguous(), ncols, **engine_kw)
            self.local_own = part(is_own, 0, p.num_own)
            self.local_halo = part(~is_own, p.num_own, p.num_halo)
        self.local = make(p.local_indptr, p.local_indices, lv, p.num_own + p.num_halo,
                          **engine_kw)
        self._halo_sel = None
        self._h_sel = None

    # --------------------------------------------------------------- helpers
    def local_rows(self, t: torch.Tensor) -> torch.Tensor:
        """Slice of a global per-node tensor owned by this rank."""
        r0, r1 = self.bounds[self.rank], self.bounds[self.rank + 1]
        return t[r0:r1].to(self.device).contiguous()

    def _exchange(self, send_rows: torch.Tensor, width: int, dtype, reverse: bool = False):
        p = self.plan
        sc, rc = (p.recv_counts, p.send_counts) if reverse else (p.send_counts, p.recv_counts)
        out = torch.empty((sum(rc), width), dtype=dtype, device=self.device)
        a2a(out, send_rows.contiguous(), rc, sc)
        return out

    # --------------------------------------------------------------- compute
    def gather_halo_cbsr(self, data_own: torch.Tensor, sel_own: torch.Tensor):
        """All-to-all-v of packed CBSR rows -> (data, sel) for own + halo columns."""
        p = self.plan
        k = data_own.shape[1]
        packed = torch.cat([data_own[p.send_local].view(torch.uint8).reshape(-1, 4 * k),
                            sel_own[p.send_local]], dim=1)
        recv = self._exchange(packed, 5 * k, torch.uint8)
        h_data = recv[:, : 4 * k].contiguous().view(torch.float32).reshape(-1, k)
        h_sel = recv[:, 4 * k:].contiguous()
        data = torch.cat([data_own, h_data]).contiguous()
        sel = torch.cat([sel_own, h_sel]).contiguous()
        return data, sel

    def forward(self, data_own: torch.Tensor, sel_own: torch.Tensor, dim_origin: int = 256):
        if self.overlap:
            return self._forward_overlap(data_own, sel_own, dim_origin)
        data, sel = self.gather_halo_cbsr(data_own, sel_own)
        self._halo_sel = sel
        return self.local.forward(data, sel, dim_origin)

    def _forward_overlap(self, data_own, sel_own, dim_origin):
        p = self.plan
        k = data_own.shape[1]
        packed = torch.cat([data_own[p.send_local].view(torch.uint8).reshape(-1, 4 * k),
                            sel_own[p.send_local]], dim=1).contiguous()
        recv = torch.empty((sum(p.recv_counts), 5 * k), dtype=torch.uint8, device=self.device)
        work = a2a(recv, packed, p.recv_counts, p.send_counts, async_op=True)
        y = self.local_own.forward(data_own, sel_own, dim_origin)   # overlaps the exchange
        work.wait()
        h_data = recv[:, : 4 * k].contiguous().view(torch.float32).reshape(-1, k)
        h_sel = recv[:, 4 * k:].contiguous()
        self._h_sel = h_sel
        self._halo_sel = None
        y += self.local_halo.forward(h_data, h_sel, dim_origin)
        return y

    def backward(self, grad_own: torch.Tensor, sel_own: torch.Tensor | None = None):
        p = self.plan
        if self._halo_sel is None and self._h_sel is not None and sel_own is not None:
            self._halo_sel = torch.cat([sel_own, self._h_sel]).contiguous()
        sel = self._halo_sel
        if sel is None or (sel_own is not None and sel.shape[0] != p.num_own + p.num_halo):
            if sel_own is None:
                raise RuntimeError("backward needs the forward's selectors (call forward first)")
            k = sel_own.shape[1]
            recv = self._exchange(sel_own[p.send_local], k, torch.uint8)
            sel = torch.cat([sel_own, recv]).contiguous()
        dxs = self.local.backward(grad_own, sel)
        k = dxs.shape[1]
        partial = dxs[p.num_own:]                               # halo partial sums, by owner
        back = self._exchange(partial, k, torch.float32, reverse=True)
        own = dxs[: p.num_own]
        own.index_add_(0, p.send_local, back)
        return own

    def algorithmic_bytes(self, k: int, h: int) -> int:
        """This rank's share of 8E + 5kE + 4hV (fwd) = (bwd)."""
        e = self.plan.local_indices.numel()
        return 8 * e + 5 * k * e + 4 * h * self.plan.num_own
