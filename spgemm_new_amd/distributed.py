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

import warnings

import torch
import torch.distributed as dist

from . import _lib
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


def ag(out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
    """all_gather_into_tensor (every rank's equal-sized chunk, in rank order);
    with gloo the device tensors are staged through host memory and the call
    completes before it returns (tests on one GPU)."""
    if out.is_cuda and dist.get_backend() == "gloo":
        world = dist.get_world_size()
        chunks = [torch.empty_like(inp, device="cpu") for _ in range(world)]
        dist.all_gather(chunks, inp.cpu())
        out.copy_(torch.cat(chunks))
        return _Done() if async_op else out
    if async_op:
        return dist.all_gather_into_tensor(out, inp, async_op=True)
    dist.all_gather_into_tensor(out, inp)
    return out


# overlap="auto": split a rank's block into own | halo parts (the forward's
# exchange hidden behind the own part) only when the halo records, sized at the
# benchmark's k = 32 (160 B per node), reach this many bytes
OVERLAP_MIN_HALO_BYTES = 64 << 20
OVERLAP_BYTES_PER_HALO_NODE = 160

# rounds="auto": a two-round pipelined exchange when some rank's halo has at least
# this many times its own nodes and its records reach ROUNDS_MIN_HALO_BYTES
ROUNDS_MIN_HALO_RATIO = 4.0
ROUNDS_MIN_HALO_BYTES = 256 << 20

# all-gather the CBSR instead of the all-to-all-v of halo records when some
# rank's halo covers more than this fraction of V ("when the halo
# is close to the full vertex set"; then both move about (N-1)/N of the table)
HALO_ALLGATHER_FRAC = 0.75


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

    def __init__(self, indptr, indices, bounds, rank, world, device, local_block: bool = False):
        self.rank, self.world, self.bounds = rank, world, bounds
        r0, r1 = bounds[rank], bounds[rank + 1]
        e0, e1 = int(indptr[r0]), int(indptr[r1])
        self.num_own = r1 - r0
        # local_block: `indices` holds only this rank's edges [e0, e1)
        cols = (indices if local_block else indices[e0:e1]).to(device).long()
        if cols.numel() != e1 - e0:
            raise RuntimeError(f"rank {rank}: expected {e1 - e0} edges of rows [{r0}, {r1}), "
                               f"got {cols.numel()}")
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


def _train_fwd(eng, data, sel, dim_origin):
    """A training forward of a local block: its backward follows with the same
    selector tensor, so a MaxKGraph engine writes the edge selectors when its
    AUTO backward chose an edge-selector algorithm (edge_sel="auto", as
    SpGEMMFunction does)."""
    if isinstance(eng, MaxKGraph):
        return eng.forward(data, sel, dim_origin, edge_sel="auto")
    return eng.forward(data, sel, dim_origin)


def _default_engine(local_indptr, local_indices, local_values, num_cols, **kw):
    return MaxKGraph(local_indptr, local_indices, local_values, num_cols=num_cols, **kw)


def _records_ok(k: int) -> bool:
    """k for which the halo records (maxk_cbsr_gather_records) exist."""
    return 4 <= k <= 256 and k & (k - 1) == 0


class PartitionedMaxK:
    """A rank's share of the graph + its halo exchange.

    ``forward(data_own, sel_own, dim)`` returns Y for own rows;
    ``backward(G_own, sel_own)`` returns dXs for own nodes (halo sums added).
    With ``values`` fp32[E, R] (R edge-feature relations, BASELINE config 5)
    ``forward_multi`` / ``backward_multi`` are the partitioned fused
    multi-relation forward ([R, own rows, h]) and its backward.

    The halo CBSR travels as records (k fp32 + k selector bytes, 5k B per node,
    one all-to-all-v message) that the receiver's forward reads in place
    (MaxKGraph.forward_records); with ``overlap`` the rank's block is split
    by column into own | halo parts, the own part computes while the records
    are in flight and the halo part accumulates onto it.

    ``engine(indptr, indices, values, num_cols, **kw)`` builds the local
    compute object: ``forward(data, sel, dim)``, ``backward(grad, sel)``,
    optionally ``forward_records(records, k, dim, out=, accumulate=)`` (used
    when present and k is a power of two in [4, 256]; otherwise the halo rows
    are unpacked and concatenated), and ``forward_multi`` / ``backward_multi``
    for relations.
    """

    def __init__(self, indptr, indices, values, rank: int, world: int, device,
                 engine=None, row_cost: int = 16, overlap: bool | str = True, records: bool = True,
                 local_block: bool = False, overlap_backward: bool | None = None,
                 bwd_algo: int | None = None, halo_mode: str = "auto", rounds: int | str = "auto",
                 pipeline_fwd: bool = True, own_bwd_algo: int | str | None = "auto",
                 **engine_kw):
        """indptr: the GLOBAL row pointer (V + 1 entries, cheap); indices /
        values: the global arrays, or with ``local_block=True`` only this rank's
        edges (rows [bounds[rank], bounds[rank + 1]) of ``row_partition(indptr,
        world, row_cost)``), so no rank materialises the whole graph.

        ``bwd_algo`` pins the local backward algorithm (a ``_lib.MAXK_BWD_*``
        code) of every part; None keeps the engine's AUTO, which tunes the
        single block and the own / halo parts separately and may pick
        different algorithms (so different fp32 summation orders) for them.

        ``halo_mode``: "records" -- the forward's all-to-all-v
        of exactly the halo rows; "allgather" -- every rank all-gathers the
        whole CBSR as records (5k B per node, its own rows one chunk; no
        per-peer packing) and the halo part reads the halo rows in place from
        that table; "auto" -- allgather when some rank's halo exceeds
        HALO_ALLGATHER_FRAC of V (products at N = 8: 87 %),
        decided once with an all-reduce so every rank calls the same collective.
        The halo part computes on the same edges in the same order either way,
        so Y is bitwise the same; the backward's reverse exchange is the
        all-to-all-v of halo partial sums in both modes.

        ``rounds`` (R >= 1): every exchange is split into R
        all-to-all-v rounds, round j carrying the j-th slice of each peer's rows
        (slices of equal count), and the halo columns are numbered round-major so
        a round's rows are one contiguous range.  With the own | halo split, the
        records forward issues all R rounds at once and runs the halo columns of
        round j as soon as round j has arrived (one engine per round), and the
        backward sends round j's partial sums as soon as its columns are done, so
        the exchange pipelines with the halo compute instead of only with the
        own part.  Backward: with an order-independent local algorithm (TILE with
        one source range, LOCAL) dXs is bitwise the R = 1 result; the forward adds
        each row's halo edges round by round (a different fp32 grouping, 1e-4).
        ``pipeline_fwd=False`` keeps the rounds in the exchange and the backward
        but runs the forward's halo columns once, after the last round.

        ``own_bwd_algo``: the own-column part's backward in the overlapped
        backward, which runs while the reverse exchange is in flight.  A kernel
        that holds every CU's registers (TILE: one 16-wave workgroup per CU)
        leaves no room for the collective's kernel, so the two serialise
        (modeled wire, products N = 8 rank step 3.76 -> 3.58 ms at
        500 GB/s); "auto" (default) therefore takes STAGED where the part's own
        choice would be TILE, a MAXK_BWD_* code pins it, None keeps the part's
        choice (``bwd_algo``, when given, pins every part instead)."""
        self.rank, self.world, self.device = rank, world, torch.device(device)
        self.bounds = row_partition(indptr, world, row_cost)
        self.plan = HaloPlan(indptr, indices, self.bounds, rank, world, self.device,
                             local_block=local_block)
        p = self.plan
        # overlap and rounds are decided together, collectively (one all-reduce MAX of
        # the halo size and the halo / own ratio), so every rank splits the same way and
        # calls the same number of collectives
        if overlap != "auto" and not isinstance(overlap, bool):
            raise RuntimeError("overlap must be True, False or 'auto'")
        if rounds != "auto" and (not isinstance(rounds, int) or rounds < 1):
            raise RuntimeError("rounds must be an int >= 1 or 'auto'")
        if overlap == "auto" or rounds == "auto":
            hmax, ratio = self._max_over_ranks(float(p.num_halo),
                                               p.num_halo / max(1, p.num_own))
            if overlap == "auto":
                # split only when the exchange is worth hiding: the split costs 0.15-0.4
                # ms of compute per step on Reddit blocks (two engines, their own launches
                # and partials: N=2/4/8 step 3.10/1.84/1.04 ms split vs 2.72/1.57/0.89
                # single, tools/exp_rank_step.py) against 19-33 MB of halo records, a few
                # tenths of that over 7 xGMI links; products' 200-340 MB are not
                overlap = hmax * OVERLAP_BYTES_PER_HALO_NODE >= OVERLAP_MIN_HALO_BYTES
            if rounds == "auto":
                # two rounds when the halo dwarfs the own block (products N = 8: halo 7x
                # own, 342 MB of records; modeled wire at 300 / 500 GB/s: step 4.43 ->
                # 4.00 / 3.59 -> 3.39 ms; at N = 4, halo 3x own, two rounds measured
                # slower at every rate: DESIGN §6)
                rounds = 2 if (overlap and ratio >= ROUNDS_MIN_HALO_RATIO and
                               hmax * OVERLAP_BYTES_PER_HALO_NODE >= ROUNDS_MIN_HALO_BYTES) else 1
        self.rounds = int(rounds) if world > 1 else 1
        self.pipeline_fwd = bool(pipeline_fwd)
        self.own_bwd_algo = own_bwd_algo
        self._round_tab = self._round_major(p, self.rounds)
        e0, e1 = p.edge_range
        if values.dim() not in (1, 2):
            raise RuntimeError("values must be fp32[E] or fp32[E, R]")
        self.num_rel = 1 if values.dim() == 1 else values.shape[1]
        lv_all = (values if local_block else values[e0:e1]).to(self.device).contiguous()
        if lv_all.shape[0] != e1 - e0:
            raise RuntimeError("values must match indices")
        self.values_local = lv_all                       # [E_local] or [E_local, R]
        lv = lv_all if self.num_rel == 1 else lv_all[:, 0].contiguous()
        make = engine or _default_engine
        self.send_rows = p.send_local.to(torch.int32).contiguous()
        # reverse exchange: the partial sums come back in send order; the owners'
        # add runs per own node over its (sorted) returns -- no atomics
        # the peer of every send entry; a node's returns are added in peer order
        # whatever the send order (rounds), so R does not change the sum
        peer = self._send_peer
        order = torch.sort(p.send_local * world + peer, stable=True).indices
        nodes, counts = torch.unique_consecutive(p.send_local[order], return_counts=True)
        seg_off = torch.zeros(nodes.numel() + 1, dtype=torch.int64, device=self.device)
        seg_off[1:] = torch.cumsum(counts, 0)
        self._ret = (order.contiguous(), seg_off, nodes.to(torch.int64).contiguous())
        self.records = records
        # overlap: the block is also split by column into own | halo parts.  The
        # forward computes the own part while the halo CBSR is in flight; the
        # backward (overlap_backward, on for N > 1) computes the halo columns
        # first and their partial sums travel while the own columns are computed.
        # The column sets are disjoint, so with bwd_algo pinned to an algorithm
        # whose per-destination order ignores the other columns (LOCAL: a
        # destination's in-edges in source-row order) dXs is bitwise the single
        # block's; STAGED's merge-path panel splits depend on the whole block.  The forward
        # adds each row's own-column edges before its halo-column edges, a
        # different fp32 order than the single block's edge order.
        self.bwd_algo = bwd_algo
        self.overlap = overlap and p.num_halo > 0
        self.halo_rounds = []
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
            # one engine per round over its contiguous range of halo columns
            if self.rounds > 1:
                for (h0, h1, _, _, _, _) in self._round_tab:
                    m = (li >= p.num_own + h0) & (li < p.num_own + h1)
                    self.halo_rounds.append(part(m, p.num_own + h0, h1 - h0))
            hm = ~is_own
            ip_h = torch.zeros(p.num_own + 1, dtype=torch.int32, device=self.device)
            ip_h[1:] = torch.cumsum(torch.bincount(rows[hm], minlength=p.num_own), 0)
            # the halo part's CSR, kept to build its all-gather-table form on demand
            self._halo_csr = (ip_h, (li[hm] - p.num_own).contiguous(), lv[hm].contiguous())
        self._make, self._engine_kw = make, engine_kw
        self.halo_mode = self._pick_halo_mode(halo_mode)
        self._halo_tab = None
        self.local = make(p.local_indptr, p.local_indices, lv, p.num_own + p.num_halo,
                          **engine_kw)
        # backward overlap: the halo columns' dXs first, their reverse exchange in
        # flight while the own columns' dXs are computed (disjoint column sets, so
        # nothing is added twice); each part sweeps the rank's gradient rows
        self.overlap_backward = (self.overlap and world > 1) if overlap_backward is None \
            else bool(overlap_backward and self.overlap)
        self._bufs = {}
        self._fwd_sel = None     # sel_own of the last forward
        self._fwd_block_sel = None   # the single-block forward's own + halo selectors
        self._halo_part = None   # its halo selectors: [num_halo, k] (view of records or rows)

    # --------------------------------------------------------------- helpers
    def _round_major(self, p, R: int):
        """Renumber the plan's halo nodes and send lists round-major (round j =
        the j-th count slice of every peer's rows, peers in rank order) and
        return the round table [(recv0, recv1, recv_counts, send0, send1,
        send_counts)].  R = 1 leaves the plan as built (peer-major)."""
        world, dev = self.world, self.device

        def cuts(n):
            return [n * j // R for j in range(R + 1)]

        def order(counts):
            off = [0]
            for c in counts:
                off.append(off[-1] + c)
            perm, per_round = [], []
            for j in range(R):
                cnt = []
                for q in range(world):
                    c = cuts(counts[q])
                    perm.append((off[q] + c[j], off[q] + c[j + 1]))
                    cnt.append(c[j + 1] - c[j])
                per_round.append(cnt)
            return perm, per_round

        rperm, rcnt = order(p.recv_counts)
        sperm, scnt = order(p.send_counts)
        peer_of = torch.repeat_interleave(torch.arange(world, device=dev),
                                          torch.tensor(p.send_counts, device=dev),
                                          output_size=sum(p.send_counts))
        if R > 1:
            ridx = torch.cat([torch.arange(a, b, device=dev) for a, b in rperm]) \
                if p.num_halo else torch.zeros(0, dtype=torch.int64, device=dev)
            sidx = torch.cat([torch.arange(a, b, device=dev) for a, b in sperm]) \
                if sum(p.send_counts) else torch.zeros(0, dtype=torch.int64, device=dev)
            inv = torch.empty_like(ridx)
            inv[ridx] = torch.arange(ridx.numel(), device=dev)
            p.halo_global = p.halo_global[ridx].contiguous()
            li = p.local_indices.long()
            hm = li >= p.num_own
            li[hm] = p.num_own + inv[li[hm] - p.num_own]
            p.local_indices = li.to(torch.int32).contiguous()
            p.send_local = p.send_local[sidx].contiguous()
            peer_of = peer_of[sidx].contiguous()
        self._send_peer = peer_of
        tab, r0, s0 = [], 0, 0
        for j in range(R):
            r1, s1 = r0 + sum(rcnt[j]), s0 + sum(scnt[j])
            tab.append((r0, r1, rcnt[j], s0, s1, scnt[j]))
            r0, s0 = r1, s1
        return tab

    def _a2a_rounds(self, out, inp, reverse: bool = False, async_op: bool = False):
        """The halo exchange (forward: inp = send rows, out = halo rows; reverse:
        inp = halo rows, out = send rows) as the plan's rounds, one
        all-to-all-v each, in round order; returns the list of handles (async) or
        out.  R = 1: the one all-to-all-v of the whole halo."""
        works = []
        for (r0, r1, rc, s0, s1, sc) in self._round_tab:
            if reverse:
                o, i, oc, ic = out[s0:s1], inp[r0:r1], sc, rc
            else:
                o, i, oc, ic = out[r0:r1], inp[s0:s1], rc, sc
            works.append(a2a(o, i, oc, ic, async_op=async_op))
        return works if async_op else out

    def _max_over_ranks(self, *xs: float) -> list[float] | float:
        """Element-wise MAX of the given floats over all ranks (one all-reduce;
        the values themselves at world 1)."""
        if self.world == 1:
            return xs[0] if len(xs) == 1 else list(xs)
        t = torch.tensor(xs, dtype=torch.float64)
        if dist.get_backend() != "gloo":
            t = t.to(self.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        out = t.cpu().tolist()
        return out[0] if len(xs) == 1 else out

    def _pick_halo_mode(self, mode: str) -> str:
        """Decided collectively: the all-gather path needs the own | halo split on
        EVERY rank (a rank without it -- overlap off, or no halo at all -- would
        call the all-to-all-v of gather_halo_cbsr while the others all-gather),
        so one all-reduce carries the largest halo fraction and whether any rank
        is unsplit; "allgather" is only taken when no rank is."""
        if mode not in ("auto", "records", "allgather"):
            raise RuntimeError("halo_mode must be 'auto', 'records' or 'allgather'")
        if self.world == 1:
            return "records" if mode == "auto" else mode
        if mode == "records":
            return mode
        if mode == "auto" and self.rounds > 1:
            # the pipelined forward runs on the records rounds (the same on every rank:
            # rounds is decided collectively); products N = 8, modeled wire 500 GB/s:
            # records in 2 rounds 3.39 ms vs all-gather 3.57 ms
            return "records"
        p = self.plan
        V = self.bounds[-1]
        frac, unsplit = self._max_over_ranks(p.num_halo / max(1, V), 0.0 if self.overlap else 1.0)
        if unsplit > 0:
            if mode == "allgather":
                # a pinned mode is not downgraded silently: the caller
                # would measure the all-to-all-v path believing it all-gathers
                warnings.warn("halo_mode='allgather' needs the own | halo split on every rank "
                              "(overlap on, a halo on each rank); using 'records'",
                              RuntimeWarning, stacklevel=3)
            return "records"
        if mode == "allgather":
            return mode
        return "allgather" if frac > HALO_ALLGATHER_FRAC else "records"

    def _allgather_ok(self, k: int) -> bool:
        # halo_mode == "allgather" implies every rank is split (_pick_halo_mode); k is
        # the same on every rank, so the records test agrees too
        return (self.halo_mode == "allgather" and self.overlap and self.world > 1
                and self._use_records(k, self.local_halo))

    def _table(self):
        """(max_own, halo table rows, halo-part engine over table rows): row r of
        rank q sits at q * max_own + (r - bounds[q]) of the all-gathered table."""
        if self._halo_tab is None:
            p = self.plan
            b = torch.tensor(self.bounds, device=self.device)
            max_own = max(self.bounds[i + 1] - self.bounds[i] for i in range(self.world))
            owner = torch.searchsorted(b, p.halo_global, right=True) - 1
            pos = (owner * max_own + (p.halo_global - b[owner])).to(torch.int32).contiguous()
            ip_h, cols_h, vals_h = self._halo_csr
            eng = self._make(ip_h, pos[cols_h.long()].contiguous(), vals_h, self.world * max_own,
                             **self._engine_kw)
            self._halo_tab = (max_own, pos, eng)
            self._halo_tab_pos64 = pos.long()
        return self._halo_tab

    def local_rows(self, t: torch.Tensor) -> torch.Tensor:
        """Slice of a global per-node tensor owned by this rank."""
        r0, r1 = self.bounds[self.rank], self.bounds[self.rank + 1]
        return t[r0:r1].to(self.device).contiguous()

    def _buf(self, key, shape, dtype):
        t = self._bufs.get(key)
        if t is None or tuple(t.shape) != tuple(shape) or t.dtype != dtype:
            t = torch.empty(shape, dtype=dtype, device=self.device)
            self._bufs[key] = t
        return t

    def _exchange(self, send_rows: torch.Tensor, width: int, dtype, reverse: bool = False):
        p = self.plan
        n = sum(p.send_counts) if reverse else sum(p.recv_counts)
        out = torch.empty((n, width), dtype=dtype, device=self.device)
        return self._a2a_rounds(out, send_rows.contiguous(), reverse=reverse)

    def _use_records(self, k: int, eng) -> bool:
        return self.records and _records_ok(k) and hasattr(eng, "forward_records")

    def _pack(self, data_own, sel_own):
        """The rows my peers need, as one uint8 message [n_send, 5k]."""
        k = data_own.shape[1]
        if _records_ok(k) and data_own.is_cuda:
            from .ops import cbsr_gather_records
            return cbsr_gather_records(data_own, sel_own, self.send_rows,
                                       out=self._buf(("send", k), (self.send_rows.numel(), 5 * k),
                                                     torch.uint8))
        rows = self.plan.send_local
        return torch.cat([data_own[rows].view(torch.uint8).reshape(-1, 4 * k), sel_own[rows]],
                         dim=1).contiguous()

    @staticmethod
    def _unpack(rec: torch.Tensor, k: int):
        data = rec[:, : 4 * k].contiguous().view(torch.float32).reshape(-1, k)
        return data, rec[:, 4 * k:]

    # --------------------------------------------------------------- compute
    def gather_halo_cbsr(self, data_own: torch.Tensor, sel_own: torch.Tensor):
        """All-to-all-v of packed CBSR rows -> (data, sel) for own + halo columns,
        written straight into the block's buffers (own rows copied while the
        exchange is in flight, halo records unpacked into the tail)."""
        p = self.plan
        k = data_own.shape[1]
        n = p.num_own + p.num_halo
        recv = self._buf(("recv", k), (p.num_halo, 5 * k), torch.uint8)
        works = self._a2a_rounds(recv, self._pack(data_own, sel_own), async_op=True)
        data = self._buf(("data_all", k), (n, k), torch.float32)
        sel = self._buf(("sel_all_fwd", k), (n, k), torch.uint8)
        data[: p.num_own] = data_own
        sel[: p.num_own] = sel_own
        for w in works:
            w.wait()
        hd = recv[:, : 4 * k]
        data[p.num_own:] = (hd if (5 * k) % 4 == 0 else hd.contiguous()).view(torch.float32)
        sel[p.num_own:] = recv[:, 4 * k:]
        self._fwd_sel, self._halo_part = sel_own, sel[p.num_own:]
        self._fwd_block_sel = sel
        return data, sel

    def forward(self, data_own: torch.Tensor, sel_own: torch.Tensor, dim_origin: int = 256):
        p = self.plan
        k = data_own.shape[1]
        if not self.overlap:
            # single block: the halo rows are appended to the own rows (a table
            # of whole 160-B records read in place measured slower than data +
            # selector rows at full size: 3.63 vs 3.31 ms, tools/exp_rank_step.py)
            data, sel = self.gather_halo_cbsr(data_own, sel_own)
            return _train_fwd(self.local, data, sel, dim_origin)
        if not self._use_records(k, self.local_halo):
            return self._forward_overlap_rows(data_own, sel_own, dim_origin)
        if self._allgather_ok(k):
            return self._forward_allgather(data_own, sel_own, dim_origin)
        recv = self._buf(("recv", k), (p.num_halo, 5 * k), torch.uint8)
        works = self._a2a_rounds(recv, self._pack(data_own, sel_own), async_op=True)
        y = _train_fwd(self.local_own, data_own, sel_own, dim_origin)   # overlaps the exchange
        if self.halo_rounds and self.pipeline_fwd:
            # round j's halo columns as soon as round j has arrived (the later rounds
            # still on the wire)
            for w, eng, (r0, r1, _, _, _, _) in zip(works, self.halo_rounds, self._round_tab):
                w.wait()
                eng.forward_records(recv[r0:r1], k, dim_origin, out=y, accumulate=True)
        else:
            for w in works:
                w.wait()
            # the halo block reads the received records in place and adds onto y
            self.local_halo.forward_records(recv, k, dim_origin, out=y, accumulate=True)
        self._fwd_sel, self._halo_part = sel_own, recv[:, 4 * k:]
        return y

    def _forward_allgather(self, data_own, sel_own, dim_origin):
        """halo_mode "allgather": every rank's own rows as one records chunk,
        all-gathered (padded to the largest block); the own part computes while
        it is in flight; the halo part then reads its rows in place from the
        table (same edges and order as the records path: bitwise the same Y)."""
        from .ops import cbsr_gather_records
        p = self.plan
        k = data_own.shape[1]
        max_own, pos, eng = self._table()
        mine = self._bufs.get(("ag_send", k))
        if mine is None:   # rows past this rank's block are padding: zeros, never read
            mine = self._bufs[("ag_send", k)] = torch.zeros((max_own, 5 * k), dtype=torch.uint8,
                                                           device=self.device)
        if data_own.is_cuda:
            cbsr_gather_records(data_own, sel_own, out=mine[: p.num_own])
        else:
            mine[: p.num_own, : 4 * k] = data_own.contiguous().view(torch.uint8).reshape(-1, 4 * k)
            mine[: p.num_own, 4 * k:] = sel_own
        table = self._buf(("ag_table", k), (self.world * max_own, 5 * k), torch.uint8)
        work = ag(table, mine, async_op=True)
        y = _train_fwd(self.local_own, data_own, sel_own, dim_origin)   # overlaps the all-gather
        work.wait()
        eng.forward_records(table, k, dim_origin, out=y, accumulate=True)
        self._fwd_sel = sel_own
        # the halo columns' selectors for the backward (maxk_records_sel_gather;
        # torch's index_select of the strided selector columns took 0.45 ms at
        # products N=8, 2.1 M rows)
        hs = self._buf(("ag_halo_sel", k), (p.num_halo, k), torch.uint8)
        if table.is_cuda:
            from . import _lib
            _lib.check(_lib.load().maxk_records_sel_gather(table.data_ptr(), k, pos.data_ptr(),
                                                            p.num_halo, hs.data_ptr(),
                                                            _lib.stream_ptr(table.device)),
                       "maxk_records_sel_gather")
        else:
            hs.copy_(torch.index_select(table[:, 4 * k:], 0, self._halo_tab_pos64))
        self._halo_part = hs
        return y

    def halo_bytes(self, k: int) -> dict:
        """Bytes this rank receives per step in each exchange, both halo modes."""
        p = self.plan
        max_own = max(self.bounds[i + 1] - self.bounds[i] for i in range(self.world))
        return {"records_fwd": p.num_halo * 5 * k,
                "allgather_fwd": (self.world - 1) * max_own * 5 * k,
                "reverse_bwd": p.num_halo * 4 * k}

    def exchange_ms(self, k: int, reps: int = 10) -> dict:
        """Wire time of this rank's exchanges, each run alone (not overlapped) with
        the step's message sizes: the forward's all-to-all-v of halo records (or
        the all-gather of the CBSR table in that mode) and the backward's reverse
        all-to-all-v of partial sums.  HIP events on the current stream around
        synchronous collectives (the current stream waits for RCCL's), mean of
        `reps` after one warm-up.  Every rank must call it (same order)."""
        p = self.plan
        dev = self.device

        def ev_ms(fn):
            fn()
            if dev.type != "cuda":
                import time
                t0 = time.perf_counter()
                for _ in range(reps):
                    fn()
                return (time.perf_counter() - t0) / reps * 1e3
            st = torch.cuda.current_stream(dev)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(reps):
                fn()
            b.record(st)
            b.synchronize()
            return a.elapsed_time(b) / reps

        out = {}
        if self._allgather_ok(k):
            max_own = max(self.bounds[i + 1] - self.bounds[i] for i in range(self.world))
            mine = torch.zeros((max_own, 5 * k), dtype=torch.uint8, device=dev)
            table = torch.empty((self.world * max_own, 5 * k), dtype=torch.uint8, device=dev)
            out["fwd_allgather_ms"] = ev_ms(lambda: ag(table, mine))
            out["fwd_bytes_in"] = (self.world - 1) * max_own * 5 * k
            del mine, table
        else:
            send = torch.zeros((self.send_rows.numel(), 5 * k), dtype=torch.uint8, device=dev)
            recv = torch.empty((p.num_halo, 5 * k), dtype=torch.uint8, device=dev)
            out["fwd_a2a_ms"] = ev_ms(lambda: a2a(recv, send, p.recv_counts, p.send_counts))
            out["fwd_bytes_in"] = p.num_halo * 5 * k
            del send, recv
        dh = torch.zeros((p.num_halo, k), dtype=torch.float32, device=dev)
        back = torch.empty((sum(p.send_counts), k), dtype=torch.float32, device=dev)
        out["bwd_a2a_ms"] = ev_ms(lambda: a2a(back, dh, p.send_counts, p.recv_counts))
        out["bwd_bytes_out"] = p.num_halo * 4 * k
        return out

    def _forward_overlap_rows(self, data_own, sel_own, dim_origin):
        p = self.plan
        k = data_own.shape[1]
        recv = torch.empty((p.num_halo, 5 * k), dtype=torch.uint8, device=self.device)
        works = self._a2a_rounds(recv, self._pack(data_own, sel_own), async_op=True)
        y = _train_fwd(self.local_own, data_own, sel_own, dim_origin)   # overlaps the exchange
        for w in works:
            w.wait()
        h_data, h_sel = self._unpack(recv, k)
        h_sel = h_sel.contiguous()
        self._fwd_sel, self._halo_part = sel_own, h_sel
        if isinstance(self.local_halo, MaxKGraph):
            self.local_halo.forward(h_data, h_sel, dim_origin, out=y, accumulate=True)
        else:
            y += self.local_halo.forward(h_data, h_sel, dim_origin)
        return y

    def last_halo_selectors(self) -> torch.Tensor:
        """The halo nodes' selectors received by the last forward (a copy: the
        exchange buffers are reused by the next forward)."""
        if self._halo_part is None:
            raise RuntimeError("no forward has run")
        return self._halo_part.contiguous().clone()

    def _block_sel(self, sel_own: torch.Tensor | None, halo_sel=None) -> torch.Tensor:
        """Selectors of the whole block (own + halo columns), contiguous."""
        p = self.plan
        if halo_sel is not None:
            if sel_own is None:
                raise RuntimeError("halo_sel needs sel_own")
            halo = halo_sel
        elif sel_own is None or sel_own is self._fwd_sel:
            if self._halo_part is None:
                raise RuntimeError("backward needs the forward's selectors (call forward first)")
            sel_own, halo = self._fwd_sel, self._halo_part
        else:
            halo = self._exchange(sel_own[p.send_local], sel_own.shape[1], torch.uint8)
        k = sel_own.shape[1]
        sel = self._buf(("sel_all", k), (p.num_own + p.num_halo, k), torch.uint8)
        sel[: p.num_own] = sel_own
        sel[p.num_own:] = halo
        return sel

    def _return_halo(self, dxs: torch.Tensor) -> torch.Tensor:
        """Send the halo partial sums home and add the ones I receive."""
        p = self.plan
        k = dxs.shape[1]
        back = self._exchange(dxs[p.num_own:], k, torch.float32, reverse=True)
        return self._add_returns(back, dxs[: p.num_own])

    def _add_returns(self, back: torch.Tensor, own: torch.Tensor) -> torch.Tensor:
        """own[node] += the partial sums the peers returned for it (fixed order)."""
        p = self.plan
        k = own.shape[1]
        order, seg_off, nodes = self._ret
        if own.is_cuda and nodes.numel() > 0:
            from . import _lib
            _lib.check(_lib.load().maxk_segment_rows_add(
                back.data_ptr(), k, order.data_ptr(), seg_off.data_ptr(), nodes.data_ptr(),
                nodes.numel(), own.data_ptr(), _lib.stream_ptr(own.device)), "maxk_segment_rows_add")
        elif nodes.numel() > 0:
            # the same fixed order as the device path: per node, its returns in peer order
            own.index_add_(0, p.send_local[order], back[order])
        return own

    def backward(self, grad_own: torch.Tensor, sel_own: torch.Tensor | None = None,
                 halo_sel: torch.Tensor | None = None):
        """dXs of the own nodes.  The block's selectors: sel_own + halo_sel when
        given (last_halo_selectors() of that forward), else the last forward's
        when sel_own is its tensor (or None), else exchanged again.  With
        overlap_backward the halo columns go first and their partial sums
        travel while the own columns are computed."""
        last = halo_sel is None and (sel_own is None or sel_own is self._fwd_sel)
        if last and not self.overlap and self._fwd_block_sel is not None:
            # the single-block forward's own selector tensor (own + halo rows as it
            # read them): the engine finds the edge selectors that forward wrote
            sel = self._fwd_block_sel
        else:
            sel = self._block_sel(sel_own, halo_sel)
        if not self.overlap_backward:
            return self._return_halo(self._local_bwd(self.local, grad_own, sel))
        p = self.plan
        k = sel.shape[1]
        back = self._buf(("back", k), (sum(p.send_counts), k), torch.float32)
        if self.halo_rounds:
            # round j's partial sums travel while the later rounds' columns (and then
            # the own columns) are computed
            works = []
            for eng, (r0, r1, rc, s0, s1, sc) in zip(self.halo_rounds, self._round_tab):
                dh = self._local_bwd(eng, grad_own, sel[p.num_own + r0:p.num_own + r1])
                works.append(a2a(back[s0:s1], dh, sc, rc, async_op=True))
        else:
            dh = self._local_bwd(self.local_halo, grad_own, sel[p.num_own:])
            works = self._a2a_rounds(back, dh, reverse=True, async_op=True)
        # the own part: the forward's selector tensor itself when it is the last one
        own_sel = self._fwd_sel if last else sel[: p.num_own]
        own = self._own_bwd(grad_own, own_sel)   # overlaps the exchange
        for w in works:
            w.wait()
        return self._add_returns(back, own)

    def _own_bwd(self, grad, sel):
        """The own-column part's backward while the reverse exchange is in flight
        (own_bwd_algo: "auto" avoids the all-CU TILE kernel there)."""
        eng, a = self.local_own, self.own_bwd_algo
        if self.bwd_algo is not None or a is None:
            return self._local_bwd(eng, grad, sel)
        if a == "auto":
            if not isinstance(eng, MaxKGraph):
                return self._local_bwd(eng, grad, sel)
            out = torch.empty((eng.num_cols, sel.shape[1]), dtype=torch.float32, device=self.device)
            a = _lib.MAXK_BWD_AUTO
            if eng.num_edges > 0 and eng.autotune_backward(grad, sel, out) == _lib.MAXK_BWD_TILE:
                a = _lib.MAXK_BWD_STAGED
            return eng.backward(grad, sel, out=out, algo=a)
        return eng.backward(grad, sel, algo=a)

    def _local_bwd(self, eng, grad, sel):
        if self.bwd_algo is None:
            return eng.backward(grad, sel)
        return eng.backward(grad, sel, algo=self.bwd_algo)

    # ------------------------------------------------- multi-relation (config 5)
    def forward_multi(self, data_own: torch.Tensor, sel_own: torch.Tensor,
                      dim_origin: int = 256) -> torch.Tensor:
        """Y[q] = A_q . X^ for own rows, q < R (values fp32[E, R] at construction):
        one halo exchange shared by all relations, then the fused local forward."""
        if self.num_rel < 2 and self.values_local.dim() == 1:
            raise RuntimeError("forward_multi needs values fp32[E, R] at construction")
        data, sel = self.gather_halo_cbsr(data_own, sel_own)
        return self.local.forward_multi(data, sel, self.values_local, dim_origin)

    def backward_multi(self, grad_own: torch.Tensor, sel_own: torch.Tensor | None = None,
                       halo_sel: torch.Tensor | None = None):
        """dXs = sum_q (A_q^T G_q) at sel for own nodes; grad_own fp32[R, own rows, h]
        (selectors as in backward())."""
        dxs = self.local.backward_multi(grad_own, self._block_sel(sel_own, halo_sel),
                                        self.values_local)
        return self._return_halo(dxs)

    def algorithmic_bytes(self, k: int, h: int) -> int:
        """This rank's share of 8E + 5kE + 4hV (fwd) = (bwd)."""
        e = self.plan.local_indices.numel()
        return 8 * e + 5 * k * e + 4 * h * self.plan.num_own

    def algorithmic_bytes_multi(self, k: int, h: int) -> int:
        """This rank's share of the fused multi-relation forward E(4 + 4R + 5k) + R*4hV."""
        e = self.plan.local_indices.numel()
        R = self.num_rel
        return e * (4 + 4 * R + 5 * k) + R * 4 * h * self.plan.num_own
