#!/usr/bin/env python3
"""One rank's whole partitioned step (PartitionedMaxK: pack, exchange, forward
with overlap split, backward, reverse exchange, index_add) at world sizes
2/4/8 on ONE GPU, with the all-to-all-v replaced by a loopback that delivers
exactly what the peers would send (computed from the global graph).  Measures
everything a rank does except the xGMI wire time.  Development tool.

usage: tools/exp_rank_step.py [--graph reddit] [--k 32] [--worlds 1,2,4,8] [--rows]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spgemm_new_amd.distributed as D  # noqa: E402
from spgemm_new_amd.graphs import CONFIGS, synthetic_csr_gpu  # noqa: E402
from spgemm_new_amd.ops import topk_cbsr  # noqa: E402


class Loopback:
    """Stands in for torch.distributed.all_to_all_single for rank p."""

    def __init__(self, indptr, indices, bounds, p, data, sel):
        self.data, self.sel, self.k = data, sel, data.shape[1]
        world = len(bounds) - 1
        r0, r1 = bounds[p], bounds[p + 1]
        reqs = []
        for q in range(world):   # what peer q needs from me: its halo within my range
            if q == p:
                reqs.append(torch.empty(0, dtype=torch.int64, device=indices.device))
                continue
            e0, e1 = int(indptr[bounds[q]]), int(indptr[bounds[q + 1]])
            c = indices[e0:e1].long()
            reqs.append(torch.unique(c[(c >= r0) & (c < r1)]))
        self.counts = torch.tensor([r.numel() for r in reqs], dtype=torch.int64,
                                   device=indices.device)
        self.req = torch.cat(reqs)
        self.calls = 0
        self.halo = None
        self._bounds_t = torch.tensor(bounds, device=indices.device)

    wire = None   # a wire_model.Wire: the delivery on a side stream behind a modeled wire

    def __call__(self, out, inp, out_split=None, in_split=None, async_op=False):
        self.calls += 1
        if self.calls == 1:                      # HaloPlan: request counts
            out.copy_(self.counts)
            return D._Done() if async_op else out
        if self.calls == 2:                      # HaloPlan: requested ids
            out.copy_(self.req)
            self.halo = inp.clone()              # my halo ids, grouped by owner
            self.halo32 = self.halo.to(torch.int32)
            world = self._bounds_t.numel() - 1   # owner slices, once (no sync in a timed call)
            self._owner_counts = torch.bincount(
                torch.searchsorted(self._bounds_t, self.halo, right=True) - 1,
                minlength=world).tolist()
            return D._Done() if async_op else out
        if out.dtype == torch.uint8 and out.shape[1] == 5 * self.k:   # halo CBSR rows
            def deliver():
                if out_split is not None and sum(out_split) != self.halo32.numel():
                    # one round of a pipelined exchange: the rows of this round
                    rows = self._round_rows(out_split)
                    D_ops.cbsr_gather_records(self.data, self.sel, rows, out=out)
                else:
                    D_ops.cbsr_gather_records(self.data, self.sel, self.halo32, out=out)
        elif out.dtype == torch.uint8:           # halo selectors only
            def deliver():
                out.copy_(self.sel[self.halo])
        else:                                    # reverse: partial sums from the peers
            def deliver():
                out.copy_(inp[: out.shape[0]] if inp.shape[0] >= out.shape[0] else
                          torch.ones_like(out))
        if self.wire is None:
            deliver()
            return D._Done() if async_op else out
        w = self.wire.issue(out.numel() * out.element_size(), deliver, (out, inp), async_op)
        return w if async_op else out

    def _round_rows(self, out_split):
        """Global ids of the halo rows one round of a pipelined exchange carries:
        from every owner q, the next out_split[q] of its halo nodes (in order)."""
        if not hasattr(self, "_next"):
            self._next = None
        world = len(out_split)
        if self._next is None or all(n == 0 for n in self._next_left):
            owner_counts = self._owner_counts
            starts = [0]
            for c in owner_counts[:-1]:
                starts.append(starts[-1] + c)
            self._next, self._next_left = list(starts), list(owner_counts)
        parts = []
        for q in range(world):
            n = out_split[q]
            parts.append(self.halo32[self._next[q]:self._next[q] + n])
            self._next[q] += n
            self._next_left[q] -= n
        return torch.cat(parts)


import spgemm_new_amd.ops as D_ops  # noqa: E402
from spgemm_new_amd import _lib as D_lib  # noqa: E402


class GatherLoopback:
    """Stands in for the all-gather of the "allgather" halo mode: the table of
    every rank's own records, rank q's block at rows q * max_own ..."""

    def __init__(self, bounds, data, sel):
        self.bounds, self.data, self.sel = bounds, data, sel

    wire = None

    def __call__(self, out, inp, async_op=False):
        world = len(self.bounds) - 1
        max_own = out.shape[0] // world

        def deliver():
            for q in range(world):
                r0, r1 = self.bounds[q], self.bounds[q + 1]
                rows = torch.arange(r0, r1, device=out.device, dtype=torch.int32)
                D_ops.cbsr_gather_records(self.data, self.sel, rows,
                                          out=out[q * max_own:q * max_own + r1 - r0])
        if self.wire is None:
            deliver()
            return D._Done() if async_op else out
        nbytes = (world - 1) * max_own * out.shape[1]
        w = self.wire.issue(nbytes, deliver, (out, inp), async_op)
        return w if async_op else out


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graph", default="reddit")
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--h", type=int, default=256)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--rows", action="store_true", help="unpacked-rows halo path (no records)")
    ap.add_argument("--halo-mode", default="records", choices=["records", "allgather"])
    ap.add_argument("--no-overlap", action="store_true", help="single block: no own / halo split")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    V, E = CONFIGS[a.graph]
    h, k = a.h, a.k
    indptr, indices = synthetic_csr_gpu(V, E, device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(5)
    values = torch.rand(E, generator=gen, device=dev)
    X = torch.rand((V, h), generator=gen, device=dev)
    G = torch.rand((V, h), generator=gen, device=dev)
    data, sel = topk_cbsr(X, k)
    for world in [int(w) for w in a.worlds.split(",")]:
        bounds = D.row_partition(indptr, world)
        for p in sorted({0, world - 1}):
            lb = Loopback(indptr, indices, bounds, p, data, sel)
            D.a2a = lb
            D.ag = GatherLoopback(bounds, data, sel)
            # no process group here: the collective decisions (halo mode, overlap) take
            # this rank's own values, as if every rank had the same
            D.PartitionedMaxK._max_over_ranks = lambda self, *xs: xs[0] if len(xs) == 1 else list(xs)
            m = D.PartitionedMaxK(indptr, indices, values, p, world, dev, records=not a.rows,
                                  halo_mode=a.halo_mode if world > 1 else "records",
                                  overlap=not a.no_overlap)
            d_l, s_l, g_l = m.local_rows(data), m.local_rows(sel), m.local_rows(G)
            tf = timed(lambda: m.forward(d_l, s_l, h))
            tb = timed(lambda: m.backward(g_l, s_l))
            ts = timed(lambda: (m.forward(d_l, s_l, h), m.backward(g_l, s_l)))
            pl = m.plan
            if m.halo_mode == "allgather":
                max_own, pos, eng = m._table()
                tab = m._bufs[("ag_table", k)]
                y_h = torch.empty((pl.num_own, h), device=dev)
                parts = {
                    "table (loopback all-gather)": lambda: D.ag(tab, None),
                    "halo part over table": lambda: eng.forward_records(tab, k, h, out=y_h,
                                                                        accumulate=True),
                    "halo selectors": lambda: D_lib.load().maxk_records_sel_gather(
                        tab.data_ptr(), k, pos.data_ptr(), pl.num_halo,
                        m._bufs[("ag_halo_sel", k)].data_ptr(), D_lib.stream_ptr(dev)),
                    "own part": lambda: m.local_own.forward(d_l, s_l, h),
                }
                print("   " + ", ".join(f"{n} {timed(f, reps=10):.3f}" for n, f in parts.items()))
            print(f"world={world} rank={p}: own={pl.num_own} halo={pl.num_halo} "
                  f"send={m.send_rows.numel()} edges={pl.local_indices.numel()} | fwd {tf:.3f} "
                  f"bwd {tb:.3f} step {ts:.3f} ms (no wire time) | halo fwd "
                  f"{pl.num_halo * 5 * k / 1e6:.1f} MB in, {m.send_rows.numel() * 5 * k / 1e6:.1f}"
                  f" MB out; bwd algo {m.local.last_bwd_algo}; halo mode {m.halo_mode}", flush=True)
            for nm in ("local", "local_own", "local_halo"):
                e = getattr(m, nm, None)
                if e is not None and hasattr(e, "_tile"):
                    tp = {kk: (None if v is None else (v["num_groups"], v["group_size"],
                                                       v["num_workgroups"]))
                          for kk, v in e._tile.items()}
                    print(f"   {nm}: rows {e.num_rows} cols {e.num_cols} edges {e.num_edges} "
                          f"tile plans {tp} bwd choice {e._bwd_choice} "
                          f"cands {getattr(e, 'bwd_candidates', None)}", flush=True)
                if e is not None:
                    print(f"   {nm}: bwd {getattr(e, 'last_bwd_algo', None)}, fwd blocks "
                          f"{getattr(e, '_fwd_blocks', {})}", flush=True)
            del m, lb, d_l, s_l, g_l
            torch.cuda.empty_cache()




def breakdown_single(graph="reddit", k=32, world=8, rank=0):
    """Per-component times of one rank's single-block step (overlap off: the
    bench's choice on Reddit), loopback exchange."""
    dev = torch.device("cuda:0")
    V, E = CONFIGS[graph]
    h = 256
    indptr, indices = synthetic_csr_gpu(V, E, device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(5)
    values = torch.rand(E, generator=gen, device=dev)
    X = torch.rand((V, h), generator=gen, device=dev)
    G = torch.rand((V, h), generator=gen, device=dev)
    data, sel = topk_cbsr(X, k)
    bounds = D.row_partition(indptr, world)
    lb = Loopback(indptr, indices, bounds, rank, data, sel)
    D.a2a = lb
    m = D.PartitionedMaxK(indptr, indices, values, rank, world, dev, halo_mode="records",
                          overlap=False)
    d_l, s_l, g_l = m.local_rows(data), m.local_rows(sel), m.local_rows(G)
    m.forward(d_l, s_l, h)
    m.backward(g_l, s_l)
    p = m.plan
    dall, sall = m.gather_halo_cbsr(d_l, s_l)
    dx = m.local.backward(g_l, sall)
    rows = {
        "pack": lambda: m._pack(d_l, s_l),
        "gather_halo_cbsr (pack+exchange+copies)": lambda: m.gather_halo_cbsr(d_l, s_l),
        "local forward": lambda: m.local.forward(dall, sall, h),
        "local backward": lambda: m.local.backward(g_l, sall),
        "return halo (exchange + add)": lambda: m._return_halo(dx),
        "whole forward": lambda: m.forward(d_l, s_l, h),
        "whole backward": lambda: m.backward(g_l, s_l),
        "whole step": lambda: (m.forward(d_l, s_l, h), m.backward(g_l, s_l)),
    }
    e = m.local
    print(f"{graph} k={k} world={world} rank={rank} single block: own={p.num_own} "
          f"halo={p.num_halo} edges={e.num_edges} bwd {e.last_bwd_algo} fwd blocks "
          f"{e._fwd_blocks} tile {[(kk, None if v is None else (v['num_groups'], v['group_size'], v['num_workgroups'])) for kk, v in e._tile.items()]}")
    for name, fn in rows.items():
        print(f"  {name:40s} {timed(fn, reps=20):.3f} ms", flush=True)


def breakdown(graph="products", k=32, world=8, rank=0):
    """Per-component times of one rank's step (loopback exchange)."""
    dev = torch.device("cuda:0")
    V, E = CONFIGS[graph]
    h = 256
    indptr, indices = synthetic_csr_gpu(V, E, device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(5)
    values = torch.rand(E, generator=gen, device=dev)
    X = torch.rand((V, h), generator=gen, device=dev)
    G = torch.rand((V, h), generator=gen, device=dev)
    data, sel = topk_cbsr(X, k)
    bounds = D.row_partition(indptr, world)
    lb = Loopback(indptr, indices, bounds, rank, data, sel)
    D.a2a = lb
    m = D.PartitionedMaxK(indptr, indices, values, rank, world, dev, halo_mode="records")
    d_l, s_l, g_l = m.local_rows(data), m.local_rows(sel), m.local_rows(G)
    m.forward(d_l, s_l, h)
    m.backward(g_l, s_l)
    p = m.plan
    send = m._pack(d_l, s_l)
    recv = torch.empty((p.num_halo, 5 * k), dtype=torch.uint8, device=dev)
    y = torch.empty((p.num_own, h), device=dev)
    rows = {
        "pack": lambda: m._pack(d_l, s_l),
        "exchange (loopback)": lambda: lb(recv, send),
        "own-column forward": lambda: m.local_own.forward(d_l, s_l, h, out=y),
        "halo-column forward (records, +=)": lambda: m.local_halo.forward_records(recv, k, h, out=y,
                                                                                accumulate=True),
        "single-block forward": lambda: m.local.forward(*m.gather_halo_cbsr(d_l, s_l), h),
        "block selectors": lambda: m._block_sel(s_l),
        "local backward": lambda: m.local.backward(g_l, m._block_sel(s_l)),
        "whole forward": lambda: m.forward(d_l, s_l, h),
        "whole backward": lambda: m.backward(g_l, s_l),
    }
    if m.overlap:
        hsel = m._block_sel(s_l)[p.num_own:].clone()
        rows["own-column backward"] = lambda: m.local_own.backward(g_l, s_l)
        rows["halo-column backward"] = lambda: m.local_halo.backward(g_l, hsel)
    dx = m.local.backward(g_l, m._block_sel(s_l))
    back = torch.empty((m.send_rows.numel(), k), device=dev)
    rows["reverse exchange (loopback)"] = lambda: lb(back, dx[p.num_own:])
    own = dx[: p.num_own]
    rows["index_add"] = lambda: own.index_add_(0, p.send_local, back)
    rows["return (whole)"] = lambda: m._return_halo(dx)
    print(f"{graph} k={k} world={world} rank={rank}: own={p.num_own} halo={p.num_halo} "
          f"bwd algo {m.local.last_bwd_algo}; parts: own {getattr(m, 'local_own', None) and m.local_own.last_bwd_algo}"
          f" halo {getattr(m, 'local_halo', None) and m.local_halo.last_bwd_algo}")
    for name, fn in rows.items():
        print(f"  {name:36s} {timed(fn, reps=10):.3f} ms", flush=True)


def wire_table(graph="products", k=32, worlds=(4, 8), rates=(None, 0, 300, 500, 700),
               reps=20, rounds=(1,), **pm_kw):
    """Rank 0's whole step (forward + backward) with the exchanges delivered on a
    side stream behind a modeled wire (tools/wire_model.Wire: bytes received /
    rate + 10 us), so the overlap paths really overlap: rate None = the plain
    loopback (delivery inline, no wire: the step before the wire), 0 = side
    stream with no spin (the delivery copies alone), else GB/s per rank."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from wire_model import Wire
    dev = torch.device("cuda:0")
    V, E = CONFIGS[graph]
    h = 256
    indptr, indices = synthetic_csr_gpu(V, E, device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(5)
    values = torch.rand(E, generator=gen, device=dev)
    X = torch.rand((V, h), generator=gen, device=dev)
    G = torch.rand((V, h), generator=gen, device=dev)
    data, sel = topk_cbsr(X, k)
    D.PartitionedMaxK._max_over_ranks = lambda self, *xs: xs[0] if len(xs) == 1 else list(xs)
    if isinstance(worlds, int):
        worlds = (worlds,)
    if isinstance(rates, int):
        rates = (rates,)
    rates = tuple(None if r == -1 else r for r in rates)   # -1 on the command line: inline
    pm_kw = {key: (None if v == "none" else v) for key, v in pm_kw.items()}
    for key in ("overlap", "pipeline_fwd"):
        if isinstance(pm_kw.get(key), int):
            pm_kw[key] = bool(pm_kw[key])
    if isinstance(rounds, int):
        rounds = (rounds,)
    elif isinstance(rounds, str):   # "auto" / "none": PartitionedMaxK's own choice
        rounds = ("auto",)
    for world, R in [(w, r) for w in worlds for r in rounds]:
        bounds = D.row_partition(indptr, world)
        lb = Loopback(indptr, indices, bounds, 0, data, sel)
        gl = GatherLoopback(bounds, data, sel)
        D.a2a, D.ag = lb, gl
        m = D.PartitionedMaxK(indptr, indices, values, 0, world, dev, rounds=R, **pm_kw)
        d_l, s_l, g_l = m.local_rows(data), m.local_rows(sel), m.local_rows(G)
        hb = m.halo_bytes(k)
        fwd_in = hb["allgather_fwd"] if m.halo_mode == "allgather" else hb["records_fwd"]
        print(f"{graph} k={k} N={world} rank 0: own {m.plan.num_own} halo {m.plan.num_halo} "
              f"mode {m.halo_mode} overlap {m.overlap} rounds {getattr(m, 'rounds', 1)} | wire "
              f"bytes in {fwd_in / 1e6:.0f} MB fwd, {hb['reverse_bwd'] / 1e6:.0f} MB bwd", flush=True)
        for rate in rates:
            w = None if rate is None else Wire(dev, rate_GBs=rate if rate else None)
            lb.wire = gl.wire = w
            tf = timed(lambda: m.forward(d_l, s_l, h), reps=reps)
            tb = timed(lambda: m.backward(g_l, s_l), reps=reps)
            ts = timed(lambda: (m.forward(d_l, s_l, h), m.backward(g_l, s_l)), reps=reps)
            wire_ms = "" if rate in (None, 0) else \
                f" | modeled wire fwd {(fwd_in / (rate * 1e6)) + 0.01:.3f} bwd " \
                f"{hb['reverse_bwd'] / (rate * 1e6) + 0.01:.3f} ms"
            label = "inline (no wire)" if rate is None else "side stream, no spin" if rate == 0 \
                else f"{rate} GB/s"
            print(f"  {label:22s} fwd {tf:.3f} bwd {tb:.3f} step {ts:.3f} ms{wire_ms}", flush=True)
        lb.wire = gl.wire = None
        del m, lb, gl, d_l, s_l, g_l
        torch.cuda.empty_cache()


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "wire":
        kw = {}
        for a in sys.argv[3:]:
            key, val = a.split("=")
            kw[key] = (tuple(int(x) for x in val.split(",")) if "," in val else
                       int(val) if val.isdigit() else val)
        wire_table(sys.argv[2] if len(sys.argv) > 2 else "products", **kw)
    elif len(sys.argv) > 1 and sys.argv[1] == "breakdown":   # breakdown [graph] [world]
        breakdown(sys.argv[2] if len(sys.argv) > 2 else "products", 32,
                  int(sys.argv[3]) if len(sys.argv) > 3 else 8)
    elif len(sys.argv) > 1 and sys.argv[1] == "single":
        for w in [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "2,4,8").split(",")]:
            breakdown_single(sys.argv[2] if len(sys.argv) > 2 else "reddit", 32, w, 0)
    else:
        main()
