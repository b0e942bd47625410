#!/usr/bin/env python3
"""Benchmark of the MaxK-GNN aggregation hot path on MI355X.

One step = forward SpGEMM + backward SSpMM over the whole (synthetic,
Reddit-shaped by default) graph, inputs resident in HBM.  Prints ONE JSON
line on rank 0 (contract in the task statement / DESIGN.md "Measurement").

  python bench.py [--gpus N] [--steps K] [--warmup W] [--graph reddit] [--k 32] [--h 256]

N>1: launched by torch.distributed.run, one rank per GPU; the graph is 1-D
row-partitioned (nnz-balanced) and halo CBSR rows / dXs partial sums move with
RCCL all-to-all-v (spgemm_new_amd.distributed).  value = algorithmic bytes of
the WHOLE graph per step / max-over-ranks step time (strong scaling).
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--graph", default="reddit")
    p.add_argument("--k", type=int, default=32)
    p.add_argument("--h", type=int, default=256)
    p.add_argument("--seed", type=int, default=123)
    p.add_argument("--bwd-algo", default="auto",
                   choices=["auto", "atomic", "staged", "local", "tile", "staged_edge", "edge_gather"])
    p.add_argument("--panel-cost", type=int, default=None)
    p.add_argument("--row-cost", type=int, default=None)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=15.0)
    p.add_argument("--partitioned", action="store_true",
                   help="use the multi-GPU (row partition + halo exchange) path even at N=1")
    p.add_argument("--verbose", action="store_true")
    p.add_argument("--no-vendor", action="store_true",
                   help="skip the rocSPARSE (torch.sparse.mm) forward baseline")
    p.add_argument("--cbsr-order", default="column", choices=["column", "lane", "value"],
                   help="entry order the HIP top-k producer emits (any order is valid CBSR)")
    p.add_argument("--relations", type=int, default=1,
                   help="R > 1: BASELINE config 5, the fused R-relation forward "
                        "(use with --graph proteins) vs R single-relation forwards")
    return p.parse_args()


@contextlib.contextmanager
def stdout_to_stderr():
    """Send file descriptor 1 (also what native libraries write) to stderr."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_threads():
    """Host threads for the CPU baseline: every core this process may run on
    (sched_getaffinity), capped by OMP_NUM_THREADS when the launcher sets it
    (the GPU box sets it to its per-GPU CPU share)."""
    visible = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else \
        (os.cpu_count() or 1)
    cap = os.environ.get("OMP_NUM_THREADS")
    threads = min(visible, int(cap)) if cap and cap.isdigit() and int(cap) > 0 else visible
    return threads, visible, cap


def cpu_baseline(indptr, indices, values, x_masked, grad, mask, k, h, budget_s):
    """The reference's CPU aggregation path (utils/models.py:281-287:
    torch.sparse.mm(adj, x) and its mean form torch.sparse.mm(adj, x) /
    (adj.sum(1) + 1e-6)), forward and backward (A^T G * mask), on a bounded
    row sample of the same graph, timed on the host cores.  `value` is the
    sum form's fwd + bwd rate on the sample (same byte formula as the GPU
    line); the full-graph time is the sample's time scaled by E / e_sample."""
    import numpy as np
    threads, visible, cap = cpu_threads()
    torch.set_num_threads(threads)
    log(f"[bench] CPU baseline on {threads} threads ({visible} visible, OMP_NUM_THREADS={cap})")
    ip = indptr.cpu().numpy().astype(np.int64)
    V = len(ip) - 1
    E = int(ip[-1])

    def run(rows):
        e = int(ip[rows])
        a = torch.sparse_csr_tensor(torch.from_numpy(ip[: rows + 1]),
                                    indices[:e].cpu().long(), values[:e].cpu(), size=(rows, V))
        xm = x_masked
        g = grad[:rows]
        t0 = time.perf_counter()
        y = torch.sparse.mm(a, xm)                                   # forward, sum form
        t1 = time.perf_counter()
        dx = torch.sparse.mm(a.to_sparse_coo().t().coalesce(), g) * mask   # backward
        t2 = time.perf_counter()
        # mean form (utils/models.py:287): / (row sums + 1e-6); the reference adds
        # the scalar to the sparse sum, which torch 2.10 rejects -- the same math on
        # the dense row sums
        ym = torch.sparse.mm(a, xm) / (torch.sparse.sum(a.to_sparse_coo(), 1).to_dense()
                                       .unsqueeze(1) + 1e-6)
        t3 = time.perf_counter()
        del y, dx, ym
        return e, t1 - t0, t2 - t1, t3 - t2

    rows = max(1, min(V, V // 200))
    e, tf, tb, _ = run(rows)
    per_edge = (tf + tb) / max(e, 1)
    target_e = min(E, int(budget_s / 3 / max(per_edge, 1e-12)))
    rows = int(np.searchsorted(ip, target_e))
    rows = max(1, min(V, rows))
    run(rows)  # warm-up
    res = [run(rows) for _ in range(3)]
    e = res[0][0]
    tf, tb, tm = (sorted(r[i] for r in res)[1] for i in (1, 2, 3))
    nbytes = 2 * (8 * e + 5 * k * e + 4 * h * rows)
    scale = E / max(e, 1)
    return {
        "value": round(nbytes / (tf + tb) / 1e9, 3), "unit": "GB/s", "cores": threads,
        "cores_visible": visible, "kind": "reference",
        "ms_per_step_sample": round((tf + tb) * 1e3, 2),
        "fwd_ms_sample": round(tf * 1e3, 2), "bwd_ms_sample": round(tb * 1e3, 2),
        "mean_form_fwd_ms_sample": round(tm * 1e3, 2),
        "mean_form_GBs": round((nbytes / 2) / tm / 1e9, 3),
        "ms_per_step_full_graph_extrapolated": round((tf + tb) * scale * 1e3, 1),
        "sample": (f"rows [0,{rows}) of the same graph ({e} edges, {e / E:.1%} of E; full-graph "
                   f"time extrapolated x{scale:.2f} by edges): torch.sparse.mm(A,X*mask) + "
                   "torch.sparse.mm(A^T,G)*mask on CPU fp32 (sum form = value), plus the mean "
                   "form /(rowsum+1e-6), median of 3 after 1 warm-up (reference CPU path "
                   f"utils/models.py:281-287), {threads} threads"),
        "cpu_model": _cpu_model(),
    }


TRAIN_STEP_DOC = ("one MaxK-SAGE layer training step (utils/models.py:230, 242-253): top-k -> "
                  "SpGEMM -> fc_self(x) + fc_neigh(agg) (Linear h x h, hipBLASLt) -> loss <out, G> "
                  "-> backward (Linear, SSpMM, dense scatter) -> SGD step")


def train_step_fn(h, k, graph, X, G, values=None, num_rel=1):
    """One training step of a MaxK-SAGE layer (spgemm_new_amd.layers) on the
    whole graph: the aggregation op in its model context."""
    from spgemm_new_amd.layers import MaxKRelSAGELayer, MaxKSAGELayer
    torch.manual_seed(0)
    layer = (MaxKSAGELayer(h, k) if num_rel == 1 else MaxKRelSAGELayer(h, k, num_rel)).to(X.device)
    opt = torch.optim.SGD(layer.parameters(), lr=1e-3)
    x = X.clone().requires_grad_(True)

    def step():
        opt.zero_grad(set_to_none=True)
        out = layer(graph, x) if num_rel == 1 else layer(graph, x, values)
        out.backward(G)
        opt.step()
    return step


def workload_key(args, bwd_algo):
    return f"{args.graph}_h{args.h}_k{args.k}_{bwd_algo}"


def pmc_traffic(key, call, algo=None, bands=1):
    """HBM bytes of one hot-path call (`spgemm_forward` / `sspmm_backward`)
    measured by rocprofv3 PMC passes (FETCH_SIZE x2 + WRITE_SIZE,
    MI355X_MICROARCH.md §HBM) for this exact workload, from the committed
    profile summary (tools/profile.sh + tools/summarize_profile.py): per-kernel
    bytes per launch times the launches the call makes (the LOCAL backward
    launches once per source band).  None when no such profile exists."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        ent = json.load(open(path))[key]
        k = ent["kernels"]
    except (OSError, KeyError, ValueError, TypeError):
        return None, None
    fix = k.get("carry_fixup_kernel", 0.0)
    if call == "spgemm_forward":
        parts = [k.get("fwd_panel_kernel"), k.get("carry_fixup_owner_kernel", fix)]
    elif algo == "local":
        parts = [None if "bwd_local_kernel" not in k else k["bwd_local_kernel"] * bands]
    elif algo == "tile":
        parts = [k.get("bwd_tile_kernel"), k.get("tile_combine_kernel", 0.0)]
    elif algo in ("staged", "staged_edge", "edge_gather"):
        parts = [k.get("bwd_panel_kernel"), k.get("bwd_segsum_kernel"), fix]
    else:
        parts = [k.get("bwd_panel_kernel")]
    if any(p is None for p in parts):
        return None, None
    return int(sum(parts)), f"profiles/{ent['profile']}_summary.json"


def vendor_baseline(g, indptr, indices, values, X, sel, y, fwd_ms, ev_ms):
    """The dense SpMMs the reference compares its kernel with (README.md:136,
    direct_kernel_interface.py:240-269): Y = A . (X masked to its top-k) with
    the dense h-wide operand, on the same GPU and inputs, checked against our
    forward.  Two of them: our own HIP dense SpMM (the GNNAdvisor-style
    baseline, MaxKGraph.spmm_dense) and cuSPARSE's counterpart rocSPARSE
    through torch.sparse.mm."""
    V, h = X.shape
    xm = torch.zeros_like(X).scatter_(1, sel.long(), torch.gather(X, 1, sel.long()))
    out = {}
    if h % 4 == 0:
        ms = ev_ms(lambda: g.spmm_dense(xm))
        err = float(((g.spmm_dense(xm) - y).abs() / y.abs().clamp_min(1)).max())
        out["hip_dense"] = {"kind": "HIP dense SpMM (spmm_dense, merge-path panels)",
                            "fwd_ms": round(ms, 3), "speedup": round(ms / fwd_ms, 2),
                            "max_rel_diff": err}
    a = torch.sparse_csr_tensor(indptr.long(), indices.long(), values, size=(V, V))
    try:
        ms = ev_ms(lambda: torch.sparse.mm(a, xm), reps=3)
        ref = torch.sparse.mm(a, xm)
        err = float(((ref - y).abs() / ref.abs().clamp_min(1)).max())
        out.update({"kind": "rocSPARSE SpMM via torch.sparse.mm (dense masked operand)",
                    "fwd_ms": round(ms, 3), "speedup_vs_vendor": round(ms / fwd_ms, 2),
                    "max_rel_diff": err})
    except RuntimeError as e:  # a vendor path missing on this build is reported, not fatal
        out.update({"kind": "rocSPARSE SpMM via torch.sparse.mm", "error": str(e)[:200]})
    del a, xm
    return out


def bench_multi_partitioned(args, indptr, indices, vals, data, sel, V, E, h, k, R, dev, world,
                            rank, dist, gen, b_fused):
    """Config 5 on N GPUs: rows partitioned as in the single-relation path, one
    halo exchange per step shared by the R relations, the fused local forward
    (forward_multi) and the composed backward with one reverse exchange.
    value = the whole-graph fused-forward bytes / the forward time (max over
    ranks); the backward is reported beside it."""
    from spgemm_new_amd.distributed import PartitionedMaxK
    kw = {"panel_cost": args.panel_cost} if args.panel_cost else {}
    model = PartitionedMaxK(indptr, indices, vals, rank, world, dev, local_block=True, **kw)
    r0, r1 = model.bounds[rank], model.bounds[rank + 1]
    data_l, sel_l = model.local_rows(data), model.local_rows(sel)
    G_l = torch.rand((R, r1 - r0, h), generator=gen, device=dev)

    def timed(fn):
        for _ in range(args.warmup):
            fn()
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        torch.cuda.synchronize()
        dist.barrier()
        tt = torch.tensor([time.perf_counter() - t0], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt) / args.steps * 1e3
    model.forward_multi(data_l, sel_l, h)   # plans, workspaces, AUTO choice
    model.backward_multi(G_l, sel_l)
    t_f = timed(lambda: model.forward_multi(data_l, sel_l, h))
    t_b = timed(lambda: model.backward_multi(G_l, sel_l))
    val = b_fused / (t_f / 1e3) / 1e9
    b_rank = torch.tensor([float(model.algorithmic_bytes_multi(k, h))], device=dev,
                          dtype=torch.float64)
    dist.all_reduce(b_rank, op=dist.ReduceOp.MAX)
    p = model.plan
    result = {
        "metric": f"fused {R}-relation SpGEMM forward GB/s, {args.graph} h={h} k={k}",
        "value": round(val, 2), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(t_f, 4), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (power-law degrees, uniform columns, seed 123; values/X U(0,1))",
        "config": {"workload": f"{args.graph} fused multi-relation forward", "graph": args.graph,
                   "num_nodes": V, "num_edges": E, "hidden": h, "k": k, "relations": R,
                   "parallelism": f"rowpart{world}", "halo_nodes_rank0": p.num_halo,
                   "own_nodes_rank0": p.num_own},
        "roofline": {"bound": "hbm", "achieved": round(float(b_rank) / (t_f / 1e3) / 1e9, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(float(b_rank) / (t_f / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                     "traffic": None,
                     "kernel": "spgemm_forward_multi (per rank, incl. halo exchange)",
                     "algorithmic_bytes_per_launch": int(float(b_rank))},
        "bwd_multi_ms": round(t_b, 4),
    }
    if rank == 0:
        print(json.dumps(result), flush=True)


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def bench_multi(args, S, indptr, indices, data, sel, V, E, h, k, dev, world, rank=0, dist=None,
                edges=None):
    """BASELINE config 5 (ogbn-proteins, R edge-feature relations): the fused
    multi-relation forward Y[q] = A_q . X^ (one CSR + CBSR gather shared by R
    relations) timed against R single-relation forwards.  Bytes per fused call
    (SURVEY.md §8d): E*(4 + 4R + 5k) + R*4hV; unfused: R*(8E + 5kE + 4hV)."""
    from spgemm_new_amd.graphs import synthetic_values
    R = args.relations
    gen = torch.Generator(device=dev)
    gen.manual_seed(args.seed + 7)
    e0, e1 = edges or (0, E)
    # relation q's edge values: hashes of (seed + 7 + q, edge id) -> this rank's edges only
    vals = torch.stack([synthetic_values(args.seed + 7 + q, e0, e1, device=dev)
                        for q in range(R)], dim=1).contiguous()
    b_fused = E * (4 + 4 * R + 5 * k) + R * 4 * h * V
    if dist is not None:
        return bench_multi_partitioned(args, indptr, indices, vals, data, sel, V, E, h, k, R, dev,
                                       world, rank, dist, gen, b_fused)
    cols = [vals[:, q].contiguous() for q in range(R)]
    g = S.MaxKGraph(indptr, indices, cols[0])
    y = torch.empty((R, V, h), device=dev)

    def fused():
        g.forward_multi(data, sel, vals, h, out=y)

    def unfused():
        for q in range(R):
            g.forward(data, sel, h, out=y[q], values=cols[q])

    def timed(fn):
        for _ in range(args.warmup):
            fn()
        st = torch.cuda.current_stream()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(args.steps):
            fn()
        b.record(st)
        b.synchronize()
        return a.elapsed_time(b) / args.steps
    G = torch.rand((R, V, h), generator=gen, device=dev)
    dx = torch.empty((V, k), device=dev)

    def backward():
        g.backward_multi(G, sel, vals, out=dx)
    fused()
    unfused()
    backward()  # plans, workspaces and the AUTO choice before any timing
    t_f, t_u = timed(fused), timed(unfused)
    t_b = timed(backward)
    b_unf = R * (8 * E + 5 * k * E + 4 * h * V)
    val = b_fused / (t_f / 1e3) / 1e9
    X = torch.rand((V, h), generator=gen, device=dev)
    step = train_step_fn(h, k, (indptr, indices), X, G.sum(0), values=vals, num_rel=R)
    t_train = timed(step)
    del X
    result = {
        "metric": f"fused {R}-relation SpGEMM forward GB/s, {args.graph} h={h} k={k}",
        "value": round(val, 2), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(t_f, 4), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (power-law degrees, uniform columns, seed 123; values/X U(0,1))",
        "config": {"workload": f"{args.graph} fused multi-relation forward", "graph": args.graph,
                   "num_nodes": V, "num_edges": E, "hidden": h, "k": k, "relations": R,
                   "parallelism": "single"},
        "train_step_ms": round(t_train, 4),
        "train_step": (f"one {R}-relation MaxK-SAGE layer training step (spgemm_new_amd.layers."
                       "MaxKRelSAGELayer): top-k -> fused R-relation SpGEMM -> fc_self(x) + "
                       "sum_q agg_q W_q (bmm, hipBLASLt) -> loss <out, G> -> backward (bmm, "
                       "relation-interleaved SSpMM, dense scatter) -> SGD step"),
        "roofline": {"bound": "hbm", "achieved": round(val, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(val / HBM_PEAK_GBS, 4), "traffic": None,
                     "kernel": "spgemm_forward_multi", "algorithmic_bytes_per_launch": b_fused},
        "unfused_ms": round(t_u, 4), "fused_speedup": round(t_u / t_f, 3),
        "bwd_multi_ms": round(t_b, 4), "bwd_algo": g.last_bwd_algo,
        "unfused_bytes": b_unf,
    }
    print(json.dumps(result), flush=True)


def main():
    args = parse()
    import spgemm_new_amd as S
    from spgemm_new_amd import _lib
    from spgemm_new_amd.graphs import (CONFIGS, synthetic_columns, synthetic_indptr,
                                       synthetic_values)
    from spgemm_new_amd.ops import topk_cbsr

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        log(f"warning: WORLD_SIZE={world} but --gpus {args.gpus}")
    # one GPU per rank; ranks beyond the visible GPUs share them (only for the
    # BENCH_BACKEND=gloo rehearsal of the N>1 path on a one-GPU box)
    dev_index = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    dist = None
    partitioned = world > 1 or args.partitioned
    if partitioned:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        backend = os.environ.get("BENCH_BACKEND", "nccl")   # nccl = RCCL over xGMI
        # RCCL prints a version banner on stdout when its communicator starts;
        # stdout is reserved for the one JSON line, so the banner goes to stderr
        with stdout_to_stderr():
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world)
            else:  # rehearsal only: exchanges staged through host memory
                dist.init_process_group(backend, rank=rank, world_size=world)
            dist.barrier()

    V, E = CONFIGS[args.graph]
    h, k = args.h, args.k
    t0 = time.time()
    # the synthetic graph: every rank computes the (cheap) global indptr, then
    # generates only the edges of its own row block (columns and values are
    # hashes of the edge id, so the blocks are exactly rows of the N=1 graph)
    indptr = synthetic_indptr(V, E, seed=args.seed, device=dev)
    rows = None
    if partitioned:
        from spgemm_new_amd.distributed import row_partition
        b = row_partition(indptr, world)
        rows = (b[rank], b[rank + 1])
    r0, r1 = rows or (0, V)
    e0, e1 = int(indptr[r0]), int(indptr[r1])
    indices = synthetic_columns(indptr, seed=args.seed, rows=rows,
                                self_loops=(args.graph == "flickr"))
    values = synthetic_values(args.seed, e0, e1, device=dev)   # main.cu:83-84 U(0,1)
    gen = torch.Generator(device=dev)
    gen.manual_seed(args.seed + 1)
    X = torch.rand((V, h), generator=gen, device=dev)
    G = torch.rand((V, h), generator=gen, device=dev)
    data, sel = topk_cbsr(X, k, order=args.cbsr_order)  # HIP CBSR producer
    log(f"[bench] graph {args.graph} V={V} E={E}: rows [{r0}, {r1}) ({e1 - e0} edges) built "
        f"in {time.time() - t0:.1f}s")

    algo = {"auto": _lib.MAXK_BWD_AUTO, "atomic": _lib.MAXK_BWD_ATOMIC,
            "staged": _lib.MAXK_BWD_STAGED, "local": _lib.MAXK_BWD_LOCAL,
            "tile": _lib.MAXK_BWD_TILE, "staged_edge": _lib.MAXK_BWD_STAGED_EDGE,
            "edge_gather": _lib.MAXK_BWD_EDGE_GATHER}[args.bwd_algo]
    kw = {}
    if args.panel_cost:
        kw["panel_cost"] = args.panel_cost
    if args.row_cost:
        kw["row_cost"] = args.row_cost

    if args.relations > 1:
        return bench_multi(args, S, indptr, indices, data, sel, V, E, h, k, dev, world, rank,
                           dist if partitioned else None, (e0, e1))

    if partitioned:
        from spgemm_new_amd.distributed import PartitionedMaxK
        model = PartitionedMaxK(indptr, indices, values, rank, world, dev, local_block=True, **kw)
        data_l, sel_l = model.local_rows(data), model.local_rows(sel)
        G_l = model.local_rows(G)

        def step():
            y = model.forward(data_l, sel_l, h)
            dx = model.backward(G_l, sel_l)
            return y, dx
        fwd_call = bwd_call = None
        step()  # plans, workspaces and the AUTO backward choice, whatever --warmup is
    else:
        g = S.MaxKGraph(indptr, indices, values, **kw)
        y = torch.empty((V, h), device=dev)
        dx = torch.empty((V, k), device=dev)
        g.backward(G, sel, out=dx, algo=algo)  # builds CSC/workspaces once

        def fwd_call():
            g.forward(data, sel, h, out=y)

        def bwd_call():
            g.backward(G, sel, out=dx, algo=algo)

        def step():
            fwd_call()
            bwd_call()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t_el = time.perf_counter() - t_start
    if dist:
        tt = torch.tensor([t_el], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_el = float(tt)
    ms = t_el / args.steps * 1e3
    nbytes_iter = 2 * (8 * E + 5 * k * E + 4 * h * V)
    value = nbytes_iter / (ms / 1e3) / 1e9

    result = {
        "metric": "effective HBM GB/s + ms/iter, SpGEMM fwd+SSpMM bwd, Reddit h=256 k=32",
        "value": round(value, 2), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "fp32",
        "data": "synthetic (power-law degrees, uniform columns, seed 123; values/X/G U(0,1))",
        "config": {"workload": f"{args.graph} fwd SpGEMM + bwd SSpMM", "graph": args.graph,
                   "num_nodes": V, "num_edges": E, "hidden": h, "k": k,
                   "parallelism": f"rowpart{world}" if partitioned else "single",
                   "bwd_algo": args.bwd_algo},
    }

    if partitioned:
        p = model.plan
        result["config"]["halo_nodes_rank0"] = p.num_halo
        result["config"]["own_nodes_rank0"] = p.num_own
        result["config"]["overlap"] = model.overlap
        # per-call timing on each rank (HIP events on the launch stream; the
        # calls include their halo all-to-all-v), max over ranks
        st = torch.cuda.current_stream()
        fw, bw = [], []
        for _ in range(args.steps):
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            e0.record(st)
            model.forward(data_l, sel_l, h)
            e1.record(st)
            model.backward(G_l, sel_l)
            e2.record(st)
            e2.synchronize()
            fw.append(e0.elapsed_time(e1))
            bw.append(e1.elapsed_time(e2))
        b_rank = model.algorithmic_bytes(k, h)
        t = torch.tensor([sum(fw) / len(fw), sum(bw) / len(bw), float(b_rank)], device=dev,
                         dtype=torch.float64)
        if dist:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        fms, bms, b_max = float(t[0]), float(t[1]), float(t[2])
        dom = ("sspmm_backward", bms) if bms >= fms else ("spgemm_forward", fms)
        ach = b_max / (dom[1] / 1e3) / 1e9
        result["roofline"] = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                              "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                              "traffic": None, "kernel": dom[0] + " (per rank, incl. halo exchange)",
                              "algorithmic_bytes_per_launch": int(b_max)}
        result["fwd_ms"] = round(fms, 4)
        result["bwd_ms"] = round(bms, 4)
    if not partitioned:
        # per-call timing with HIP events on the launch stream (the current stream)
        st = torch.cuda.current_stream()
        fw, bw = [], []
        for _ in range(args.steps):
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            e0.record(st)
            fwd_call()
            e1.record(st)
            bwd_call()
            e2.record(st)
            e2.synchronize()
            fw.append(e0.elapsed_time(e1))
            bw.append(e1.elapsed_time(e2))
        fms, bms = sum(fw) / len(fw), sum(bw) / len(bw)
        b_call = 8 * E + 5 * k * E + 4 * h * V
        dom = ("sspmm_backward", bms) if bms >= fms else ("spgemm_forward", fms)
        ach = b_call / (dom[1] / 1e3) / 1e9
        bands = 1
        if g.last_bwd_algo == "local":
            bands = g.local_bands(g.local_plan(k), h)[1]
        traffic, tsrc = pmc_traffic(workload_key(args, g.last_bwd_algo), dom[0],
                                    g.last_bwd_algo, bands)
        result["roofline"] = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                              "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                              "traffic": traffic, "traffic_source": tsrc, "kernel": dom[0],
                              "algorithmic_bytes_per_launch": b_call,
                              "launches_per_call": bands if dom[0] == "sspmm_backward" else 1}
        # per-launch figures, directly comparable with the rocprofv3 kernel stats
        # (achieved = bytes per launch / launch average = bytes per call / call time)
        rf = result["roofline"]
        rf["algorithmic_bytes_per_call"] = b_call
        rf["algorithmic_bytes_per_launch"] = b_call // rf["launches_per_call"]
        rf["launch_avg_ms"] = round(dom[1] / rf["launches_per_call"], 4)
        if traffic is not None:
            rf["traffic_per_launch"] = traffic // rf["launches_per_call"]
        result["config"]["bwd_algo"] = g.last_bwd_algo
        # untimed parity check of the timed outputs: dx of the timed algorithm vs
        # STAGED (an independent algorithm), and the exact adjoint identity
        # <A.X^, G> = <X^_s, dXs> (fp64 sums) for the timed y and dx
        torch.cuda.synchronize()
        dx_ref = g.backward(G, sel, algo=_lib.MAXK_BWD_STAGED)
        lhs = float((y.double() * G.double()).sum())
        rhs = float((data.double() * dx.double()).sum())
        result["bwd_check"] = {
            "vs": "staged",
            "max_rel_diff": float(((dx - dx_ref).abs() / dx_ref.abs().clamp_min(1)).max()),
            "adjoint_rel_err": abs(lhs - rhs) / max(abs(lhs), 1e-30)}
        del dx_ref
        result["fwd_ms"] = round(fms, 4)
        result["bwd_ms"] = round(bms, 4)
        result["fwd_GBs"] = round(b_call / fms / 1e6, 1)
        result["bwd_GBs"] = round(b_call / bms / 1e6, 1)
        # reported separately: CBSR producer and dense-gradient scatter
        from spgemm_new_amd.ops import cbsr_scatter

        def ev_ms(fn, reps=5):  # noqa: E306
            fn()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            for _ in range(reps):
                fn()
            b.record(st)
            b.synchronize()
            return a.elapsed_time(b) / reps
        dx_tmp = torch.empty((V, k), device=dev)
        # compulsory bytes (each operand once) and the achievable
        # ceiling of a plain device copy (read + write of 1 GiB)
        result["compulsory_bytes_fwd"] = 8 * E + 5 * k * V + 4 * h * V
        src = torch.empty(1 << 28, dtype=torch.float32, device=dev)
        dst = torch.empty_like(src)
        result["copy_GBs"] = round(2 * src.numel() * 4 / ev_ms(lambda: dst.copy_(src)) / 1e6, 1)
        del src, dst
        result["topk_ms"] = round(ev_ms(lambda: topk_cbsr(X, k, order=args.cbsr_order)), 4)
        # end-to-end autograd step: SpGEMMFunction forward + backward =
        # top-k, SpGEMM, SSpMM and the dense gradient scatter
        from spgemm_new_amd.models import SpGEMMFunction
        xg = X.clone().requires_grad_(True)

        def autograd_step():
            SpGEMMFunction.apply(xg, (indptr, indices, values), k).backward(G)
        result["autograd_step_ms"] = round(ev_ms(autograd_step), 4)
        del xg
        result["train_step_ms"] = round(ev_ms(train_step_fn(h, k, (indptr, indices, values), X, G)),
                                        4)
        result["train_step"] = TRAIN_STEP_DOC
        result["scatter_ms"] = round(ev_ms(lambda: cbsr_scatter(dx_tmp, sel, h)), 4)
        if not args.no_vendor and rank == 0:
            result["vendor_baseline"] = vendor_baseline(g, indptr, indices, values, X, sel, y, fms,
                                                        ev_ms)
        if not args.no_cpu_baseline and rank == 0:
            mask = torch.zeros((V, h), device=dev)
            mask.scatter_(1, sel.long(), 1.0)
            xm = (X * mask).cpu()
            result["cpu_baseline"] = cpu_baseline(indptr, indices, values, xm, G.cpu(),
                                                  mask.cpu(), k, h, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
