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
# committed per-workload PMC results (tools/summarize_profile.py writes it)
PMC_INDEX = os.path.join(ROOT, "profiles", "pmc_traffic.json")


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
    p.add_argument("--cpu-seconds", type=float, default=40.0,
                   help="CPU-baseline budget: the whole graph when 4 runs of it fit, else "
                        "the rows holding half of E")
    p.add_argument("--partitioned", action="store_true",
                   help="use the multi-GPU (row partition + halo exchange) path even at N=1")
    p.add_argument("--verbose", action="store_true")
    p.add_argument("--auto", default="fixed", choices=["fixed", "measure"],
                   help="AUTO algorithm choice: a rule of the shape that reproduces the measured "
                        "picks on the BASELINE shapes (bitwise repeatable), or timed per graph")
    p.add_argument("--overlap", default="auto", choices=["auto", "on", "off"],
                   help="N > 1: split each rank's block into own | halo parts to hide the "
                        "exchange (auto: when the halo records reach 64 MB)")
    p.add_argument("--no-vendor", action="store_true",
                   help="skip the rocSPARSE (torch.sparse.mm) forward baseline")
    p.add_argument("--cbsr-order", default="column", choices=["column", "lane", "value"],
                   help="entry order the HIP top-k producer emits (any order is valid CBSR)")
    p.add_argument("--relations", type=int, default=1,
                   help="R > 1: BASELINE config 5, the fused R-relation forward "
                        "(use with --graph proteins) vs R single-relation forwards")
    p.add_argument("--no-configs", action="store_true",
                   help="skip the BASELINE config 1 / 3 / 5 sweep appended to the N=1 line "
                        "(Flickr on the CPU, products k in {8,16,32,64}, proteins R=8)")
    p.add_argument("--configs-only", default=None,
                   help="comma list of sweep entries to run (flickr_cpu,products_k8,...,proteins_r8)")
    p.add_argument("--config-steps", type=int, default=20,
                   help="timed steps per config entry (at least 20 by default; fewer only for "
                        "rehearsals of the plumbing)")
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


def _median(xs):
    xs = sorted(xs)
    n = len(xs)
    return 0.5 * (xs[(n - 1) // 2] + xs[n // 2]) if n else float("nan")


def cpu_threads():
    """Thread counts for the CPU baseline: os.cpu_count(), the
    cores this process may run on (sched_getaffinity) and the OMP_NUM_THREADS
    cap the launcher sets (the GPU box: its per-GPU CPU share)."""
    count = os.cpu_count() or 1
    visible = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else count
    cap = os.environ.get("OMP_NUM_THREADS")
    capped = min(visible, int(cap)) if cap and cap.isdigit() and int(cap) > 0 else visible
    return count, visible, cap, capped


def _cgroup_cpu_quota():
    """The cgroup v2 CPU quota in cores (None when unlimited or unknown)."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        return None


def cpu_baseline(indptr, indices, values, x_masked, grad, mask, k, h, budget_s):
    """The reference's CPU aggregation path (utils/models.py:281-287:
    torch.sparse.mm(adj, x) and its mean form torch.sparse.mm(adj, x) /
    (adj.sum(1) + 1e-6)), forward and backward (A^T G * mask), timed on the
    host cores.  Threads: os.cpu_count() as SURVEY.md §8d asks; when the
    launcher caps OMP_NUM_THREADS below it (the GPU box: its per-GPU share),
    both counts are probed on a small sample and the faster one times the main
    sample (both probes are in the line).  The main sample is the rows holding
    at least half of E -- the whole graph when the projected time fits the
    budget -- timed 1 warm-up + 3 runs (median), the reference's protocol
    (SURVEY.md §8d).  `value` is the sum form's fwd + bwd rate on that sample
    (same byte formula as the GPU line)."""
    import numpy as np
    count, visible, cap, capped = cpu_threads()
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

    # thread probe: a small sample (~2 % of E) per candidate count
    probe_rows = max(1, min(V, int(np.searchsorted(ip, E // 50))))
    probes = {}
    for t in sorted({count, capped}):
        torch.set_num_threads(t)
        run(probe_rows)
        e_p, tf, tb, _ = run(probe_rows)
        probes[t] = (tf + tb) / max(e_p, 1)
    threads = min(probes, key=probes.get)
    torch.set_num_threads(threads)
    log(f"[bench] CPU baseline on {threads} threads (os.cpu_count() {count}, affinity {visible}, "
        f"OMP_NUM_THREADS={cap}; probe s/edge {probes})")
    per_edge = probes[threads]
    # at least half of E; the whole graph when 4 runs of it fit the budget
    target_e = max(E // 2, min(E, int(budget_s / 4.6 / max(per_edge, 1e-12))))
    rows = max(1, min(V, int(np.searchsorted(ip, target_e))))
    run(rows)  # warm-up
    res = [run(rows) for _ in range(3)]
    e = res[0][0]
    tf, tb, tm = (sorted(r[i] for r in res)[1] for i in (1, 2, 3))
    nbytes = 2 * (8 * e + 5 * k * e + 4 * h * rows)
    scale = E / max(e, 1)
    return {
        "value": round(nbytes / (tf + tb) / 1e9, 3), "unit": "GB/s", "cores": threads,
        "os_cpu_count": count, "cores_affinity": visible, "omp_num_threads": cap,
        "cgroup_cpu_quota_cores": _cgroup_cpu_quota(),
        "thread_probe_us_per_kedge": {str(t): round(v * 1e9, 2) for t, v in probes.items()},
        "kind": "reference",
        "rows_sampled": rows, "edges_sampled": e, "edge_fraction": round(e / E, 4),
        "ms_per_step_sample": round((tf + tb) * 1e3, 2),
        "fwd_ms_sample": round(tf * 1e3, 2), "bwd_ms_sample": round(tb * 1e3, 2),
        "mean_form_fwd_ms_sample": round(tm * 1e3, 2),
        "mean_form_GBs": round((nbytes / 2) / tm / 1e9, 3),
        "ms_per_step_full_graph": round((tf + tb) * scale * 1e3, 1),
        "sample": (f"rows [0,{rows}) of the same graph ({e} edges, {e / E:.1%} of E"
                   + ("" if e == E else f"; full-graph time scaled x{scale:.3f} by edges")
                   + "): torch.sparse.mm(A,X*mask) + torch.sparse.mm(A^T,G)*mask on CPU fp32 "
                   "(sum form = value; the backward's A^T coalesce is inside its time, as in "
                   "torch's autograd of the reference op), plus the mean form /(rowsum+1e-6); "
                   "median of 3 after 1 warm-up (reference CPU path utils/models.py:281-287), "
                   f"{threads} threads (the faster of os.cpu_count()={count} and the "
                   f"OMP_NUM_THREADS cap {capped} on a 2 %-of-E probe)"),
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


KERNEL_SOURCES = ("spgemm_new_amd/csrc/maxk_spgemm.hip", "spgemm_new_amd/csrc/maxk_plan.hip",
                  "spgemm_new_amd/csrc/tile_format.h")


def kernel_source_sha(root=ROOT) -> str:
    """sha256 (16 hex) of the kernel and plan-builder sources: the key that ties a
    committed PMC profile to the code it measured (tools/summarize_profile.py
    stores it; bench.py refuses a profile whose key differs)."""
    import hashlib
    h = hashlib.sha256()
    for rel in KERNEL_SOURCES:
        with open(os.path.join(root, rel), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def pmc_traffic(key, call, algo=None, bands=1):
    """HBM bytes of one hot-path call (`spgemm_forward` / `sspmm_backward`)
    measured by rocprofv3 PMC passes (FETCH_SIZE x2 + WRITE_SIZE,
    MI355X_MICROARCH.md §HBM) for this exact workload, from the committed
    profile summary (tools/profile.sh + tools/summarize_profile.py): per-kernel
    bytes per launch times the launches the call makes (the LOCAL backward
    launches once per source band).  Returns (bytes, source, stale): bytes is
    None when no profile exists for the workload or when the profile was taken
    on other kernel sources than these (its `source_sha` differs from
    kernel_source_sha(): a stale profile is reported, never used)."""
    try:
        ent = json.load(open(PMC_INDEX))[key]
        k = ent["kernels"]
    except (OSError, KeyError, ValueError, TypeError):
        return None, None, None
    src = f"profiles/{ent['profile']}_summary.json"
    sha = ent.get("source_sha")
    if sha != kernel_source_sha():
        return None, src, {"profile": ent["profile"], "profiled_source_sha": sha,
                           "current_source_sha": kernel_source_sha(),
                           "reason": "kernel sources changed since this profile: not used"}
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
        return None, src, None
    return int(sum(parts)), src, None


# issue capacity per CU and cycle (MI355X_MICROARCH.md): one scalar instruction,
# two wave64 vector instructions (4 SIMD-32, 2 cycles each), LDS-array cycles by
# the instruction's width (ds_read_b32: 2 cycles per wave-instruction)
ISSUE_PEAK_PER_CU_CYCLE = {"SQ_INSTS_SALU": 1.0, "SQ_INSTS_VALU": 2.0, "SQ_INSTS_SMEM": 1.0}


def issue_bound(key, kernel, launch_ms, cus):
    """Issue-rate roofline of one kernel from the committed SQ counters of its
    profile (same source key as pmc_traffic): instructions of each class per
    CU-cycle against that class's peak issue rate, cycles = GRBM_GUI_ACTIVE / 8
    (the counter sums the 8 XCDs, MI355X_MICROARCH.md 'DVFS give-back'); LDS
    busy = SQ_LDS_IDX_ACTIVE (LDS-array cycles, summed over CUs) per CU-cycle.
    None without such counters."""
    try:
        ent = json.load(open(PMC_INDEX))[key]
        c = ent["issue"][kernel]
    except (OSError, KeyError, ValueError, TypeError):
        return None
    if ent.get("source_sha") != kernel_source_sha() or not c.get("GRBM_GUI_ACTIVE"):
        return None
    cycles = c["GRBM_GUI_ACTIVE"] / 8.0
    out = {"profile": ent["profile"], "kernel": kernel, "cycles": int(cycles),
           "clock_GHz": round(cycles / (c.get("avg_ms", launch_ms) * 1e6), 3) if c.get("avg_ms")
           else None}
    fr = {}
    for name, peak in ISSUE_PEAK_PER_CU_CYCLE.items():
        if name in c:
            fr[name] = round(c[name] / (cus * cycles * peak), 4)
    if "SQ_LDS_IDX_ACTIVE" in c:
        fr["SQ_LDS_IDX_ACTIVE"] = round(c["SQ_LDS_IDX_ACTIVE"] / (cus * cycles), 4)
    out["busy_frac"] = fr
    if fr:
        out["bound"] = max(fr, key=fr.get)
        out["frac"] = fr[out["bound"]]
    return out


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
        # GNNAdvisor's SAG (kernels/spmm_gnna.cu:60-140) restated for gfx950: parts of
        # E / V neighbours, one wave each, float atomics; weighted by the edge values
        # here so its output is comparable with our forward
        ms = ev_ms(lambda: g.spmm_sag(xm))
        err = float(((g.spmm_sag(xm) - y).abs() / y.abs().clamp_min(1)).max())
        out["gnna_sag"] = {"kind": "GNNAdvisor-style SAG (spmm_sag: parts of E/V neighbours, "
                                   "float atomics), edge-weighted",
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


def vendor_backward_reference(indptr, indices, values, grad, sel, num_cols=None):
    """An independent per-element reference of the backward SSpMM at any size
    (VERDICT r3): dXs_ref = (A^T . G) gathered at sel, with A^T built by torch
    (COO transpose + coalesce) and the product by rocSPARSE fp32 SpMM through
    torch.sparse.mm -- no code of this repository on the path.  Matches the
    reference kernel's math (kernels/spmm_maxk_backward.cu:15-115: dXs[c, l] =
    sum over in-edges e of c of val[e] * G[row(e), sel[c, l]])."""
    V = indptr.numel() - 1
    C = V if num_cols is None else num_cols
    e0, e1 = int(indptr[0]), int(indptr[-1])
    rows = torch.repeat_interleave(torch.arange(V, device=indptr.device),
                                   (indptr[1:] - indptr[:-1]).long(), output_size=e1 - e0)
    idx = torch.stack([indices[e0:e1].long(), rows])
    del rows
    at = torch.sparse_coo_tensor(idx, values[e0:e1], (C, V)).coalesce().to_sparse_csr()
    del idx
    full = torch.sparse.mm(at, grad)
    del at
    ref = torch.gather(full, 1, sel.long())
    del full
    return ref


def bwd_check(dx, ref, y, grad, data, staged=None):
    """The timed dx against the rocSPARSE reference (per element, |d| / max(1,
    |ref|)), the exact adjoint identity <A.X^, G> = <X^_s, dXs> (fp64 sums) and,
    when given, STAGED (another algorithm of this repository)."""
    lhs = float((y.double() * grad.double()).sum())
    rhs = float((data.double() * dx.double()).sum())
    out = {"vs": "rocsparse",
           "ref": "torch.sparse.mm(A^T, G) gathered at sel (rocSPARSE fp32 SpMM, A^T by torch)",
           "max_rel_diff": float(((dx - ref).abs() / ref.abs().clamp_min(1)).max()),
           "adjoint_rel_err": abs(lhs - rhs) / max(abs(lhs), 1e-30)}
    if staged is not None:
        out["vs_staged_max_rel_diff"] = float(((dx - staged).abs()
                                               / staged.abs().clamp_min(1)).max())
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


def _timed_calls(calls, steps, warmup):
    """Per-call HIP-event times (ms) of a step made of `calls` (functions run in
    order), on the current stream: `warmup` untimed steps, then `steps` timed
    ones; returns one list per call."""
    st = torch.cuda.current_stream()
    for _ in range(warmup):
        for fn in calls:
            fn()
    out = [[] for _ in calls]
    for _ in range(steps):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(calls) + 1)]
        ev[0].record(st)
        for i, fn in enumerate(calls):
            fn()
            ev[i + 1].record(st)
        ev[-1].synchronize()
        for i in range(len(calls)):
            out[i].append(ev[i].elapsed_time(ev[i + 1]))
    return out


def _ms_stats(xs):
    return {"mean": round(sum(xs) / len(xs), 4), "median": round(_median(xs), 4),
            "min": round(min(xs), 4)}


SWEEP_ENTRIES = ("flickr_cpu", "products_k8", "products_k16", "products_k32", "products_k64",
                 "proteins_r8")


def flickr_config1(args, dev):
    """BASELINE config 1: Flickr (89,250 nodes, 899,756 edges + self-loops, as
    scripts_train/flickr_maxk.sh:15 --selfloop; values 1), h=64, k=16 -- the
    reference's CPU aggregation path (utils/models.py:281-287: torch.sparse.mm
    sum and mean forms, and the backward A^T G * mask) timed on the host cores
    over the WHOLE graph, ms and GB/s; our GPU forward + backward of the same
    shape beside it."""
    import spgemm_new_amd as S
    from spgemm_new_amd.graphs import CONFIGS, synthetic_columns, synthetic_indptr
    from spgemm_new_amd.ops import topk_cbsr
    V, E = CONFIGS["flickr"]
    h, k = 64, 16
    indptr = synthetic_indptr(V, E, seed=args.seed, device=dev)
    indices = synthetic_columns(indptr, seed=args.seed, self_loops=True)
    values = torch.ones(indices.numel(), device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(args.seed + 1)
    X = torch.rand((V, h), generator=gen, device=dev)
    G = torch.rand((V, h), generator=gen, device=dev)
    data, sel = topk_cbsr(X, k)
    mask = torch.zeros((V, h), device=dev).scatter_(1, sel.long(), 1.0)
    cpu = cpu_baseline(indptr, indices, values, (X * mask).cpu(), G.cpu(), mask.cpu(), k, h,
                       budget_s=max(args.cpu_seconds, 20.0))
    g = S.MaxKGraph(indptr, indices, values)
    y = torch.empty((V, h), device=dev)
    dx = torch.empty((V, k), device=dev)
    g.backward(G, sel, out=dx)
    fw, bw = _timed_calls([lambda: g.forward(data, sel, h, out=y, edge_sel="auto"),
                           lambda: g.backward(G, sel, out=dx)], max(args.steps, 20),
                          max(args.warmup, 5))
    b = g.nbytes_fwd(k, h)
    cpu_fwd_ms = cpu["fwd_ms_sample"] * cpu["ms_per_step_full_graph"] / max(cpu["ms_per_step_sample"],
                                                                              1e-9)
    return {"graph": "flickr (self-loops)", "num_nodes": V, "num_edges": E, "hidden": h, "k": k,
            "algorithmic_bytes_per_call": b,
            "cpu_reference": cpu,
            "cpu_fwd_sum_form_ms": round(cpu_fwd_ms, 3),
            "cpu_fwd_sum_form_GBs": round(b / (cpu_fwd_ms / 1e3) / 1e9, 3),
            "cpu_fwd_mean_form_ms": cpu["mean_form_fwd_ms_sample"],
            "cpu_fwd_mean_form_GBs": cpu["mean_form_GBs"],
            "gpu_fwd_ms": _ms_stats(fw), "gpu_bwd_ms": _ms_stats(bw),
            "gpu_bwd_algo": g.last_bwd_algo,
            "gpu_step_GBs": round(2 * b / ((sum(fw) + sum(bw)) / len(fw) / 1e3) / 1e9, 1)}


def config_sweep(args, dev, only=None):
    """BASELINE configs 3 and 5 on this GPU, appended to the N=1 line (VERDICT r2
    item 2): ogbn-products-shaped h=256 with k in {8, 16, 32, 64} -- the k sweep of
    the reference harness (kernels/main.cu:111-116) -- and ogbn-proteins-shaped
    h=256 k=32 with R=8 relations (fused forward + multi-relation backward).
    Per entry: >= 5 warm-up steps then `steps` (>= 20) timed steps of forward +
    backward, HIP events per call; mean and median ms; fraction of the 8 TB/s
    roofline on the algorithmic bytes; the algorithms AUTO
    chose; the timed dx checked against STAGED and the exact adjoint identity."""
    import spgemm_new_amd as S
    from spgemm_new_amd import _lib
    from spgemm_new_amd.graphs import (CONFIGS, synthetic_columns, synthetic_indptr,
                                       synthetic_values)
    from spgemm_new_amd.ops import topk_cbsr
    steps, warmup = max(args.steps, 20), max(args.warmup, 5)
    h = 256
    out = {"protocol": f"{warmup} warm-up + {steps} timed steps, HIP events per call, "
                       f"AUTO algorithms (MAXK_AUTO={os.environ.get('MAXK_AUTO')}), same "
                       "synthetic generator as the headline (seed 123)"}
    want = set(only) if only else set(SWEEP_ENTRIES)
    t_all = time.time()
    if "flickr_cpu" in want:
        t0 = time.time()
        out["flickr_cpu"] = flickr_config1(args, dev)
        out["flickr_cpu"]["wall_s"] = round(time.time() - t0, 1)
        log(f"[bench] sweep flickr (config 1): CPU fwd {out['flickr_cpu']['cpu_fwd_sum_form_ms']} ms "
            f"in {time.time() - t0:.1f}s")
        torch.cuda.empty_cache()
    ks = [k for k in (8, 16, 32, 64) if f"products_k{k}" in want]
    if ks:
        V, E = CONFIGS["products"]
        t0 = time.time()
        indptr = synthetic_indptr(V, E, seed=args.seed, device=dev)
        indices = synthetic_columns(indptr, seed=args.seed)
        values = synthetic_values(args.seed, 0, E, device=dev)
        g = S.MaxKGraph(indptr, indices, values)
        gen = torch.Generator(device=dev)
        gen.manual_seed(args.seed + 1)
        X = torch.rand((V, h), generator=gen, device=dev)
        G = torch.rand((V, h), generator=gen, device=dev)
        y = torch.empty((V, h), device=dev)
        log(f"[bench] sweep: products V={V} E={E} built in {time.time() - t0:.1f}s")
        for k in ks:
            t0 = time.time()
            data, sel = topk_cbsr(X, k)
            dx = torch.empty((V, k), device=dev)
            g.backward(G, sel, out=dx)        # AUTO choice, plans, workspaces
            fw, bw = _timed_calls([lambda: g.forward(data, sel, h, out=y, edge_sel="auto"),
                                   lambda: g.backward(G, sel, out=dx)], steps, warmup)
            algo = g.last_bwd_algo
            nb = g._fwd_blocks.get((k, h), 0)
            # the non-deterministic APPEND backward, timed beside
            # the deterministic choice (min of 3 after one call; AUTO never takes it)
            from spgemm_new_amd.ops import _min_ms
            dx_a = torch.empty_like(dx)
            append_ms = round(_min_ms(lambda: g.backward(G, sel, out=dx_a,
                                                         algo=_lib.MAXK_BWD_APPEND)), 4)
            append_err = float(((dx_a - dx).abs() / dx.abs().clamp_min(1)).max())
            del dx_a
            g._append.clear()
            b = g.nbytes_fwd(k, h)
            torch.cuda.synchronize()
            dx_st = g.backward(G, sel, algo=_lib.MAXK_BWD_STAGED)
            chk = bwd_check(dx, vendor_backward_reference(indptr, indices, values, G, sel), y, G,
                            data, dx_st)
            fs, bs = _ms_stats(fw), _ms_stats(bw)
            st = [a + c for a, c in zip(fw, bw)]
            out[f"products_k{k}"] = {
                "graph": "products", "num_nodes": V, "num_edges": E, "hidden": h, "k": k,
                "fwd_ms": fs, "bwd_ms": bs, "ms_per_step": _ms_stats(st),
                "algorithmic_bytes_per_call": b,
                "fwd_frac": round(b / (fs["mean"] / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                "bwd_frac": round(b / (bs["mean"] / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                "step_GBs": round(2 * b / (sum(st) / len(st) / 1e3) / 1e9, 1),
                "bwd_algo": algo,
                "bwd_candidates_ms": getattr(g, "bwd_candidates", {}).get((k, h, True)),
                "append_bwd_ms_nondeterministic": append_ms,
                "append_vs_timed_max_rel_diff": append_err,
                "fwd_form": (f"column-blocked nb={nb}" if nb else
                                               "packed CBSR records" if k <= 16 else "plain"),
                "bwd_check": chk,
                "wall_s": round(time.time() - t0, 1)}
            log(f"[bench] sweep products k={k}: fwd {fs['mean']:.3f} bwd {bs['mean']:.3f} ms "
                f"({algo}) in {time.time() - t0:.1f}s")
            del data, sel, dx, dx_st
            # drop the per-k plans and buffers before the next k
            g._ws.clear()
            g._esel.clear()
            g._tile.clear()
            g._local.clear()
            g._blocked.clear()
            torch.cuda.empty_cache()
        del g, X, G, y, indptr, indices, values
        torch.cuda.empty_cache()
    if "proteins_r8" in want:
        t0 = time.time()
        V, E = CONFIGS["proteins"]
        R, k = 8, 32
        indptr = synthetic_indptr(V, E, seed=args.seed, device=dev)
        indices = synthetic_columns(indptr, seed=args.seed)
        vals = torch.stack([synthetic_values(args.seed + 7 + q, 0, E, device=dev)
                            for q in range(R)], dim=1).contiguous()
        g = S.MaxKGraph(indptr, indices, vals[:, 0].contiguous())
        gen = torch.Generator(device=dev)
        gen.manual_seed(args.seed + 1)
        X = torch.rand((V, h), generator=gen, device=dev)
        G = torch.rand((R, V, h), generator=gen, device=dev)
        data, sel = topk_cbsr(X, k)
        y = torch.empty((R, V, h), device=dev)
        dx = torch.empty((V, k), device=dev)
        g.forward_multi(data, sel, vals, h, out=y)
        g.backward_multi(G, sel, vals, out=dx)      # AUTO choice
        fw, bw = _timed_calls([lambda: g.forward_multi(data, sel, vals, h, out=y),
                               lambda: g.backward_multi(G, sel, vals, out=dx)], steps, warmup)
        torch.cuda.synchronize()
        algo_b = g.last_bwd_algo
        y0 = g.forward(data, sel, h, values=vals[:, 0].contiguous())
        fwd_err = float(((y[0] - y0).abs() / y0.abs().clamp_min(1)).max())
        lhs = float((y.double() * G.double()).sum())
        rhs = float((data.double() * dx.double()).sum())
        # independent per-element references (rocSPARSE through torch.sparse.mm): every
        # relation's forward A_q . X^ and the backward sum_q (A_q^T G_q) gathered at sel
        xm = torch.zeros((V, h), device=dev).scatter_(1, sel.long(), data)
        fwd_vendor, ref = 0.0, None
        for q in range(R):
            vq = vals[:, q].contiguous()
            a = torch.sparse_csr_tensor(indptr.long(), indices.long(), vq, size=(V, V))
            yq = torch.sparse.mm(a, xm)
            fwd_vendor = max(fwd_vendor, float(((y[q] - yq).abs() / yq.abs().clamp_min(1)).max()))
            del a, yq
            rq = vendor_backward_reference(indptr, indices, vq, G[q], sel)
            ref = rq if ref is None else ref.add_(rq)
            del rq, vq
        bwd_vendor = float(((dx - ref).abs() / ref.abs().clamp_min(1)).max())
        del xm, ref
        # every backward candidate, timed the same way (min of 3 after one call): the
        # fused forms and the composed one (the register and bank-ordered phase-1
        # forms, measured slower, are in the ablation build: tools/variants_lib)
        from spgemm_new_amd.ops import _min_ms
        cand_b = {}
        for nm, a in (("multi_staged", _lib.MAXK_BWD_MULTI_STAGED),
                      ("multi_edge_gather", _lib.MAXK_BWD_MULTI_EDGE_GATHER),
                      ("local_rel8", _lib.MAXK_BWD_LOCAL)):
            cand_b[nm] = round(_min_ms(lambda: g.backward_multi(G, sel, vals, out=dx, algo=a)), 4)
        cand_b["composed"] = round(_min_ms(lambda: g._backward_composed(G, sel, vals, dx,
                                                                        _lib.MAXK_BWD_AUTO)), 4)
        # the non-deterministic write-combined form, reported beside
        # the deterministic choice; AUTO never takes it (measured slower)
        cand_b["multi_append_nondeterministic"] = round(_min_ms(
            lambda: g.backward_multi(G, sel, vals, out=dx, algo=_lib.MAXK_BWD_MULTI_APPEND)), 4)
        g.forward_multi(data, sel, vals, h, out=y)
        g.backward_multi(G, sel, vals, out=dx)
        b = E * (4 + 4 * R + 5 * k) + R * 4 * h * V
        fs, bs = _ms_stats(fw), _ms_stats(bw)
        out["proteins_r8"] = {
            "graph": "proteins", "num_nodes": V, "num_edges": E, "hidden": h, "k": k,
            "relations": R, "fwd_ms": fs, "bwd_ms": bs,
            "algorithmic_bytes_per_call": b,
            "bytes_formula": "E*(4 + 4R + 5k) + R*4hV (SURVEY.md §8d, fused)",
            "fwd_frac": round(b / (fs["mean"] / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "bwd_frac": round(b / (bs["mean"] / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "bwd_algo": algo_b,
            "fwd_form": "lds (relation-vector, interleaved lanes, bank-ordered CBSR)",
            "bwd_candidates_ms": cand_b,
            "check": {"fwd_rel0_vs_single_max_rel_diff": fwd_err,
                      "fwd_vs_rocsparse_max_rel_diff": fwd_vendor,
                      "bwd_vs_rocsparse_max_rel_diff": bwd_vendor,
                      "ref": "per relation torch.sparse.mm(A_q, X^) and sum_q torch.sparse.mm"
                             "(A_q^T, G_q) gathered at sel (rocSPARSE fp32)",
                      "adjoint_rel_err": abs(lhs - rhs) / max(abs(lhs), 1e-30)},
            "wall_s": round(time.time() - t0, 1)}
        log(f"[bench] sweep proteins R=8: fwd {fs['mean']:.3f} bwd {bs['mean']:.3f} ms "
            f"in {time.time() - t0:.1f}s")
        del g, X, G, y, y0, dx, data, sel, vals, indptr, indices
        torch.cuda.empty_cache()
    out["wall_s"] = round(time.time() - t_all, 1)
    return out


def _dist_step_ms(fn, steps, warmup, dist, dev):
    """Whole-job ms per call of `fn` on every rank: `warmup` untimed calls, then
    `steps` timed ones bracketed by synchronize + barrier on both sides, the MAX
    over ranks of the elapsed time (the headline's protocol)."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    dist.barrier()
    tt = torch.tensor([time.perf_counter() - t0], device=dev, dtype=torch.float64)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    return float(tt) / steps * 1e3


def _dist_call_stats(calls, steps, dist, dev):
    """Per-call HIP-event times on each rank (_timed_calls, no extra warm-up),
    then per call the MAX over ranks of the mean and of the median (ms)."""
    ts = _timed_calls(calls, steps, 0)
    t = torch.tensor([v for xs in ts for v in (sum(xs) / len(xs), _median(xs))], device=dev,
                     dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    t = t.tolist()
    return [{"mean_max_over_ranks": round(t[2 * i], 4), "median_max_over_ranks": round(t[2 * i + 1], 4)}
            for i in range(len(calls))]


def _dist_sum(dist, dev, *xs):
    t = torch.tensor(xs, device=dev, dtype=torch.float64)
    dist.all_reduce(t)
    return t.tolist()


def partitioned_configs(args, dev, world, rank, dist, kw):
    """BASELINE configs 4 and 5 in the same N > 1 launch as the headline (VERDICT
    r4 item 1): the row-partitioned products h=256 k=32 step (config 4:
    forward + backward with their halo exchanges) and the row-partitioned
    proteins R=8 step (config 5: fused multi-relation forward + multi-relation
    backward).  Each rank builds only its own row block of the N=1 graph (hashed
    columns and values), times the step with the headline's protocol (barrier +
    synchronize both sides, max over ranks), and checks the adjoint identity
    sum_ranks <Y, G> = sum_ranks <X^_s, dXs> over the whole graph (fp64).  The
    per-graph state is freed before the next graph, so a rank's peak memory is
    one graph's."""
    from spgemm_new_amd.distributed import PartitionedMaxK, row_partition
    from spgemm_new_amd.graphs import (CONFIGS, synthetic_columns, synthetic_indptr,
                                       synthetic_values)
    from spgemm_new_amd.ops import topk_cbsr
    steps, warmup = max(args.steps, args.config_steps), max(min(args.warmup, args.config_steps), 1)
    only = set(args.configs_only.split(",")) if args.configs_only else None
    h = 256
    out = {"protocol": f"{warmup} warm-up + {steps} timed steps per graph, synchronize + barrier "
                       "on both sides, max over ranks; per-call HIP events (max over ranks of the "
                       "mean and median); same synthetic generator as N=1 (seed 123)"}

    def block(graph):
        V, E = CONFIGS[graph]
        indptr = synthetic_indptr(V, E, seed=args.seed, device=dev)
        b = row_partition(indptr, world)
        rows = (b[rank], b[rank + 1])
        e0, e1 = int(indptr[rows[0]]), int(indptr[rows[1]])
        indices = synthetic_columns(indptr, seed=args.seed, rows=rows)
        return V, E, indptr, indices, e0, e1

    if only is None or "products_k32" in only:
        t0 = time.time()
        k = 32
        V, E, indptr, indices, e0, e1 = block("products")
        values = synthetic_values(args.seed, e0, e1, device=dev)
        gen = torch.Generator(device=dev)
        gen.manual_seed(args.seed + 1)
        X = torch.rand((V, h), generator=gen, device=dev)
        G = torch.rand((V, h), generator=gen, device=dev)
        data, sel = topk_cbsr(X, k)
        del X
        model = PartitionedMaxK(indptr, indices, values, rank, world, dev, local_block=True,
                                overlap={"auto": "auto", "on": True, "off": False}[args.overlap],
                                **kw)
        data_l, sel_l, G_l = model.local_rows(data), model.local_rows(sel), model.local_rows(G)
        del data, sel, G
        res = {}

        def step():
            res["y"] = model.forward(data_l, sel_l, h)
            res["dx"] = model.backward(G_l, sel_l)
        step()   # plans, workspaces, the local AUTO choices
        ms = _dist_step_ms(step, steps, warmup, dist, dev)
        fw, bw = _dist_call_stats([lambda: model.forward(data_l, sel_l, h),
                                   lambda: model.backward(G_l, sel_l)], steps, dist, dev)
        step()
        lhs, rhs = _dist_sum(dist, dev, float((res["y"].double() * G_l.double()).sum()),
                             float((data_l.double() * res["dx"].double()).sum()))
        ex = model.exchange_ms(k)
        names = sorted(kk for kk in ex if kk.endswith("_ms"))
        t = torch.tensor([ex[kk] for kk in names], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        b_iter = 2 * (8 * E + 5 * k * E + 4 * h * V)
        p = model.plan
        out[f"products_k32_rowpart{world}"] = {
            "baseline_config": 4, "graph": "products", "num_nodes": V, "num_edges": E,
            "hidden": h, "k": k, "parallelism": f"rowpart{world}", "n_gpus": world,
            "ms_per_step": round(ms, 4), "fwd_ms": fw, "bwd_ms": bw,
            "value_GBs": round(b_iter / (ms / 1e3) / 1e9, 1),
            "value_def": "2*(8E + 5kE + 4hV) of the whole graph / ms_per_step",
            "overlap": model.overlap, "halo_mode": model.halo_mode if model.overlap else "records",
            "own_nodes_rank0": p.num_own, "halo_nodes_rank0": p.num_halo,
            "halo_bytes_rank0": model.halo_bytes(k),
            "exchange_ms_max_over_ranks": {kk: round(float(v), 4) for kk, v in zip(names, t)},
            "exchange_rounds": model.rounds,
            "local_bwd_algo_rank0": model.local.last_bwd_algo if not model.overlap else
            {"own": model.local_own.last_bwd_algo,
             "halo": (model.halo_rounds[0] if model.halo_rounds else model.local_halo).last_bwd_algo},
            "check": {"adjoint_rel_err": abs(lhs - rhs) / max(abs(lhs), 1e-30),
                      "what": "sum over ranks <Y_own, G_own> vs <X^_s own, dXs own> (fp64)"},
            "wall_s": round(time.time() - t0, 1)}
        log(f"[bench] rowpart{world} products k=32: {ms:.3f} ms/step in {time.time() - t0:.1f}s")
        del model, data_l, sel_l, G_l, res, indptr, indices, values
        torch.cuda.empty_cache()
    if only is None or "proteins_r8" in only:
        t0 = time.time()
        k, R = 32, 8
        V, E, indptr, indices, e0, e1 = block("proteins")
        vals = torch.stack([synthetic_values(args.seed + 7 + q, e0, e1, device=dev)
                            for q in range(R)], dim=1).contiguous()
        gen = torch.Generator(device=dev)
        gen.manual_seed(args.seed + 1)
        X = torch.rand((V, h), generator=gen, device=dev)
        data, sel = topk_cbsr(X, k)
        del X
        model = PartitionedMaxK(indptr, indices, vals, rank, world, dev, local_block=True, **kw)
        r0, r1 = model.bounds[rank], model.bounds[rank + 1]
        data_l, sel_l = model.local_rows(data), model.local_rows(sel)
        del data, sel
        G_l = torch.rand((R, r1 - r0, h), generator=gen, device=dev)
        res = {}

        def step():
            res["y"] = model.forward_multi(data_l, sel_l, h)
            res["dx"] = model.backward_multi(G_l, sel_l)
        step()
        ms = _dist_step_ms(step, steps, warmup, dist, dev)
        fw, bw = _dist_call_stats([lambda: model.forward_multi(data_l, sel_l, h),
                                   lambda: model.backward_multi(G_l, sel_l)], steps, dist, dev)
        step()
        lhs, rhs = _dist_sum(dist, dev, float((res["y"].double() * G_l.double()).sum()),
                             float((data_l.double() * res["dx"].double()).sum()))
        b_call = E * (4 + 4 * R + 5 * k) + R * 4 * h * V
        p = model.plan
        out[f"proteins_r8_rowpart{world}"] = {
            "baseline_config": 5, "graph": "proteins", "num_nodes": V, "num_edges": E,
            "hidden": h, "k": k, "relations": R, "parallelism": f"rowpart{world}",
            "n_gpus": world, "ms_per_step": round(ms, 4), "fwd_ms": fw, "bwd_ms": bw,
            "algorithmic_bytes_per_call": b_call,
            "bytes_formula": "E*(4 + 4R + 5k) + R*4hV (SURVEY.md §8d, fused)",
            "value_GBs": round(2 * b_call / (ms / 1e3) / 1e9, 1),
            "own_nodes_rank0": p.num_own, "halo_nodes_rank0": p.num_halo,
            "local_bwd_algo_rank0": model.local.last_bwd_algo,
            "check": {"adjoint_rel_err": abs(lhs - rhs) / max(abs(lhs), 1e-30),
                      "what": "sum over ranks and relations <Y_q, G_q> vs <X^_s, dXs> (fp64)"},
            "wall_s": round(time.time() - t0, 1)}
        log(f"[bench] rowpart{world} proteins R=8: {ms:.3f} ms/step in {time.time() - t0:.1f}s")
        del model, data_l, sel_l, G_l, res, vals, indptr, indices
        torch.cuda.empty_cache()
    return out


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


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args) -> int:
    """`python bench.py --gpus N` (N > 1) without an outside launcher: this process
    makes NO GPU call (torch.cuda.device_count() does not initialise the device on
    this image); it starts N ranks as ONE child `python -m torch.distributed.run
    --nproc-per-node N` with the same arguments, relays rank 0's JSON line and
    returns non-zero when N exceeds the visible devices (RCCL: one GPU per rank),
    when any rank fails, or when the line's n_gpus is not N.  BENCH_BACKEND=gloo
    (a rehearsal of the N > 1 logic) may share GPUs between ranks."""
    import subprocess
    n = args.gpus
    backend = os.environ.get("BENCH_BACKEND", "nccl")
    visible = torch.cuda.device_count()
    if backend == "nccl" and n > visible:
        log(f"[bench] --gpus {n} but {visible} GPU(s) visible: refusing (one GPU per rank)")
        return 3
    if visible < 1:
        log("[bench] no GPU visible")
        return 3
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", port, os.path.abspath(__file__),
           *sys.argv[1:]]
    log(f"[bench] launching {n} ranks: {' '.join(cmd)}")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, env=env, text=True)
    lines = [ln for ln in proc.stdout.splitlines() if ln.startswith("{")]
    for ln in proc.stdout.splitlines():
        if not ln.startswith("{"):
            log(ln)
    if proc.returncode != 0:
        log(f"[bench] a rank failed (torch.distributed.run rc={proc.returncode})")
        return proc.returncode or 1
    if len(lines) != 1:
        log(f"[bench] expected one JSON line from rank 0, got {len(lines)}")
        return 4
    try:
        d = json.loads(lines[0])
    except ValueError:
        log("[bench] rank 0's line is not JSON")
        return 4
    if d.get("n_gpus") != n:
        log(f"[bench] rank 0 reports n_gpus={d.get('n_gpus')} for --gpus {n}")
        return 5
    print(lines[0], flush=True)
    return 0


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus:
        # a launcher that started another number of ranks than --gpus asks for
        log(f"[bench] WORLD_SIZE={world_env} but --gpus {args.gpus}: refusing")
        sys.exit(6)
    # the algorithm choices (forward column blocks, backward algorithm): by rule of the
    # shape (default; the same choices, summation order and bits on every box) or timed
    os.environ.setdefault("MAXK_AUTO", args.auto)
    import spgemm_new_amd as S
    from spgemm_new_amd import _lib
    from spgemm_new_amd.graphs import (CONFIGS, synthetic_columns, synthetic_indptr,
                                       synthetic_values)
    from spgemm_new_amd.ops import topk_cbsr

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
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
        ov = {"auto": "auto", "on": True, "off": False}[args.overlap]
        model = PartitionedMaxK(indptr, indices, values, rank, world, dev, local_block=True,
                                overlap=ov, **kw)
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

        from spgemm_new_amd.ops import _ESEL_ALGOS
        # a training forward: its backward follows with this sel (an explicitly chosen
        # edge-selector backward makes every forward write the edge selectors)
        esel_mode = True if algo in _ESEL_ALGOS else "auto"

        def fwd_call():
            g.forward(data, sel, h, out=y, edge_sel=esel_mode)

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
                   "bwd_algo": args.bwd_algo, "auto_mode": os.environ.get("MAXK_AUTO")},
    }

    if partitioned:
        p = model.plan
        result["config"]["halo_nodes_rank0"] = p.num_halo
        result["config"]["own_nodes_rank0"] = p.num_own
        result["config"]["overlap"] = model.overlap
        # the all-gather table path exists only with the own | halo split
        result["config"]["halo_mode"] = model.halo_mode if model.overlap else "records"
        result["config"]["halo_bytes_rank0"] = model.halo_bytes(k)
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
        med = torch.tensor([_median([a + b for a, b in zip(fw, bw)]), _median(fw), _median(bw)],
                           device=dev, dtype=torch.float64)
        if dist:
            dist.all_reduce(med, op=dist.ReduceOp.MAX)
        result["ms_per_step_median"] = round(float(med[0]), 4)
        result["fwd_ms_median"] = round(float(med[1]), 4)
        result["bwd_ms_median"] = round(float(med[2]), 4)
        dom = ("sspmm_backward", bms) if bms >= fms else ("spgemm_forward", fms)
        ach = b_max / (dom[1] / 1e3) / 1e9
        result["roofline"] = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                              "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                              "traffic": None, "kernel": dom[0] + " (per rank, incl. halo exchange)",
                              "algorithmic_bytes_per_launch": int(b_max)}
        result["fwd_ms"] = round(fms, 4)
        result["bwd_ms"] = round(bms, 4)
        # each exchange alone on the wire (HIP events around the synchronous
        # collective, step-sized messages), max over ranks; the step overlaps them
        # with compute where it can
        ex = model.exchange_ms(k)
        names = sorted(kk for kk in ex if kk.endswith("_ms"))
        t = torch.tensor([ex[kk] for kk in names], device=dev, dtype=torch.float64)
        if dist:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        result["exchange_ms_max_over_ranks"] = {kk: round(float(v), 4) for kk, v in zip(names, t)}
        result["exchange_bytes_rank0"] = {kk: v for kk, v in ex.items() if not kk.endswith("_ms")}
        result["local_bwd_algo_rank0"] = model.local.last_bwd_algo if not model.overlap else \
            {"own": model.local_own.last_bwd_algo,
             "halo": (model.halo_rounds[0] if model.halo_rounds else model.local_halo).last_bwd_algo}
        result["exchange_rounds"] = model.rounds
        if dist and not args.no_configs and args.graph == "reddit":
            # configs 4 and 5 in the same launch (the driver's scaling runs are
            # `bench.py --gpus N`): the Reddit state is freed first
            del model, data_l, sel_l, G_l, X, G, data, sel, indices, values
            torch.cuda.empty_cache()
            result["configs"] = partitioned_configs(args, dev, world, rank, dist, kw)
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
        wkey = workload_key(args, g.last_bwd_algo)
        traffic, tsrc, stale = pmc_traffic(wkey, dom[0], g.last_bwd_algo, bands)
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
        rf["source_sha"] = kernel_source_sha()
        if stale is not None:
            rf["traffic_stale"] = stale
        if traffic is not None:
            rf["traffic_per_launch"] = traffic // rf["launches_per_call"]
            # what the counters say the kernel really moves: fabric bytes / time / peak
            rf["traffic_GBs"] = round(traffic / (dom[1] / 1e3) / 1e9, 1)
            rf["traffic_frac"] = round(rf["traffic_GBs"] / HBM_PEAK_GBS, 4)
        main_kernel = {"tile": "bwd_tile_kernel", "local": "bwd_local_kernel"}.get(
            g.last_bwd_algo, "bwd_panel_kernel") if dom[0] == "sspmm_backward" else "fwd_panel_kernel"
        cus = torch.cuda.get_device_properties(dev).multi_processor_count
        iss = issue_bound(wkey, main_kernel, rf["launch_avg_ms"], cus)
        if iss is not None:
            rf["issue"] = iss
        steps_ms = sorted(a + b for a, b in zip(fw, bw))
        result["ms_per_step_median"] = round(_median(steps_ms), 4)
        result["ms_per_step_events_mean"] = round(sum(steps_ms) / len(steps_ms), 4)
        result["fwd_ms_median"] = round(_median(fw), 4)
        result["bwd_ms_median"] = round(_median(bw), 4)
        result["config"]["bwd_algo"] = g.last_bwd_algo
        # untimed parity check of the timed outputs: dx of the timed algorithm vs
        # rocSPARSE's A^T G gathered at sel (independent of this repository), vs
        # STAGED, and the exact adjoint identity <A.X^, G> = <X^_s, dXs> (fp64 sums)
        torch.cuda.synchronize()
        dx_st = g.backward(G, sel, algo=_lib.MAXK_BWD_STAGED)
        result["bwd_check"] = bwd_check(dx, vendor_backward_reference(indptr, indices, values, G,
                                                                      sel), y, G, data, dx_st)
        del dx_st
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
        if not args.no_configs and args.graph == "reddit" and rank == 0:
            only = args.configs_only.split(",") if args.configs_only else None
            result["configs"] = config_sweep(args, dev, only)
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
