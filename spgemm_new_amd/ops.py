"""Host-side API of the MI355X MaxK aggregation path.

``MaxKGraph`` owns a CSR adjacency resident in HBM plus everything the kernels
need that the reference kept in files or rebuilt per call:

* the merge-path panel schedule (replaces the ``.warp4`` file of
  kernels/generate_meta.py:26-48, read per call at spmm_maxk.cu:117);
* the CSC transpose (edge -> CSC slot, CSC row pointer and its own panel
  schedule) used by the STAGED backward;
* the LOCAL backward plan (destination ranges, in-edges sorted by source row,
  source bands) and the measured AUTO backward choice;
* cached workspaces (carry rows, staging rows, packed CBSR records).

Also here: the CBSR producer (top-k), the dense gradient scatter / MaxK mask,
the fused multi-relation forward, and the halo records of the multi-GPU path
(packed CBSR rows read in place, accumulating forward).

All compute goes through the C ABI (``_lib``); there is no CPU or PyTorch
fallback for the kernels.  The plans (panel schedules, CSC transpose, LOCAL
ranges and bands) are built once per graph by the library's device builders
(csrc/maxk_plan.hip); torch only allocates.
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _lib

__all__ = ["MaxKGraph", "check_tensor", "spgemm_forward", "spgemm_forward_multi",
           "spgemm_forward_records", "cbsr_gather_records", "sspmm_backward", "spmm_dense",
           "warp4_build", "topk_cbsr", "cbsr_scatter", "cbsr_mask"]


def check_tensor(t, name: str, dtype=None, cuda: bool = True, dim: int | None = None):
    """TORCH_CHECK-style validation (cuda_kernel_bindings.cpp:52-62)."""
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if cuda and not t.is_cuda:
        raise RuntimeError(f"{name} must be CUDA tensor")
    if dtype is not None and t.dtype != dtype:
        raise RuntimeError(f"{name} must be {str(dtype).replace('torch.', '')}")
    if dim is not None and t.dim() != dim:
        raise RuntimeError(f"{name} must be {dim}D tensor")
    if not t.is_contiguous():
        raise RuntimeError(f"{name} must be contiguous")
    return t


def _stream(t):
    return _lib.stream_ptr(t.device)


def _tensor_key(t):
    return (t.data_ptr(), t.numel(), t._version)


# LOCAL backward: target LDS bytes per wave (16 waves per CU share 160 KiB)
LOCAL_WAVE_LDS_BYTES = int(os.environ.get("MAXK_LOCAL_WAVE_LDS", 10 * 1024))
LOCAL_WAVES_PER_CU = int(os.environ.get("MAXK_LOCAL_WAVES_PER_CU", 16))
# LOCAL backward: gradient-row bytes per source band (one launch each); about 32 MB keeps a
# band's G rows resident in the Infinity Cache (tools/exp_local_window.py)
LOCAL_BAND_BYTES = int(os.environ.get("MAXK_LOCAL_BAND_BYTES", 32 << 20))
# AUTO backward: timed calls per candidate (the minimum decides)
AUTOTUNE_REPS = int(os.environ.get("MAXK_AUTOTUNE_REPS", 3))
# panel schedule: at least this many panels (waves) per graph when the default
# 2048-cost panels would give fewer
MIN_PANELS = int(os.environ.get("MAXK_MIN_PANELS", 16384))
# TILE backward among the AUTO candidates (k = 32, h = 256)
TILE_AUTO = os.environ.get("MAXK_TILE", "1") != "0"
# STAGED_EDGE backward (edge selectors written by the forward) among the AUTO candidates
ESEL_AUTO = os.environ.get("MAXK_ESEL", "1") != "0"
# MAXK_AUTO=fixed takes STAGED_EDGE at k = 32 only when the selector table (num_cols * k
# bytes) is at least this large: smaller tables keep STAGED's per-edge selector reads in
# the caches (products rank blocks at N = 2 / 4, 39 / 20 MB: STAGED 3.74 / 1.33 ms vs
# STAGED_EDGE 3.88 / 1.48 fwd + bwd; products N = 1, 78 MB: STAGED_EDGE)
ESEL_MIN_SEL_BYTES = int(os.environ.get("MAXK_ESEL_MIN_SEL_BYTES", 64 << 20))
# AUTO backward: "measure" (time the candidates once per graph and shape; the fastest
# is kept) or "fixed" (a rule of the shape alone, no timing: the same algorithm on every
# run and machine, and so the same fp32 summation order on every run of one machine;
# TILE's source-range count follows the device's CU count, so across machines with
# different CU counts TILE's partial sums may group differently)
AUTO_MODE = os.environ.get("MAXK_AUTO", "measure")
# MAXK_AUTO=fixed: the CU count its TILE rank-block rule is stated in (MI355X)
FIXED_RULE_CUS = 256
# MAXK_DETERMINISTIC=1: AUTO never takes an algorithm whose fp32 sum order follows
# arrival order (ATOMIC; APPEND is never an AUTO candidate: measured slower)
DETERMINISTIC = os.environ.get("MAXK_DETERMINISTIC", "0") == "1"
# edge-selector buffers kept per graph (one per live selector tensor: a forward
# per layer before the backwards)
ESEL_CACHE = int(os.environ.get("MAXK_ESEL_CACHE", 4))


def tile_shape_ok(dim_k: int, dim_origin: int) -> bool:
    return dim_k in (32, 64) and dim_origin == 256
# forward at k in {4, 8, 16}: pack CBSR into one record per node (MAXK_FWD_PACKED=0 disables)
FWD_PACKED = os.environ.get("MAXK_FWD_PACKED", "1") != "0"
# column-blocked forward (k >= 32): MAXK_FWD_BLOCKS = -1 (default) measures it against
# the plain forward once per (k, h) on graphs whose mean degree reaches
# FWD_BLOCKED_MIN_DEGREE; 0 never; n > 0 always, with n column blocks
FWD_BLOCKS = int(os.environ.get("MAXK_FWD_BLOCKS", "-1"))
FWD_BLOCKED_MIN_DEGREE = 128
FWD_BLOCKED_CANDIDATES = (3, 4, 6, 8)  # Reddit: 4 best at k = 32 and 64
# fused multi-relation forward: reorder CBSR entries against LDS store conflicts
MULTI_BANK_ORDER = os.environ.get("MAXK_MULTI_BANK_ORDER", "1") != "0"
# (the register-accumulator and bank-ordered multi-relation forms and the BINNED
# backward, all measured slower, live in the ablation build: tools/variants_lib)


def _build_schedule(indptr: torch.Tensor, num_rows: int, num_edges: int, panel_cost: int,
                    row_cost: int):
    L = _lib.load()
    import ctypes
    n = ctypes.c_int64(0)
    _lib.check(L.maxk_schedule_num_panels(num_rows, num_edges, panel_cost, row_cost,
                                          ctypes.byref(n)), "maxk_schedule_num_panels")
    P = int(n.value)
    sched = torch.empty(2 * (P + 1), dtype=torch.int32, device=indptr.device)
    _lib.check(L.maxk_schedule_build(indptr.data_ptr(), num_rows, panel_cost, row_cost,
                                     sched.data_ptr(), P, _stream(indptr)), "maxk_schedule_build")
    return sched, P


def _validate_csr(indptr: torch.Tensor, indices: torch.Tensor, num_cols: int) -> None:
    """One-time device check that the kernels will stay in bounds: indptr
    non-decreasing within [0, E], and the referenced columns in [0, num_cols).
    (The reference kernels do not check; an out-of-range index there reads
    out of bounds.)  One O(E) reduction and one host sync per graph."""
    E = indices.numel()
    if indptr.numel() == 0:
        raise RuntimeError("indptr must have at least one element")
    lo, hi = indptr[0], indptr[-1]
    checks = [lo < 0, hi > E, (indptr[1:] < indptr[:-1]).any() if indptr.numel() > 1
              else torch.zeros((), dtype=torch.bool, device=indptr.device)]
    bad_cols = torch.zeros((), dtype=torch.bool, device=indptr.device)
    if E > 0:
        e0, e1 = int(lo.clamp(0, E)), int(hi.clamp(0, E))
        if e1 > e0:
            mn, mx = torch.aminmax(indices[e0:e1])
            bad_cols = (mn < 0) | (mx >= num_cols)
    flags = torch.stack([c.reshape(()).bool() for c in checks] + [bad_cols]).tolist()
    if flags[0] or flags[1]:
        raise RuntimeError(f"indptr out of range: must satisfy 0 <= indptr[0] <= indptr[-1] <= {E}")
    if flags[2]:
        raise RuntimeError("indptr must be non-decreasing")
    if flags[3]:
        raise RuntimeError(f"indices out of range: every column must be in [0, {num_cols})")


_ESEL_ALGOS = (_lib.MAXK_BWD_STAGED_EDGE, _lib.MAXK_BWD_EDGE_GATHER, _lib.MAXK_BWD_APPEND_EDGE)
# non-deterministic algorithms (the sum order follows the arrival order of the
# products, as the reference's atomicAdd K2): never chosen under MAXK_DETERMINISTIC=1
_NONDET_ALGOS = (_lib.MAXK_BWD_ATOMIC, _lib.MAXK_BWD_APPEND, _lib.MAXK_BWD_APPEND_EDGE)


_ALGO_NAMES = {_lib.MAXK_BWD_ATOMIC: "atomic", _lib.MAXK_BWD_STAGED: "staged",
               _lib.MAXK_BWD_LOCAL: "local", _lib.MAXK_BWD_TILE: "tile",
               _lib.MAXK_BWD_STAGED_EDGE: "staged_edge", _lib.MAXK_BWD_EDGE_GATHER: "edge_gather",
               _lib.MAXK_BWD_APPEND: "append", _lib.MAXK_BWD_APPEND_EDGE: "append_edge"}


def _edge_gather_ok(k: int) -> bool:
    return 4 <= k <= 256 and k & (k - 1) == 0


_append_ok = _edge_gather_ok   # APPEND: k a power of two in [4, 256] as well


def _min_ms(fn, reps: int | None = None) -> float:
    """fn's minimum time over a few calls (HIP events on the current stream),
    after one untimed call."""
    fn()
    ms = float("inf")
    for _ in range(AUTOTUNE_REPS if reps is None else reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ms = min(ms, e0.elapsed_time(e1))
    return ms


class MaxKGraph:
    """A CSR graph on one GPU, ready for the MaxK SpGEMM / SSpMM kernels.

    Parameters mirror the reference's graph tuple ``(indptr, indices, values)``
    (utils/models.py:67, 227); ``values`` defaults to ones (sum aggregation, as
    in training, utils/models.py:227).

    Every call runs asynchronously on the current stream and reuses the graph's
    cached workspaces (carry slots, staging rows, edge selectors, TILE partial
    planes), so the calls on one graph must be ordered on one stream; work on
    several streams at once needs one MaxKGraph per stream.
    """

    def __init__(self, indptr: torch.Tensor, indices: torch.Tensor,
                 values: torch.Tensor | None = None, *, panel_cost: int | None = None,
                 row_cost: int = _lib.DEFAULT_ROW_COST, bwd_panel_cost: int | None = None,
                 csc_panel_cost: int | None = None, num_cols: int | None = None,
                 validate: bool = True, tile_splits: int | None = None):
        check_tensor(indptr, "indptr", torch.int32, dim=1)
        check_tensor(indices, "indices", torch.int32, dim=1)
        if values is None:
            values = torch.ones(indices.numel(), dtype=torch.float32, device=indices.device)
        check_tensor(values, "values", torch.float32, dim=1)
        if values.numel() != indices.numel():
            raise RuntimeError("values and indices must have the same length")
        if indptr.device != indices.device or values.device != indices.device:
            raise RuntimeError("graph tensors must be on the same device")
        self.num_rows = indptr.numel() - 1
        # A may be rectangular (a multi-GPU rank's row block with halo columns)
        self.num_cols = self.num_rows if num_cols is None else int(num_cols)
        if validate:
            _validate_csr(indptr, indices, self.num_cols)
        # a row slice of a bigger CSR (indptr[0] != 0, or fewer edges than indices
        # holds) is rebased once: the graph's edges are indices[indptr[0]:indptr[-1]],
        # and every plan (CSC, LOCAL) and per-call values array refers to those
        base, end = (int(v) for v in indptr[[0, -1]].tolist()) if indptr.numel() > 0 else (0, 0)
        # the caller's tensors stay referenced: graph caches key on their storage
        # addresses, which must not be reused while this graph lives
        self._src = (indptr, indices, values)
        if base != 0 or end != indices.numel():
            indptr = (indptr - base).contiguous()
            indices = indices[base:end]
            values = values[base:end]
        self.num_edges = indices.numel()
        if self.num_edges == 0:  # the C ABI wants valid pointers even for an empty edge list
            indices = torch.zeros(1, dtype=torch.int32, device=indices.device)
            values = torch.zeros(1, dtype=torch.float32, device=indices.device)
        self.indptr, self.indices, self.values = indptr, indices, values
        self.device = indices.device
        if panel_cost is None:
            # 2048 (MAXK_DEFAULT_PANEL_COST) for big graphs; smaller panels when
            # that would leave fewer than MIN_PANELS waves (a rank's block, a
            # small graph): the own-column block of a Reddit rank at N=8 took
            # 0.137 ms with 2048-cost panels, 0.089 ms with >= 16 K panels
            cost = self.num_edges + row_cost * self.num_rows
            want = max(1, cost // max(MIN_PANELS, 1))
            # rounded to the NEAREST power of two: rank blocks of Reddit measured
            # slower at the in-between costs (N=4: 1805 -> 0.77 ms vs 2048 -> 0.65 ms
            # column-blocked forward; N=8: 903 -> 0.42 ms vs 1024 -> 0.35 ms;
            # tools/exp_rank_fwd.py, round 4)
            p2 = 1 << max(0, want.bit_length() - 1)
            if want - p2 > 2 * p2 - want:
                p2 *= 2
            panel_cost = int(min(_lib.DEFAULT_PANEL_COST, max(256, p2)))
        self.panel_cost, self.row_cost = panel_cost, row_cost
        self.sched, self.num_panels = _build_schedule(indptr, self.num_rows, self.num_edges,
                                                      panel_cost, row_cost)
        if bwd_panel_cost is not None and bwd_panel_cost != panel_cost:
            self.bwd_sched, self.bwd_num_panels = _build_schedule(
                indptr, self.num_rows, self.num_edges, bwd_panel_cost, row_cost)
        else:
            self.bwd_sched, self.bwd_num_panels = self.sched, self.num_panels
        self.csc_panel_cost = csc_panel_cost or panel_cost
        self._csc = None
        self._local = {}
        self._tile = {}
        self._append = {}
        # TILE source ranges (None: enough to fill the CUs); 1 makes each
        # destination's sum one sequential FMA chain in source-row order, the same
        # bits whatever other columns the graph holds (tests of the row partition)
        self.tile_splits = tile_splits
        self._ws = {}
        self._bwd_choice = {}
        self._multi_timings = {}  # ((multi key), algo) -> ms, AUTO's backward_multi timings
        self._bwd_alt = {}        # AUTO's best algorithm other than STAGED_EDGE, per key
        self._esel_on = set()     # (k, h): forwards write edge selectors (AUTO chose STAGED_EDGE)
        self._esel = []           # [(sel key, sel, uint8 buffer[E * k], pinned)], most recent last
        self.last_bwd_algo = None
        self._blocked = {}        # column-blocked forward plans, per block count
        self._fwd_blocks = {}     # (k, h) -> block count chosen (0: plain forward)

    # ------------------------------------------------------------------ utils
    def _workspace(self, key, nbytes: int) -> torch.Tensor:
        t = self._ws.get(key)
        if t is None or t.numel() < nbytes:
            t = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=self.device)
            self._ws[key] = t
        return t

    def blocked_plan(self, num_blocks: int) -> dict:
        """The CSR restacked block-major for the column-blocked forward: row
        b * V + r holds row r's edges whose source column lies in block b of
        num_blocks (equal column ranges), in CSR order; built once.  The sweep
        then reads one block's CBSR rows at a time, from L2 (include/maxk_spgemm.h,
        maxk_rows_sum)."""
        plan = self._blocked.get(num_blocks)
        if plan is None:
            V, C, nb, E = self.num_rows, self.num_cols, num_blocks, self.num_edges
            L = _lib.load()
            indptr = torch.empty(nb * V + 1, dtype=torch.int32, device=self.device)
            indices = torch.empty(E, dtype=torch.int32, device=self.device)
            order = torch.empty(E, dtype=torch.int32, device=self.device)
            ws = torch.empty(max(1, L.maxk_blocked_plan_workspace_bytes(E, V, nb)), dtype=torch.uint8,
                             device=self.device)
            _lib.check(L.maxk_blocked_plan_build(self.indptr.data_ptr(), self.indices.data_ptr(), None,
                                                 V, C, E, nb, indptr.data_ptr(), indices.data_ptr(),
                                                 None, order.data_ptr(), ws.data_ptr(), ws.numel(),
                                                 _stream(indptr)), "maxk_blocked_plan_build")
            del ws
            sched, P = _build_schedule(indptr, nb * V, E, self.panel_cost, self.row_cost)
            plan = {"num_blocks": nb, "order": order, "indptr": indptr, "indices": indices,
                    "sched": sched, "num_panels": P, "values": None, "values_key": None}
            _blocked_split(self, plan)
            self._blocked[num_blocks] = plan
        return plan

    def _blocked_values(self, plan: dict, values: torch.Tensor) -> torch.Tensor:
        """values in the plan's edge order (maxk_permute_f32): kept for the
        graph's own values (refreshed when they change in place; always re-gathered
        under hipGraph capture), gathered per call for others."""
        L = _lib.load()

        def permute(dst):
            _lib.check(L.maxk_permute_f32(values.data_ptr(), plan["order"].data_ptr(),
                                          self.num_edges, dst.data_ptr(), _stream(dst)),
                       "maxk_permute_f32")
            return dst
        if values is not self.values:
            return permute(torch.empty(self.num_edges, dtype=torch.float32, device=self.device))
        key = _tensor_key(values)
        capturing = torch.cuda.is_current_stream_capturing()
        if plan["values"] is None:
            plan["values"] = torch.empty(self.num_edges, dtype=torch.float32, device=self.device)
            plan["values_key"] = None
        if capturing or plan["values_key"] != key:
            permute(plan["values"])
            plan["values_key"] = key
        return plan["values"]

    def csc(self):
        """(csc_pos, csc_indptr, csc_sched, csc_num_panels), built once on the
        device (maxk_csc_build: stable radix sort of the columns)."""
        if self._csc is None:
            L = _lib.load()
            E, C = self.num_edges, self.num_cols
            csc_pos = torch.empty(max(E, 1), dtype=torch.int32, device=self.device)
            csc_indptr = torch.empty(C + 1, dtype=torch.int32, device=self.device)
            ws = torch.empty(max(1, L.maxk_csc_workspace_bytes(E, C)), dtype=torch.uint8,
                             device=self.device)
            _lib.check(L.maxk_csc_build(self.indices.data_ptr(), E, C, csc_indptr.data_ptr(),
                                        csc_pos.data_ptr(), ws.data_ptr(), ws.numel(),
                                        _stream(csc_pos)), "maxk_csc_build")
            del ws
            sched, P = _build_schedule(csc_indptr, C, E, self.csc_panel_cost, self.row_cost)
            self._csc = (csc_pos, csc_indptr, sched, P)
        return self._csc

    def csc_perm(self) -> torch.Tensor:
        """CSC slot -> CSR edge (the inverse of csc_pos; MAXK_BWD_EDGE_GATHER), once."""
        if getattr(self, "_csc_perm", None) is None:
            csc_pos = self.csc()[0]
            perm = torch.empty(max(self.num_edges, 1), dtype=torch.int32, device=self.device)
            _lib.check(_lib.load().maxk_csc_perm_build(csc_pos.data_ptr(), self.num_edges,
                                                       perm.data_ptr(), _stream(perm)),
                       "maxk_csc_perm_build")
            self._csc_perm = perm
        return self._csc_perm

    def local_plan(self, dim_k: int):
        """Plan of the LOCAL backward (maxk_sspmm_backward_local), or None when
        the shape does not suit it.  Destinations are cut into ranges of at
        most dmax nodes balanced by in-degree; each range's in-edges are listed
        in source-row order.  Built on the device (maxk_local_plan_build; one
        host read of the range count)."""
        if dim_k in self._local:
            plan = self._local[dim_k]
            # under capture the gather is always recorded: replays see the graph's
            # values as they are then, also after an in-place change
            if plan is not None and (plan["values_key"] != _tensor_key(self.values)
                                     or torch.cuda.is_current_stream_capturing()):
                plan["edge_val"] = self.values[: self.num_edges][plan["perm"].long()].contiguous()
                plan["values_key"] = _tensor_key(self.values)
            return plan
        plan = None
        V, E = self.num_cols, self.num_edges      # V: destinations (columns of A)
        if E > 0 and self.num_rows < (1 << 24) and 64 % dim_k == 0:
            import ctypes
            L = _lib.load()
            dmax = max(1, min(256, LOCAL_WAVE_LDS_BYTES // (5 * dim_k)))
            _, csc_indptr, _, _ = self.csc()
            cus = torch.cuda.get_device_properties(self.device).multi_processor_count
            T = max(-(-V // dmax), min(cus * LOCAL_WAVES_PER_CU, V))
            ws = torch.empty(max(1, L.maxk_local_plan_workspace_bytes(E, V, T)),
                             dtype=torch.uint8, device=self.device)
            st = _stream(ws)
            n = ctypes.c_int32(0)
            args = (self.indptr.data_ptr(), self.indices.data_ptr(), self.values.data_ptr(),
                    self.num_rows, V, E, csc_indptr.data_ptr(), dmax, T)
            _lib.check(L.maxk_local_plan_build(*args, None, None, None, None, None,
                                               ctypes.byref(n), ws.data_ptr(), ws.numel(), st),
                       "maxk_local_plan_build(count)")
            W = int(n.value)
            i32 = dict(dtype=torch.int32, device=self.device)
            dstart, woff = torch.empty(W + 1, **i32), torch.empty(W + 1, **i32)
            erc, perm = torch.empty(E, **i32), torch.empty(E, **i32)
            ev = torch.empty(E, dtype=torch.float32, device=self.device)
            _lib.check(L.maxk_local_plan_build(*args, dstart.data_ptr(), woff.data_ptr(),
                                               erc.data_ptr(), perm.data_ptr(), ev.data_ptr(),
                                               ctypes.byref(n), ws.data_ptr(), ws.numel(), st),
                       "maxk_local_plan_build")
            del ws
            plan = {"dmax": dmax, "num_waves": W, "dstart": dstart, "woff": woff,
                    "edge_rc": erc, "perm": perm, "bands": {}, "edge_val": ev,
                    "values_key": _tensor_key(self.values)}
        self._local[dim_k] = plan
        return plan

    def local_bands(self, plan, dim_origin: int):
        """(seg_edge_off, num_segments) of the LOCAL plan for gradient rows of
        dim_origin floats: source rows cut into equal bands of about
        LOCAL_BAND_BYTES of G; seg_edge_off[s*W + w] = first edge of wave w in
        band s (a wave's edges are sorted by source row), row NS = wave ends."""
        ns = max(1, -(-self.num_rows * dim_origin * 4 // max(LOCAL_BAND_BYTES, 1)))
        ns = min(ns, self.num_rows)
        hit = plan["bands"].get(ns)
        if hit is not None:
            return hit
        W = plan["num_waves"]
        seg = torch.empty((ns + 1) * W, dtype=torch.int32, device=self.device)
        L = _lib.load()
        _lib.check(L.maxk_local_bands_build(plan["woff"].data_ptr(), plan["edge_rc"].data_ptr(), W,
                                            self.num_rows, ns, seg.data_ptr(), _stream(seg)),
                   "maxk_local_bands_build")
        hit = (seg, ns)
        plan["bands"][ns] = hit
        return hit

    def local_values(self, plan, values: torch.Tensor) -> torch.Tensor:
        """Edge values other than the graph's own, permuted into the LOCAL plan's
        edge order; cached per values tensor (and version)."""
        cache = plan.setdefault("val_cache", {})
        key = _tensor_key(values)
        hit = cache.get(key)
        if hit is None:
            if len(cache) >= 32:
                cache.clear()
            ev = values[: self.num_edges][plan["perm"].long()].contiguous()
            # the entry holds `values` too: while cached its address cannot be
            # reused by another tensor that would then match the key
            hit = cache[key] = (ev, values)
        return hit[0]

    def tile_plan(self, dim_k: int = 32):
        """Plan of the TILE backward (k = 32 or 64, h = 256; spgemm_new_amd/tile.py),
        or None when the shape does not suit it (then the other algorithms serve
        it).  Built once per k on the device (maxk_tile_plan_build).  Its records
        carry edge values; ``tile_values`` makes them hold a given values tensor."""
        if dim_k not in self._tile:
            from . import tile
            plan = None
            if self.num_edges > 0 and self.device.type == "cuda":
                cus = torch.cuda.get_device_properties(self.device).multi_processor_count
                shape = None
                if self.tile_splits is not None:
                    # S equal source ranges per group: G * S workgroups
                    G, GS, _ = tile.choose_shape(self.num_rows, self.num_cols, cus, dim_k)
                    shape = (G, GS, G * max(1, min(int(self.tile_splits), self.num_rows)))
                plan = tile.build(self.indptr, self.indices[: self.num_edges],
                                  self.values[: self.num_edges], self.num_rows, self.num_cols,
                                  cus=cus, k=dim_k, shape=shape)
            if plan is not None:
                # the values the records hold: key + the tensor (kept alive so its
                # address cannot be reused by another tensor with the same key)
                plan["values_key"] = _tensor_key(self.values)
                plan["values_ref"] = self.values
                plan["part"] = torch.empty(max(1, plan["part_planes"] * self.num_cols * dim_k),
                                           dtype=torch.float32, device=self.device)
            self._tile[dim_k] = plan
        return self._tile[dim_k]

    def append_plan(self, dim_k: int) -> dict:
        """Plan of the APPEND backward (maxk_append_plan_build): the destination
        bins and the first entry of every (bin, XCD group) region for this graph's
        backward panel schedule.  Built once per k on the device."""
        if dim_k not in self._append:
            L = _lib.load()
            nb, bs = ctypes.c_int(0), ctypes.c_int(0)
            _lib.check(L.maxk_append_bins(self.num_cols, dim_k, ctypes.byref(nb), ctypes.byref(bs)),
                       "maxk_append_bins")
            base = torch.empty(nb.value * 8 + 1, dtype=torch.int32, device=self.device)
            _lib.check(L.maxk_append_plan_build(
                self.bwd_sched.data_ptr(), self.bwd_num_panels, self.indptr.data_ptr(),
                self.indices.data_ptr(), self.num_rows, self.num_cols, dim_k, base.data_ptr(),
                nb.value, bs.value, _stream(base)), "maxk_append_plan_build")
            self._append[dim_k] = {"region_base": base, "num_bins": nb.value, "bin_size": bs.value}
        return self._append[dim_k]

    def tile_values(self, plan, values: torch.Tensor) -> None:
        """Make the TILE records hold ``values`` (fp32[E]: the graph's own, changed
        in place or not, or per-call ones): one scatter of E values into the
        records (maxk_tile_plan_set_values) when they hold anything else.  While
        a hipGraph is captured the scatter is always recorded, so replays pick
        up values changed between them; once a capture has recorded it, every
        eager call rewrites the records as well (a replay may have rewritten
        them with other values than the ones the Python state names)."""
        key = _tensor_key(values)
        capturing = torch.cuda.is_current_stream_capturing()
        if capturing:
            # a replay rewrites the records behind the Python state's back: from
            # now on every eager call rewrites them too
            plan["captured_values"] = True
        if plan["values_key"] != key or plan["values_ref"] is not values or capturing or \
                plan.get("captured_values"):
            from . import tile
            tile.set_values(plan, values[: self.num_edges])
            plan["values_key"], plan["values_ref"] = key, values

    def local_fits(self, dim_k: int) -> bool:
        """True when the LOCAL plan's waves are all co-resident (one sweep of G)."""
        plan = self.local_plan(dim_k)
        if plan is None:
            return False
        cus = torch.cuda.get_device_properties(self.device).multi_processor_count
        L = _lib.load()
        per_block = L.maxk_backward_local_lds_bytes(plan["dmax"], dim_k)
        blocks_per_cu = max(1, (160 * 1024) // max(per_block, 1))
        return plan["num_waves"] <= cus * blocks_per_cu * 4

    def edge_selectors(self, sel: torch.Tensor):
        """The edge selectors of ``sel`` (uint8[E * k], CSR edge order) when a
        forward wrote them for this selector tensor (MAXK_BWD_STAGED_EDGE), else None."""
        key = _tensor_key(sel)
        for k_, s_, buf, _ in reversed(self._esel):
            if k_ == key and s_ is sel:
                return buf
        return None

    def _esel_slot(self, sel: torch.Tensor) -> torch.Tensor:
        """A buffer for the edge selectors of ``sel`` (recycles the oldest entry);
        the entry holds ``sel`` so its address is not reused while cached.  A
        buffer written under hipGraph capture is pinned: a replay rewrites it, so
        no other selector tensor may ever be given it."""
        n = max(1, self.num_edges * sel.shape[1])
        key = _tensor_key(sel)
        pinned = torch.cuda.is_current_stream_capturing()
        for i, (k_, s_, buf, pin) in enumerate(self._esel):
            if s_ is sel:
                del self._esel[i]
                pinned = pinned or pin
                break
        else:
            buf = None
            free = [i for i, e in enumerate(self._esel) if not e[3]]
            if not pinned and len(free) >= max(1, ESEL_CACHE):
                _, _, buf, _ = self._esel.pop(free[0])
            if buf is None or buf.numel() < n:
                buf = torch.empty(n, dtype=torch.uint8, device=self.device)
        self._esel.append((key, sel, buf, pinned))
        return buf

    def make_edge_selectors(self, sel: torch.Tensor) -> torch.Tensor:
        """Edge selectors for ``sel`` without a caller's forward: one forward
        pass writing them (HIP, maxk_spgemm_forward_esel) into scratch output."""
        buf = self.edge_selectors(sel)
        if buf is None:
            k = sel.shape[1]
            dummy = self._workspace(("esel_data", k), self.num_cols * k * 4)
            dummy = dummy[: self.num_cols * k * 4].view(torch.float32).view(self.num_cols, k)
            y = torch.empty((self.num_rows, 256), dtype=torch.float32, device=self.device)
            spgemm_forward(self, dummy, sel, 256, out=y, edge_sel=True)
            del y
            buf = self.edge_selectors(sel)
        return buf

    def _fixed_choice(self, k: int, h: int, own: bool) -> int:
        """MAXK_AUTO=fixed: a rule of the shape that reproduces what measurement
        picks on the BASELINE shapes, so the algorithm -- and every
        bit of the result -- repeats on every box: TILE on long-row graphs (mean
        degree >= 128: Reddit, proteins) and at k = 64; else LOCAL when the gradient
        fits a few source bands (small graphs); else TILE when the destinations fit
        one group per CU (small rank blocks); else, on large short-row graphs
        (products), EDGE_GATHER at k = 8, STAGED_EDGE at k = 32 when the selector
        table reaches ESEL_MIN_SEL_BYTES (both with the forward writing the edge
        selectors) and STAGED otherwise."""
        long_rows = self.num_edges >= FWD_BLOCKED_MIN_DEGREE * max(self.num_rows, 1)
        if (own and TILE_AUTO and tile_shape_ok(k, h) and (long_rows or k == 64)
                and self.tile_plan(k) is not None):
            return _lib.MAXK_BWD_TILE
        if self.num_rows * h * 4 <= 8 * LOCAL_BAND_BYTES and self.local_plan(k) is not None:
            return _lib.MAXK_BWD_LOCAL
        if own and TILE_AUTO and tile_shape_ok(k, h) and self.device.type == "cuda":
            # destinations that fit one TILE group per CU (a rank's own-column block at
            # products N=8: 306 K columns, TILE 0.455 vs STAGED 0.566 ms fwd+bwd measured,
            # profiles/r5_rank_products_n8_candidates.txt); BASELINE's N=1 shapes are
            # unchanged (Reddit / proteins are long-row, products has 2.45 M columns).
            # The bound is MI355X's 256 CUs as a constant, not the device's count, so
            # the fixed choice (and its summation order) is the same on every box
            # 
            from . import tile
            if self.num_cols <= tile.max_group(k) * FIXED_RULE_CUS and self.tile_plan(k) is not None:
                return _lib.MAXK_BWD_TILE
        if ESEL_AUTO and h <= 256 and k == 8:
            return _lib.MAXK_BWD_EDGE_GATHER
        if ESEL_AUTO and h <= 256 and k == 32 and self.num_cols * k >= ESEL_MIN_SEL_BYTES:
            return _lib.MAXK_BWD_STAGED_EDGE
        return _lib.MAXK_BWD_STAGED

    def autotune_backward(self, grad, sel, out, values=None) -> int:
        """MAXK_BWD_AUTO: the fastest algorithm for this graph and k, measured once
        (each candidate run once, then timed AUTOTUNE_REPS times with HIP events on
        the current stream, the minimum kept) and cached.  Candidates: STAGED,
        ATOMIC, LOCAL when its plan exists, TILE for k in {32, 64}, h = 256 and the
        graph's own values.  During stream capture nothing is timed: the choice
        already measured for the shape, else TILE if its plan exists, else STAGED.
        With several timed candidates within noise the minimum decides, so the
        choice (and with it the fp32 summation order) is fixed per graph and
        shape once made; MAXK_BWD_* pins one explicitly."""
        k = sel.shape[1]
        own = values is None or values is self.values
        # kept per (k, h, own values): with other values TILE pays a scatter of the
        # values into its records whenever they change, so the ranking can differ
        key = (k, grad.shape[1], own)
        if key in self._bwd_choice:
            return self._bwd_choice[key]
        tile_ok = TILE_AUTO and tile_shape_ok(k, grad.shape[1])
        if self.num_edges == 0:
            return _lib.MAXK_BWD_STAGED
        if AUTO_MODE == "fixed":
            choice = self._fixed_choice(k, grad.shape[1], own)
            self._bwd_choice[key] = choice
            if choice in _ESEL_ALGOS:
                # the forwards of this shape write the edge selectors from now on; this
                # call (no such forward yet) takes STAGED
                self._esel_on.add((k, grad.shape[1]))
                self._bwd_alt[key] = _lib.MAXK_BWD_STAGED
            return choice
        if torch.cuda.is_current_stream_capturing():
            # nothing can be timed (or planned) while a graph is captured: the
            # choice measured for the same shape with the graph's own values,
            # else TILE when its plan was built before the capture, else STAGED
            hit = self._bwd_choice.get((k, grad.shape[1], True))
            if hit is not None and (own or hit != _lib.MAXK_BWD_TILE):
                return hit
            if tile_ok and own and self._tile.get(k) is not None:
                return _lib.MAXK_BWD_TILE
            return _lib.MAXK_BWD_STAGED
        cands = [_lib.MAXK_BWD_STAGED] + ([] if DETERMINISTIC else [_lib.MAXK_BWD_ATOMIC])
        if self.local_plan(k) is not None:
            cands.append(_lib.MAXK_BWD_LOCAL)
        if tile_ok and self.tile_plan(k) is not None:
            cands.append(_lib.MAXK_BWD_TILE)
        pair = None
        if ESEL_AUTO and grad.shape[1] <= 256:
            # STAGED_EDGE moves work into the forward (it writes the edge
            # selectors) and the two share the caches, so every candidate is
            # timed as forward + backward (dummy CBSR values, this sel), the
            # forward writing the edge selectors only for STAGED_EDGE
            self.make_edge_selectors(sel)
            cands.append(_lib.MAXK_BWD_STAGED_EDGE)
            if _edge_gather_ok(k):
                cands.append(_lib.MAXK_BWD_EDGE_GATHER)
            dummy = self._workspace(("esel_data", k), self.num_cols * k * 4)
            dummy = dummy[: self.num_cols * k * 4].view(torch.float32).view(self.num_cols, k)
            yd = torch.empty((self.num_rows, grad.shape[1]), dtype=torch.float32,
                             device=self.device)

            def pair(a):
                spgemm_forward(self, dummy, sel, grad.shape[1], out=yd, edge_sel=a in _ESEL_ALGOS)
                sspmm_backward(self, grad, sel, out, values, a)
        best, best_ms, alt, alt_ms = None, float("inf"), None, float("inf")
        timed = {}
        for a in cands:
            if pair is not None:
                ms = _min_ms(lambda: pair(a))
            else:
                ms = _min_ms(lambda: sspmm_backward(self, grad, sel, out, values, a))
            timed[_ALGO_NAMES[a]] = round(ms, 4)
            if a not in _ESEL_ALGOS and ms < alt_ms:
                alt, alt_ms = a, ms
            if ms < best_ms:
                best, best_ms = a, ms
        self._bwd_choice[key] = best
        self._bwd_alt[key] = alt
        if best in _ESEL_ALGOS:
            self._esel_on.add((k, grad.shape[1]))
        self.bwd_timings = getattr(self, "bwd_timings", {})
        self.bwd_timings[key] = best_ms
        # every candidate's time (forward + backward when the edge-selector ones ran)
        self.bwd_candidates = getattr(self, "bwd_candidates", {})
        self.bwd_candidates[key] = timed
        return best

    def nbytes_fwd(self, dim_k: int, dim_origin: int) -> int:
        """Algorithmic bytes of one forward call: 8E + 5kE + 4hV."""
        return 8 * self.num_edges + 5 * dim_k * self.num_edges + 4 * dim_origin * self.num_rows

    nbytes_bwd = nbytes_fwd

    # ---------------------------------------------------------------- compute
    def forward(self, cbsr_data: torch.Tensor, cbsr_sel: torch.Tensor, dim_origin: int = 256,
                out: torch.Tensor | None = None, values: torch.Tensor | None = None,
                accumulate: bool = False, edge_sel: bool | str = False) -> torch.Tensor:
        """Y = A . scatter(CBSR)  (spmm_maxk.cu:17-106).  Returns fp32[V, dim_origin];
        accumulate=True adds into out instead.  edge_sel: also write the edge
        selectors for a STAGED_EDGE / EDGE_GATHER backward of this same selector
        tensor -- "auto": when AUTO chose such a backward for (k, h); only a
        caller that runs that backward next should ask (the autograd Function
        does when the input needs a gradient), else the E*k bytes are wasted."""
        return spgemm_forward(self, cbsr_data, cbsr_sel, dim_origin, out, values, accumulate,
                              edge_sel)

    def forward_records(self, records: torch.Tensor, dim_k: int, dim_origin: int = 256,
                        out: torch.Tensor | None = None, values: torch.Tensor | None = None,
                        accumulate: bool = False) -> torch.Tensor:
        """forward() with the CBSR read in place from halo records (uint8[num_cols, 5k],
        see cbsr_gather_records); accumulate=True computes out += A . X^."""
        return spgemm_forward_records(self, records, dim_k, dim_origin, out, values, accumulate)

    def forward_multi(self, cbsr_data: torch.Tensor, cbsr_sel: torch.Tensor,
                      values: torch.Tensor, dim_origin: int = 256,
                      out: torch.Tensor | None = None) -> torch.Tensor:
        """Fused multi-relation forward (BASELINE config 5, ogbn-proteins):
        Y[q] = A_q . scatter(CBSR) with A_q's values = values[:, q]
        (fp32[E, R], R <= 16).  Returns fp32[R, V, dim_origin]; equals R
        forward() calls with values[:, q].contiguous() (the relation-vector LDS
        kernel, maxk_spgemm_forward_multi)."""
        return spgemm_forward_multi(self, cbsr_data, cbsr_sel, values, dim_origin, out)

    def backward_multi(self, grad: torch.Tensor, cbsr_sel: torch.Tensor, values: torch.Tensor,
                       out: torch.Tensor | None = None, algo: int = _lib.MAXK_BWD_AUTO):
        """Backward of forward_multi: dXs = sum_q (A_q^T G_q) sampled at sel,
        with grad fp32[R, V, h] and values fp32[E, R].  Returns fp32[V, k].
        Algorithms: MAXK_BWD_MULTI_STAGED / MULTI_EDGE_GATHER -- one staged pass
        that sums the R relations per edge in phase 1 (maxk_sspmm_backward_multi;
        R in {4, 8, 16}, k in {8, 16, 32, 64}); LOCAL -- for R a multiple of 8
        and k = 32, one LOCAL pass per 8 relations over the gradient interleaved
        by relation; any single-relation algorithm -- composed from R
        single-relation calls (per-relation value columns cached), summed on the
        device.  AUTO times the fused candidates once per (k, h, R) (MAXK_AUTO=
        fixed: MULTI_STAGED when it applies, then LOCAL rel8, else composed)."""
        check_tensor(grad, "grad_output", torch.float32, dim=3)
        check_tensor(values, "values", torch.float32, dim=2)
        R = values.shape[1]
        if grad.shape[0] != R or values.shape[0] != self.num_edges:
            raise RuntimeError("grad must be [R, V, h] and values [E, R]")
        check_tensor(cbsr_sel, "sparse_selector", torch.uint8, dim=2)
        if grad.shape[1] != self.num_rows or cbsr_sel.shape[0] != self.num_cols:
            raise RuntimeError("grad must be [R, num_rows, h] and sparse_selector [num_cols, k]")
        _on_device(self, grad_output=grad, sparse_selector=cbsr_sel, values=values)
        k = cbsr_sel.shape[1]
        if out is None:
            out = torch.empty((self.num_cols, k), dtype=torch.float32, device=self.device)
        if self.num_cols == 0:
            return out
        if self.num_rows == 0:
            return out.zero_()   # an empty block: dXs = 0
        staged_ok = (R in (4, 8, 16) and k in (8, 16, 32, 64) and grad.shape[2] % 4 == 0
                     and self.num_edges > 0 and values.data_ptr() % 16 == 0
                     and grad.data_ptr() % 16 == 0)
        if algo == _lib.MAXK_BWD_AUTO:
            # the same lazily built plans the candidates need; rel8 last (its
            # LOCAL plan costs the most to build).  Measure mode also times the
            # composed form (R single-relation calls, each its own AUTO) against
            # them (a shape where no fused form pays must be able to
            # fall back); fixed mode takes MULTI_STAGED where it applies -- measured
            # best on proteins R = 8, k = 32 and the only fused form
            # that serves R in {4, 16} at other k
            fused = []
            if staged_ok:
                fused += [_lib.MAXK_BWD_MULTI_STAGED, _lib.MAXK_BWD_MULTI_EDGE_GATHER]
            key = ("multi", k, grad.shape[2], R)
            # the LOCAL plan (the costliest to build) only when rel8 will be timed or is
            # the only fused form
            want_rel8 = key not in self._bwd_choice and (
                not staged_ok or (AUTO_MODE != "fixed" and
                                  not torch.cuda.is_current_stream_capturing()))
            if want_rel8 and R % 8 == 0 and k == 32 and self.num_edges > 0 and \
                    self.local_plan(k) is not None:
                fused.append(_lib.MAXK_BWD_LOCAL)
            if key in self._bwd_choice:
                algo = self._bwd_choice[key]
                if algo in (_lib.MAXK_BWD_MULTI_STAGED, _lib.MAXK_BWD_MULTI_EDGE_GATHER) and \
                        not staged_ok:
                    # e.g. misaligned values: rel8, else composed (each call its own AUTO)
                    algo = _lib.MAXK_BWD_LOCAL if (R % 8 == 0 and k == 32 and
                                                   self.local_plan(k) is not None) \
                        else _lib.MAXK_BWD_AUTO
            elif not fused:
                algo = _lib.MAXK_BWD_AUTO   # composed, each call its own AUTO
            elif AUTO_MODE == "fixed" or len(fused) == 1 or \
                    torch.cuda.is_current_stream_capturing():
                algo = self._bwd_choice[key] = fused[0]
            else:
                # measured once per (k, h, R): each fused candidate and the composed
                # form run once, then timed AUTOTUNE_REPS times, the minimum kept
                best = None
                for a in fused + [_lib.MAXK_BWD_AUTO]:
                    def run(a=a):
                        if a == _lib.MAXK_BWD_AUTO:   # composed (not a recursive AUTO call)
                            self._backward_composed(grad, cbsr_sel, values, out, a)
                        else:
                            self.backward_multi(grad, cbsr_sel, values, out, a)
                    run()
                    t = float("inf")
                    for _ in range(AUTOTUNE_REPS):
                        e0 = torch.cuda.Event(enable_timing=True)
                        e1 = torch.cuda.Event(enable_timing=True)
                        e0.record()
                        run()
                        e1.record()
                        e1.synchronize()
                        t = min(t, e0.elapsed_time(e1))
                    self._multi_timings[(key, a)] = t
                    if best is None or t < best[0]:
                        best = (t, a)
                algo = self._bwd_choice[key] = best[1]
        if algo == _lib.MAXK_BWD_MULTI_APPEND:
            if not staged_ok:
                raise RuntimeError("multi-relation APPEND backward needs R in {4, 8, 16}, k in "
                                   "{8, 16, 32, 64}, h % 4 == 0 and 16-B aligned grad/values")
            return self._backward_multi_append(grad, cbsr_sel, values, out)
        if algo in (_lib.MAXK_BWD_MULTI_STAGED, _lib.MAXK_BWD_MULTI_EDGE_GATHER):
            if not staged_ok:
                raise RuntimeError("multi-relation STAGED backward needs R in {4, 8, 16}, k in "
                                   "{8, 16, 32, 64}, h % 4 == 0 and 16-B aligned grad/values")
            return self._backward_multi_staged(grad, cbsr_sel, values, out,
                                               algo == _lib.MAXK_BWD_MULTI_EDGE_GATHER)
        if algo == _lib.MAXK_BWD_LOCAL and R % 8 == 0 and k == 32 and self.num_edges > 0 \
                and self.local_plan(k) is not None:
            return self._backward_rel8(grad, cbsr_sel, values, out)
        return self._backward_composed(grad, cbsr_sel, values, out, algo)

    def _backward_multi_staged(self, grad, sel, values, out, edge_order: bool):
        """One pass for all R relations (maxk_sspmm_backward_multi): phase 1 writes
        per edge sum_q val[e,q] * G_q[row, sel[c, :]] (LDS form), phase 2 the CSC
        segmented sum (edge_order: rows in edge order, gathered through the CSC
        permutation)."""
        L = _lib.load()
        k, h, R = sel.shape[1], grad.shape[2], values.shape[1]
        cabi = _lib.MAXK_BWD_EDGE_GATHER if edge_order else _lib.MAXK_BWD_STAGED
        csc_pos, csc_indptr, csc_sched, CP = self.csc()
        if edge_order:
            csc_pos = self.csc_perm()
        ws = self._workspace(("bwd", k), L.maxk_backward_workspace_bytes(cabi, self.num_edges, k, CP))
        _lib.check(L.maxk_sspmm_backward_multi(
            cabi, self.bwd_sched.data_ptr(), self.bwd_num_panels, self.indptr.data_ptr(),
            self.indices.data_ptr(), values.data_ptr(), R, grad.data_ptr(), sel.data_ptr(),
            self.num_rows, self.num_cols, self.num_edges, h, k, out.data_ptr(), csc_pos.data_ptr(),
            csc_sched.data_ptr(), CP, csc_indptr.data_ptr(), ws.data_ptr(), ws.numel(),
            _stream(out)), "maxk_sspmm_backward_multi")
        self.last_bwd_algo = "multi_edge_gather" if edge_order else "multi_staged"
        return out

    def _backward_multi_append(self, grad, sel, values, out):
        """The relations summed per edge in phase 1 as MULTI_STAGED, the per-edge
        vectors appended to destination bins and reduced per bin in LDS
        (maxk_sspmm_backward_append with num_rel = R; non-deterministic order)."""
        L = _lib.load()
        k, h, R = sel.shape[1], grad.shape[2], values.shape[1]
        plan = self.append_plan(k)
        ws = self._workspace(("bwd_append", k), L.maxk_backward_append_workspace_bytes(
            self.num_edges, k, plan["num_bins"]))
        _lib.check(L.maxk_sspmm_backward_append(
            self.bwd_sched.data_ptr(), self.bwd_num_panels, self.indptr.data_ptr(),
            self.indices.data_ptr(), values.data_ptr(), R, grad.data_ptr(), sel.data_ptr(), 0,
            self.num_rows, self.num_cols, self.num_edges, h, k, plan["region_base"].data_ptr(),
            plan["num_bins"], plan["bin_size"], out.data_ptr(), ws.data_ptr(), ws.numel(),
            _stream(out)), "maxk_sspmm_backward_append")
        self.last_bwd_algo = "multi_append"
        return out

    def _backward_composed(self, grad, cbsr_sel, values, out, algo):
        R = values.shape[1]
        cols = self._multi_cols(values)
        tmp = torch.empty_like(out) if R > 1 else None
        for q in range(R):
            sspmm_backward(self, grad[q], cbsr_sel, out if q == 0 else tmp, cols[q], algo)
            if q > 0:
                out.add_(tmp)
        return out

    def _backward_rel8(self, grad, sel, values, out):
        """R = 8g, k = 32: per group of 8 relations, the gradient interleaved by
        relation ([V, h, 8]) and one dwordx4 gather per lane covering an edge's 8
        relations (maxk_sspmm_backward_local_rel8); groups summed on the device."""
        h, R = grad.shape[2], values.shape[1]
        L = _lib.load()
        gt = self._workspace(("grad_rel8", h), self.num_rows * h * 8 * 4)
        gt = gt[: self.num_rows * h * 8 * 4].view(torch.float32)
        plan = self.local_plan(32)
        seg, ns = self.local_bands(plan, h * 8)       # 8 gradient rows per source row
        ev = self.local_values(plan, values)          # [E, R] in plan order
        tmp = torch.empty_like(out) if R > 8 else None
        for g0 in range(0, R, 8):
            evg = ev if R == 8 else self._rel_group_values(plan, values, ev, g0)
            dst = out if g0 == 0 else tmp
            _lib.check(L.maxk_grad_interleave(grad[g0:g0 + 8].data_ptr(), 8, self.num_rows, h,
                                              gt.data_ptr(), _stream(out)), "maxk_grad_interleave")
            _lib.check(L.maxk_sspmm_backward_local_rel8(
                seg.data_ptr(), ns, plan["dstart"].data_ptr(), plan["num_waves"], plan["dmax"],
                plan["edge_rc"].data_ptr(), evg.data_ptr(), gt.data_ptr(), sel.data_ptr(),
                self.num_rows, h, 32, dst.data_ptr(), _stream(out)),
                "maxk_sspmm_backward_local_rel8")
            if g0 > 0:
                out.add_(tmp)
        self.last_bwd_algo = "local_rel8"
        return out

    def _rel_group_values(self, plan, values, ev, g0):
        """Columns g0..g0+7 of the plan-ordered values [E, R], contiguous (cached)."""
        cache = plan.setdefault("rel_group_cache", {})
        key = (_tensor_key(values), g0)
        hit = cache.get(key)
        if hit is None:
            if len(cache) >= 16:
                cache.clear()
            hit = cache[key] = (ev[:, g0:g0 + 8].contiguous(), values)
        return hit[0]

    def _multi_cols(self, values: torch.Tensor):
        key = _tensor_key(values)
        hit = getattr(self, "_cols_cache", None)
        if hit is None or hit[0] != key:
            cols = [values[:, q].contiguous() for q in range(values.shape[1])]
            self._cols_cache = (key, cols, values)  # holds values: its address stays unique
        return self._cols_cache[1]

    def spmm_dense(self, x: torch.Tensor, out: torch.Tensor | None = None,
                   values: torch.Tensor | None = None) -> torch.Tensor:
        """Dense SpMM baseline Y = A . x (x fp32[num_cols, h], h % 4 == 0, h <= 256):
        the comparison the reference's speedup table makes (GNNAdvisor SAG,
        kernels/spmm_gnna.cu:60-140; cuSPARSE, cuda_kernel_bindings.cpp:253-284)."""
        return spmm_dense(self, x, out, values)

    def spmm_sag(self, x: torch.Tensor, weighted: bool = True,
                 out: torch.Tensor | None = None) -> torch.Tensor:
        """GNNAdvisor-style SAG baseline (kernels/spmm_gnna.cu:60-140; README.md:136's
        second comparison): neighbours cut into parts of E / V (build_part,
        spmm_gnna.cu:20-56 -- the warp4 schedule with that chunk size), one wave
        per part, float atomics into the output.  weighted=False sums the
        neighbour rows as the reference does; True scales them by the edge values
        (= A . x, comparable with forward()).  Not on the MaxK path."""
        check_tensor(x, "input_features", torch.float32, dim=2)
        _on_device(self, input_features=x)
        if x.shape[0] != self.num_cols:
            raise RuntimeError(f"input_features has {x.shape[0]} rows, graph has {self.num_cols} columns")
        dim = x.shape[1]
        if dim % 4 or not 4 <= dim <= 256:
            raise RuntimeError("SAG needs 4 <= dim <= 256 and dim % 4 == 0")
        if getattr(self, "_sag_parts", None) is None:
            part = max(1, self.num_edges // max(self.num_rows, 1))
            self._sag_parts = warp4_build(self.indptr, part)
        parts = self._sag_parts
        if out is None:
            out = torch.zeros((self.num_rows, dim), dtype=torch.float32, device=self.device)
        else:
            check_tensor(out, "output", torch.float32, dim=2)
            out.zero_()
        L = _lib.load()
        _lib.check(L.maxk_spmm_gnna_sag(parts.data_ptr(), parts.numel() // 4, self.indices.data_ptr(),
                                        self.values.data_ptr() if weighted else None, x.data_ptr(),
                                        dim, out.data_ptr(), _stream(out)), "maxk_spmm_gnna_sag")
        return out

    def backward(self, grad: torch.Tensor, cbsr_sel: torch.Tensor, out: torch.Tensor | None = None,
                 values: torch.Tensor | None = None, algo: int = _lib.MAXK_BWD_AUTO) -> torch.Tensor:
        """dXs = (A^T G) sampled at sel  (spmm_maxk_backward.cu:15-115).  Returns fp32[V, k]."""
        return sspmm_backward(self, grad, cbsr_sel, out, values, algo)


def _on_device(g: MaxKGraph, **tensors):
    for name, t in tensors.items():
        if t is not None and t.device != g.device:
            raise RuntimeError(f"{name} must be on the graph's device ({g.device}), got {t.device}")


def _check_values(g: MaxKGraph, values):
    """Edge values other than the graph's own: fp32[E] on the graph's device."""
    if values is None:
        return g.values
    check_tensor(values, "values", torch.float32, dim=1)
    if values.numel() != g.num_edges:
        raise RuntimeError(f"values must have num_edges = {g.num_edges} elements, got {values.numel()}")
    _on_device(g, values=values)
    return values if g.num_edges > 0 else g.values


def _check_cbsr(g: MaxKGraph, data, sel):
    check_tensor(data, "input_data", torch.float32, dim=2)
    check_tensor(sel, "sparse_selector", torch.uint8, dim=2)
    if data.shape != sel.shape:
        raise RuntimeError("input_data and sparse_selector must have the same shape")
    if data.shape[0] != g.num_cols:
        raise RuntimeError(f"CBSR has {data.shape[0]} rows, graph has {g.num_cols} columns")
    if data.device != g.device or sel.device != g.device:
        raise RuntimeError("CBSR tensors must be on the graph's device")


def spgemm_forward(g: MaxKGraph, data, sel, dim_origin: int = 256, out=None, values=None,
                   accumulate: bool = False, edge_sel: bool | str = False):
    """edge_sel: also write the edge selectors of sel (kept by the graph for the
    STAGED_EDGE / EDGE_GATHER backward); "auto" = when AUTO chose such a backward
    for (k, h)."""
    _check_cbsr(g, data, sel)
    k = data.shape[1]
    values = _check_values(g, values)
    if out is None:
        if accumulate:
            raise RuntimeError("accumulate needs an output")
        out = torch.empty((g.num_rows, dim_origin), dtype=torch.float32, device=g.device)
    else:
        check_tensor(out, "output", torch.float32, dim=2)
        if tuple(out.shape) != (g.num_rows, dim_origin):
            raise RuntimeError("output has the wrong shape")
        _on_device(g, output=out)
    if g.num_rows == 0:
        return out   # an empty block (a rank of the row partition that owns no row)
    if g.num_cols == 0:
        return out if accumulate else out.zero_()   # no source nodes: Y = 0
    L = _lib.load()
    nbytes = L.maxk_forward_workspace_bytes(g.num_panels, dim_origin)
    ws = g._workspace(("fwd", dim_origin), nbytes)
    if edge_sel == "auto":
        edge_sel = (k, dim_origin) in g._esel_on
    edge_sel = edge_sel and not accumulate and g.num_edges > 0
    rs = L.maxk_cbsr_packed_row_bytes(k) if FWD_PACKED and not accumulate else 0
    rec = None
    if rs:  # k in {4, 8, 16}: one cache line per gathered neighbour (packed records)
        rec = g._workspace(("packed", k), g.num_cols * rs)
        _lib.check(L.maxk_cbsr_pack(data.data_ptr(), sel.data_ptr(), g.num_cols, k, rec.data_ptr(),
                                    _stream(out)), "maxk_cbsr_pack")
    if edge_sel:
        es = g._esel_slot(sel)
        _lib.check(L.maxk_spgemm_forward_esel(
            g.sched.data_ptr(), g.num_panels, g.indptr.data_ptr(), g.indices.data_ptr(),
            values.data_ptr(), data.data_ptr(), sel.data_ptr(), _lib.ptr(rec), g.num_rows,
            dim_origin, k, out.data_ptr(), es.data_ptr(), ws.data_ptr(), ws.numel(), _stream(out)),
            "maxk_spgemm_forward_esel")
        return out
    if rs:
        _lib.check(L.maxk_spgemm_forward_packed(
            g.sched.data_ptr(), g.num_panels, g.indptr.data_ptr(), g.indices.data_ptr(),
            values.data_ptr(), rec.data_ptr(), g.num_rows, dim_origin, k, out.data_ptr(),
            ws.data_ptr(), ws.numel(), _stream(out)), "maxk_spgemm_forward_packed")
        return out
    if not accumulate and k >= 32 and g.num_edges > 0:
        nb = _fwd_blocks(g, data, sel, dim_origin, out, values)
        if nb:
            return _forward_blocked(g, nb, data, sel, dim_origin, out, values)
    flags = _lib.MAXK_FWD_ACCUMULATE if accumulate else 0
    _lib.check(L.maxk_spgemm_forward_ex(g.sched.data_ptr(), g.num_panels, g.indptr.data_ptr(),
                                        g.indices.data_ptr(), values.data_ptr(), data.data_ptr(),
                                        sel.data_ptr(), g.num_rows, dim_origin, k, flags,
                                        out.data_ptr(), ws.data_ptr(), ws.numel(), _stream(out)),
               "maxk_spgemm_forward")
    return out


def _blocked_split(g: MaxKGraph, plan: dict) -> dict:
    """Schedules of the column-blocked forward's two launches, built once: the
    first nb-1 blocks (rows [0, (nb-1)V) of the restacked CSR, into partial
    outputs) and the last block (rows [(nb-1)V, nb V), whose row flush adds the
    partials: maxk_spgemm_forward_sum_parts)."""
    sp = plan.get("split")
    if sp is None:
        nb, V = plan["num_blocks"], g.num_rows
        ip = plan["indptr"]
        h = (nb - 1) * V
        e_head = int(ip[h].item())
        sp = {"head_rows": h, "last_indptr": ip[h:]}
        if h > 0:
            sp["head_sched"], sp["head_P"] = _build_schedule(ip[:h + 1], h, e_head, g.panel_cost,
                                                             g.row_cost)
        sp["last_sched"], sp["last_P"] = _build_schedule(sp["last_indptr"], V, g.num_edges - e_head,
                                                         g.panel_cost, g.row_cost)
        plan["split"] = sp
    return sp


def _forward_blocked(g: MaxKGraph, nb: int, data, sel, dim_origin: int, out, values):
    """Column-blocked forward: the restacked CSR's first nb-1 blocks into
    partial outputs (cacheable gathers), then the last block, whose row flush
    adds the partials in block order (bitwise the sum maxk_rows_sum gives over
    all nb parts, one partial write + read and one pass fewer)."""
    if g.num_edges == 0 or g.num_rows == 0:
        return out.zero_()
    L = _lib.load()
    plan = g.blocked_plan(nb)
    vals = g._blocked_values(plan, values)
    sp = _blocked_split(g, plan)
    P = max(sp["last_P"], sp.get("head_P", 1))
    ws = g._workspace(("fwd_blocked", nb, dim_origin), L.maxk_forward_workspace_bytes(P, dim_origin))
    n = g.num_rows * dim_origin
    k = data.shape[1]
    parts = None
    if nb > 1:
        parts = g._workspace(("fwd_parts", nb, dim_origin), 4 * (nb - 1) * n)
        _lib.check(L.maxk_spgemm_forward_ex(sp["head_sched"].data_ptr(), sp["head_P"],
                                            plan["indptr"].data_ptr(), plan["indices"].data_ptr(),
                                            vals.data_ptr(), data.data_ptr(), sel.data_ptr(),
                                            sp["head_rows"], dim_origin, k,
                                            _lib.MAXK_FWD_CACHED_GATHER, parts.data_ptr(),
                                            ws.data_ptr(), ws.numel(), _stream(out)),
                   "maxk_spgemm_forward (column-blocked, blocks 0..nb-2)")
    _lib.check(L.maxk_spgemm_forward_sum_parts(
        sp["last_sched"].data_ptr(), sp["last_P"], sp["last_indptr"].data_ptr(),
        plan["indices"].data_ptr(), vals.data_ptr(), data.data_ptr(), sel.data_ptr(), g.num_rows,
        dim_origin, k, _lib.MAXK_FWD_CACHED_GATHER, parts.data_ptr() if parts is not None else None,
        nb - 1, out.data_ptr(), ws.data_ptr(), ws.numel(), _stream(out)),
        "maxk_spgemm_forward_sum_parts (column-blocked, last block)")
    return out


def _fwd_blocks(g: MaxKGraph, data, sel, dim_origin: int, out, values) -> int:
    """Column blocks for this (k, h): MAXK_FWD_BLOCKS, or measured once
    against the plain forward (graphs with long rows only; never under capture)."""
    if FWD_BLOCKS >= 0:
        return FWD_BLOCKS
    key = (data.shape[1], dim_origin)
    nb = g._fwd_blocks.get(key)
    if nb is not None:
        return nb
    if g.num_edges < FWD_BLOCKED_MIN_DEGREE * g.num_rows:
        g._fwd_blocks[key] = 0
        return 0
    if AUTO_MODE == "fixed":
        # the measured best on Reddit at k = 32 and 64, when its partial
        # outputs fit comfortably.  A rule of the shape and the device's TOTAL memory
        # only, so the choice (and the fp32 summation order with it) does not depend
        # on how much memory happens to be free at the first call
        total = torch.cuda.get_device_properties(g.device).total_memory
        nb = 4 if 4 * 4 * g.num_rows * dim_origin + 16 * g.num_edges <= total // 8 else 0
        g._fwd_blocks[key] = nb
        return nb
    if torch.cuda.is_current_stream_capturing():
        return 0
    L = _lib.load()
    ws = g._workspace(("fwd", dim_origin), L.maxk_forward_workspace_bytes(g.num_panels, dim_origin))

    def plain():
        _lib.check(L.maxk_spgemm_forward_ex(g.sched.data_ptr(), g.num_panels, g.indptr.data_ptr(),
                                            g.indices.data_ptr(), values.data_ptr(),
                                            data.data_ptr(), sel.data_ptr(), g.num_rows,
                                            dim_origin, data.shape[1], 0, out.data_ptr(),
                                            ws.data_ptr(), ws.numel(), _stream(out)),
                   "maxk_spgemm_forward")
    def drop(c):  # what a losing candidate built
        g._blocked.pop(c, None)
        g._ws.pop(("fwd_parts", c, dim_origin), None)
        g._ws.pop(("fwd_blocked", c, dim_origin), None)
    best, best_ms = 0, _min_ms(plain)
    free, _ = torch.cuda.mem_get_info(g.device)
    for cand in FWD_BLOCKED_CANDIDATES:
        # partial outputs + restacked indices / values / order: keep within a quarter of what is free
        if 4 * cand * g.num_rows * dim_origin + 16 * g.num_edges > free // 4:
            continue
        ms = _min_ms(lambda: _forward_blocked(g, cand, data, sel, dim_origin, out, values))
        if ms < best_ms:
            if best:
                drop(best)
            best, best_ms = cand, ms
        else:
            drop(cand)
    g._fwd_blocks[key] = best
    return best


def cbsr_gather_records(data: torch.Tensor, sel: torch.Tensor, rows: torch.Tensor | None = None,
                        out: torch.Tensor | None = None) -> torch.Tensor:
    """Halo records: uint8[n, 5k], record i = (data[rows[i]] as k fp32, sel[rows[i]]).
    The multi-GPU all-to-all-v message (maxk_cbsr_gather_records)."""
    check_tensor(data, "input_data", torch.float32, dim=2)
    check_tensor(sel, "sparse_selector", torch.uint8, dim=2)
    if data.shape != sel.shape or data.device != sel.device:
        raise RuntimeError("input_data and sparse_selector must have the same shape and device")
    k = data.shape[1]
    if k < 4 or k > 256 or k & (k - 1):
        raise RuntimeError("records need k a power of two in [4, 256]")
    if rows is not None:
        check_tensor(rows, "rows", torch.int32, dim=1)
        if rows.device != data.device:
            raise RuntimeError("rows must be on the CBSR's device")
        n = rows.numel()
    else:
        n = data.shape[0]
    if out is None:
        out = torch.empty((n, 5 * k), dtype=torch.uint8, device=data.device)
    elif not out.is_contiguous() or out.dtype != torch.uint8 or out.numel() != n * 5 * k:
        raise RuntimeError("out must be a contiguous uint8 tensor of n * 5k bytes")
    L = _lib.load()
    _lib.check(L.maxk_cbsr_gather_records(data.data_ptr(), sel.data_ptr(), _lib.ptr(rows), n, k,
                                          out.data_ptr(), _stream(data)), "maxk_cbsr_gather_records")
    return out


def spgemm_forward_records(g: MaxKGraph, records: torch.Tensor, k: int, dim_origin: int = 256,
                           out=None, values=None, accumulate: bool = False):
    """Forward reading the CBSR from halo records (uint8[num_cols, 5k]);
    accumulate=True adds into out (maxk_spgemm_forward_records)."""
    check_tensor(records, "records", torch.uint8)
    if records.numel() != g.num_cols * 5 * k:
        raise RuntimeError(f"records must hold num_cols = {g.num_cols} records of 5k bytes")
    _on_device(g, records=records)
    values = _check_values(g, values)
    if out is None:
        if accumulate:
            raise RuntimeError("accumulate needs an output")
        out = torch.empty((g.num_rows, dim_origin), dtype=torch.float32, device=g.device)
    else:
        check_tensor(out, "output", torch.float32, dim=2)
        if tuple(out.shape) != (g.num_rows, dim_origin):
            raise RuntimeError("output has the wrong shape")
        _on_device(g, output=out)
    if g.num_rows == 0:
        return out
    if g.num_cols == 0:
        return out if accumulate else out.zero_()
    L = _lib.load()
    nbytes = L.maxk_forward_workspace_bytes(g.num_panels, dim_origin)
    ws = g._workspace(("fwd", dim_origin), nbytes)
    flags = _lib.MAXK_FWD_ACCUMULATE if accumulate else 0
    _lib.check(L.maxk_spgemm_forward_records(
        g.sched.data_ptr(), g.num_panels, g.indptr.data_ptr(), g.indices.data_ptr(),
        values.data_ptr(), records.data_ptr(), g.num_rows, dim_origin, k, flags, out.data_ptr(),
        ws.data_ptr(), ws.numel(), _stream(out)), "maxk_spgemm_forward_records")
    return out


def spgemm_forward_multi(g: MaxKGraph, data, sel, values, dim_origin: int = 256, out=None):
    _check_cbsr(g, data, sel)
    k = data.shape[1]
    check_tensor(values, "values", torch.float32, dim=2)
    if values.shape[0] != g.num_edges:
        raise RuntimeError("values must be [num_edges, num_relations]")
    _on_device(g, values=values)
    R = values.shape[1]
    if not 1 <= R <= 16:
        raise RuntimeError("1 <= num_relations <= 16")
    if k & (k - 1) or not 4 <= k <= 256:
        raise RuntimeError("the fused multi-relation forward needs k a power of two in [4, 256]")
    if out is None:
        out = torch.empty((R, g.num_rows, dim_origin), dtype=torch.float32, device=g.device)
    else:
        check_tensor(out, "output", torch.float32, dim=3)
        if tuple(out.shape) != (R, g.num_rows, dim_origin):
            raise RuntimeError("output must be [R, V, dim_origin]")
        _on_device(g, output=out)
    if g.num_rows == 0:
        return out
    if g.num_cols == 0:
        return out.zero_()
    vals = values if g.num_edges > 0 else torch.zeros((1, R), device=g.device)
    L = _lib.load()
    if MULTI_BANK_ORDER and R % 4 == 0 and k % 8 == 0 and k <= 64:
        # bank-aware entry order for the relation-vector kernel's LDS stores
        # (same CBSR set, bit-identical result)
        od = g._workspace(("bank_data", k), g.num_cols * k * 4).view(torch.float32)
        os_ = g._workspace(("bank_sel", k), g.num_cols * k)
        od, os_ = od[: g.num_cols * k].view(g.num_cols, k), os_[: g.num_cols * k].view(g.num_cols, k)
        _lib.check(L.maxk_cbsr_bank_order(data.data_ptr(), sel.data_ptr(), g.num_cols, k, R,
                                          od.data_ptr(), os_.data_ptr(), _stream(out)),
                   "maxk_cbsr_bank_order")
        data, sel = od, os_
    nbytes = L.maxk_forward_multi_workspace_bytes(g.num_panels, dim_origin, R)
    ws = g._workspace(("fwd_multi", dim_origin, R), nbytes)
    _lib.check(L.maxk_spgemm_forward_multi(
        g.sched.data_ptr(), g.num_panels, g.indptr.data_ptr(), g.indices.data_ptr(),
        vals.data_ptr(), R, data.data_ptr(), sel.data_ptr(), g.num_rows, dim_origin, k,
        out.data_ptr(), ws.data_ptr(), ws.numel(), _stream(out)), "maxk_spgemm_forward_multi")
    return out


def sspmm_backward(g: MaxKGraph, grad, sel, out=None, values=None, algo: int = _lib.MAXK_BWD_AUTO):
    check_tensor(grad, "grad_output", torch.float32, dim=2)
    check_tensor(sel, "sparse_selector", torch.uint8, dim=2)
    if grad.shape[0] != g.num_rows or sel.shape[0] != g.num_cols:
        raise RuntimeError("grad_output rows must equal the graph's rows and sparse_selector "
                           "rows its columns")
    dim_origin, k = grad.shape[1], sel.shape[1]
    _on_device(g, grad_output=grad, sparse_selector=sel)
    values = _check_values(g, values)
    if out is None:
        out = torch.empty((g.num_cols, k), dtype=torch.float32, device=g.device)
    else:
        check_tensor(out, "grad_input", torch.float32, dim=2)
        if tuple(out.shape) != (g.num_cols, k):
            raise RuntimeError("grad_input has the wrong shape")
        _on_device(g, grad_input=out)
    if g.num_cols == 0:
        return out
    if g.num_rows == 0:
        return out.zero_()   # no gradient rows, no edges: dXs = 0
    if algo == _lib.MAXK_BWD_AUTO:
        algo = g.autotune_backward(grad, sel, out, values)
        if algo in _ESEL_ALGOS and g.edge_selectors(sel) is None:
            # this selector tensor went through no edge-selector forward: the best
            # of the others (never a second forward pass on the hot path)
            algo = g._bwd_alt.get((k, dim_origin, values is g.values), _lib.MAXK_BWD_STAGED)
    if g.num_edges == 0:
        algo = _lib.MAXK_BWD_ATOMIC  # nothing to stage: the call just zeroes dXs
    L = _lib.load()
    if algo == _lib.MAXK_BWD_TILE:
        plan = g.tile_plan(k) if tile_shape_ok(k, dim_origin) else None
        if plan is None:
            raise RuntimeError("TILE backward unsupported for this shape (k = 32 or 64, h = 256)")
        g.tile_values(plan, values)   # the records' values (refreshed when they changed)
        g.last_bwd_algo = "tile"
        _lib.check(L.maxk_sspmm_backward_tile(
            plan["headers"].data_ptr(), plan["header_start"].data_ptr(),
            plan["records"].data_ptr(), plan["record_start"].data_ptr(),
            plan["num_chunks"].data_ptr(), plan["num_groups"], plan["num_workgroups"],
            plan["group_size"], grad.data_ptr(), plan["zero_row"].data_ptr(), sel.data_ptr(),
            g.num_rows, g.num_cols, dim_origin, k, out.data_ptr(),
            plan["part"].data_ptr() if plan["part_planes"] > 0 else None,
            _stream(out)), "maxk_sspmm_backward_tile")
        return out
    if algo == _lib.MAXK_BWD_LOCAL:
        plan = g.local_plan(k)
        if plan is None:
            raise RuntimeError("LOCAL backward unsupported for this shape (k must divide 64)")
        g.last_bwd_algo = "local"
        seg, ns = g.local_bands(plan, dim_origin)
        ev = plan["edge_val"] if values is g.values else g.local_values(plan, values)
        _lib.check(L.maxk_sspmm_backward_local(
            seg.data_ptr(), ns, plan["dstart"].data_ptr(), plan["num_waves"], plan["dmax"],
            plan["edge_rc"].data_ptr(), ev.data_ptr(), grad.data_ptr(),
            sel.data_ptr(), g.num_rows, dim_origin, k, out.data_ptr(), _stream(out)),
            "maxk_sspmm_backward_local")
        return out
    if algo in (_lib.MAXK_BWD_APPEND, _lib.MAXK_BWD_APPEND_EDGE):
        if not _append_ok(k):
            raise RuntimeError("APPEND backward needs k a power of two in [4, 256]")
        esel = algo == _lib.MAXK_BWD_APPEND_EDGE
        sel_arg = g.make_edge_selectors(sel) if esel else sel
        plan = g.append_plan(k)
        ws = g._workspace(("bwd_append", k), L.maxk_backward_append_workspace_bytes(
            g.num_edges, k, plan["num_bins"]))
        g.last_bwd_algo = _ALGO_NAMES[algo]
        _lib.check(L.maxk_sspmm_backward_append(
            g.bwd_sched.data_ptr(), g.bwd_num_panels, g.indptr.data_ptr(), g.indices.data_ptr(),
            values.data_ptr(), 1, grad.data_ptr(), sel_arg.data_ptr(), int(esel), g.num_rows,
            g.num_cols, g.num_edges, dim_origin, k, plan["region_base"].data_ptr(),
            plan["num_bins"], plan["bin_size"], out.data_ptr(), ws.data_ptr(), ws.numel(),
            _stream(out)), "maxk_sspmm_backward_append")
        return out
    csc_pos = csc_indptr = csc_sched = None
    CP = 0
    ws = None
    sel_arg = sel
    if algo == _lib.MAXK_BWD_EDGE_GATHER and not _edge_gather_ok(k):
        raise RuntimeError("EDGE_GATHER backward needs k a power of two in [4, 256]")
    if algo in _ESEL_ALGOS:
        sel_arg = g.make_edge_selectors(sel)   # written by this sel's forward (else made here)
    if algo in (_lib.MAXK_BWD_STAGED,) + _ESEL_ALGOS:
        csc_pos, csc_indptr, csc_sched, CP = g.csc()
        if algo == _lib.MAXK_BWD_EDGE_GATHER:
            csc_pos = g.csc_perm()
        nbytes = L.maxk_backward_workspace_bytes(algo, g.num_edges, k, CP)
        ws = g._workspace(("bwd", k), nbytes)
    g.last_bwd_algo = {_lib.MAXK_BWD_ATOMIC: "atomic", _lib.MAXK_BWD_STAGED: "staged",
                       _lib.MAXK_BWD_STAGED_EDGE: "staged_edge",
                       _lib.MAXK_BWD_EDGE_GATHER: "edge_gather"}[algo]
    _lib.check(L.maxk_sspmm_backward(
        algo, g.bwd_sched.data_ptr(), g.bwd_num_panels, g.indptr.data_ptr(), g.indices.data_ptr(),
        values.data_ptr(), grad.data_ptr(), sel_arg.data_ptr(), g.num_rows, g.num_cols, g.num_edges,
        dim_origin, k,
        out.data_ptr(), _lib.ptr(csc_pos), _lib.ptr(csc_sched), CP, _lib.ptr(csc_indptr),
        _lib.ptr(ws), 0 if ws is None else ws.numel(), _stream(out)), "maxk_sspmm_backward")
    return out


def spmm_dense(g: MaxKGraph, x, out=None, values=None):
    check_tensor(x, "input_features", torch.float32, dim=2)
    _on_device(g, input_features=x)
    if x.shape[0] != g.num_cols:
        raise RuntimeError(f"input_features has {x.shape[0]} rows, graph has {g.num_cols} columns")
    dim = x.shape[1]
    if dim % 4 or not 4 <= dim <= 256:
        raise RuntimeError("dense SpMM needs 4 <= dim <= 256 and dim % 4 == 0")
    values = _check_values(g, values)
    if out is None:
        out = torch.empty((g.num_rows, dim), dtype=torch.float32, device=g.device)
    else:
        check_tensor(out, "output", torch.float32, dim=2)
        if tuple(out.shape) != (g.num_rows, dim):
            raise RuntimeError("output has the wrong shape")
        _on_device(g, output=out)
    L = _lib.load()
    ws = g._workspace(("fwd", dim), L.maxk_forward_workspace_bytes(g.num_panels, dim))
    _lib.check(L.maxk_spmm_dense_forward(g.sched.data_ptr(), g.num_panels, g.indptr.data_ptr(),
                                         g.indices.data_ptr(), values.data_ptr(), x.data_ptr(),
                                         g.num_rows, dim, out.data_ptr(), ws.data_ptr(), ws.numel(),
                                         _stream(out)), "maxk_spmm_dense_forward")
    return out


def warp4_build(indptr: torch.Tensor, warp_max_nz: int = 64) -> torch.Tensor:
    """generate_meta.py:26-48 on the device: int32[4W] (row, loc, len, 0)."""
    import ctypes
    check_tensor(indptr, "indptr", torch.int32, dim=1)
    L = _lib.load()
    V = indptr.numel() - 1
    scratch = torch.empty(V + 1, dtype=torch.int32, device=indptr.device)
    n = ctypes.c_int64(0)
    st = _stream(indptr)
    _lib.check(L.maxk_warp4_build(indptr.data_ptr(), V, warp_max_nz, scratch.data_ptr(), None, 0,
                                  ctypes.byref(n), st), "maxk_warp4_build(count)")
    W = int(n.value)
    warp4 = torch.empty(4 * max(W, 1), dtype=torch.int32, device=indptr.device)
    _lib.check(L.maxk_warp4_build(indptr.data_ptr(), V, warp_max_nz, scratch.data_ptr(),
                                  warp4.data_ptr(), W, ctypes.byref(n), st), "maxk_warp4_build")
    return warp4[: 4 * W]


# ----------------------------------------------------------------- CBSR producer
_TOPK_ORDERS = {"column": _lib.MAXK_TOPK_ORDER_COLUMN, "value": _lib.MAXK_TOPK_ORDER_VALUE,
                "lane": _lib.MAXK_TOPK_ORDER_LANE}


def topk_cbsr(x: torch.Tensor, k: int, order: str = "column", dense: bool = False,
              data: torch.Tensor | None = None, sel: torch.Tensor | None = None):
    """CBSR of the row-wise top-k of x (fp32[V, h], h <= 256): (data fp32[V,k],
    sel uint8[V,k]) with data[r, j] = x[r, sel[r, j]]; with dense=True also the
    MaxK forward (top-k kept, rest 0).  Replaces torch.topk in the reference's
    producers (direct_kernel_interface.py:79-83, spmm_bindings.cpp:163-184,
    utils/models.py:44-50).  order="column": ascending column; "value":
    descending value as torch.topk(sorted=True), ties to the lower column;
    "lane": column ranks interleaved for the forward kernel's lane layout.
    NaN ranks as the largest value."""
    check_tensor(x, "input", torch.float32, dim=2)
    V, h = x.shape
    if not 1 <= k <= h or h > 256:
        raise RuntimeError(f"top-k needs 1 <= k <= dim <= 256 (k={k}, dim={h})")
    if order not in _TOPK_ORDERS:
        raise RuntimeError(f"order must be one of {sorted(_TOPK_ORDERS)}")
    if data is None:
        data = torch.empty((V, k), dtype=torch.float32, device=x.device)
    if sel is None:
        sel = torch.empty((V, k), dtype=torch.uint8, device=x.device)
    check_tensor(data, "cbsr_data", torch.float32, dim=2)
    check_tensor(sel, "cbsr_sel", torch.uint8, dim=2)
    if tuple(data.shape) != (V, k) or tuple(sel.shape) != (V, k):
        raise RuntimeError("cbsr_data / cbsr_sel must be [V, k]")
    out = torch.empty_like(x) if dense else None
    L = _lib.load()
    _lib.check(L.maxk_topk_cbsr(x.data_ptr(), V, h, h, k, _TOPK_ORDERS[order], data.data_ptr(),
                                sel.data_ptr(), _lib.ptr(out), _stream(x)), "maxk_topk_cbsr")
    return (data, sel, out) if dense else (data, sel)


def cbsr_scatter(vals: torch.Tensor, sel: torch.Tensor, dim: int,
                 out: torch.Tensor | None = None) -> torch.Tensor:
    """Dense fp32[V, dim] with out[r, sel[r, j]] = vals[r, j], 0 elsewhere: the
    sparse->dense gradient of SpGEMMFunction.backward (utils/models.py:136-141)."""
    check_tensor(vals, "vals", torch.float32, dim=2)
    check_tensor(sel, "sparse_selector", torch.uint8, dim=2)
    if vals.shape != sel.shape:
        raise RuntimeError("vals and sparse_selector must have the same shape")
    V, k = sel.shape
    if out is None:
        out = torch.empty((V, dim), dtype=torch.float32, device=vals.device)
    check_tensor(out, "output", torch.float32, dim=2)
    if tuple(out.shape) != (V, dim):
        raise RuntimeError("output must be [V, dim]")
    L = _lib.load()
    _lib.check(L.maxk_cbsr_scatter(vals.data_ptr(), sel.data_ptr(), V, k, dim, out.data_ptr(),
                                   _stream(vals)), "maxk_cbsr_scatter")
    return out


def cbsr_mask(src: torch.Tensor, sel: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """src masked to the selected columns (the MaxK backward, utils/models.py:52-59)."""
    check_tensor(src, "grad_output", torch.float32, dim=2)
    check_tensor(sel, "sparse_selector", torch.uint8, dim=2)
    V, dim = src.shape
    if sel.shape[0] != V:
        raise RuntimeError("sparse_selector rows must match grad_output rows")
    if out is None:
        out = torch.empty_like(src)
    check_tensor(out, "output", torch.float32, dim=2)
    L = _lib.load()
    _lib.check(L.maxk_cbsr_mask(src.data_ptr(), sel.data_ptr(), V, sel.shape[1], dim,
                                out.data_ptr(), _stream(src)), "maxk_cbsr_mask")
    return out
