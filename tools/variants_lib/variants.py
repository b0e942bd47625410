"""Python side of the ABLATION build (tools/variants_lib/libmaxk_variants.so,
declared in maxk_variants.h): the kernels that were built, tested bit-exact and
measured slower on every BASELINE shape, moved out of the product library in
round 5.  They run on a product
``MaxKGraph`` (its schedule, CSC and workspaces) through the ablation library,
which is the product sources plus these kernels.  Development and regression
tests only (tests/test_variants.py); nothing in spgemm_new_amd imports this.

  forward_multi_gather  register-accumulator fused R = 8 forward (h = 256, k <= 32)
  backward_multi_form   multi-relation STAGED backward with phase 1 in register
                        ("gather") or bank-ordered ("banked") form
  bin_plan / backward_binned   BINNED (propagation blocking) backward, k in {8, 16, 32}
"""
from __future__ import annotations

import ctypes
import os

import torch

from spgemm_new_amd import _lib

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libmaxk_variants.so")
SOURCES = [os.path.join(HERE, n) for n in ("maxk_variants.hip", "maxk_variants_plan.hip")]

MAXK_BWD_BINNED = 7
MAXK_BWD_BINNED_EDGE = 8
MAXK_BIN_DESTS = 255
MAXK_BIN_WINDOW = 64
BIN_MAX_SLOTS_PER_EDGE = 1.5

_P, _I, _L, _S = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_size_t
SIGNATURES = {
    "maxk_sspmm_backward_multi_gather": (_I, [_I, _P, _L, _P, _P, _P, _I, _P, _P, _I, _I, _L, _I,
                                              _I, _P, _P, _P, _L, _P, _P, _S, _P]),
    "maxk_sspmm_backward_multi_banked": (_I, [_I, _P, _L, _P, _P, _P, _I, _P, _P, _I, _I, _L, _I,
                                              _I, _P, _P, _P, _L, _P, _P, _S, _P]),
    "maxk_cbsr_bank_order_ex": (_I, [_P, _P, _I, _I, _I, _P, _P, _P, _P]),
    "maxk_cbsr_colmask": (_I, [_P, _P, _I, _I, _P, _P, _P]),
    "maxk_spgemm_forward_multi_gather": (_I, [_P, _L, _P, _P, _P, _I, _P, _P, _I, _I, _I, _P, _P,
                                              _S, _P]),
    "maxk_bin_plan_workspace_bytes": (_S, [_L, _I]),
    "maxk_bin_plan_build": (_I, [_P, _L, _P, _L, _I, _P, _P, _P, _L, ctypes.POINTER(ctypes.c_int64),
                                 _P, _S, _P]),
    "maxk_backward_binned_workspace_bytes": (_S, [_L, _I]),
    "maxk_sspmm_backward_binned": (_I, [_P, _L, _P, _P, _P, _P, _P, _I, _I, _I, _L, _I, _I, _P, _P,
                                        _P, _P, _I, _L, _P, _S, _P]),
    "maxk_forward_multi_workspace_bytes": (_S, [_L, _I, _I]),
    "maxk_backward_workspace_bytes": (_S, [_I, _L, _I, _L]),
    "maxk_abi_version": (_I, []),
}
_lib_v = None


def load():
    """The ablation library (raises when it was not built: __graft_entry__.build)."""
    global _lib_v
    if _lib_v is None:
        if not os.path.exists(LIB_PATH):
            raise _lib.MaxKError(f"ablation library not built: {LIB_PATH}")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        if L.maxk_abi_version() != _lib.ABI_VERSION:
            raise _lib.MaxKError(f"{LIB_PATH} was built from other sources")
        _lib_v = L
    return _lib_v


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def multi_gather_ok(R: int, k: int, dim_origin: int) -> bool:
    return R == 8 and dim_origin == 256 and k in (4, 8, 16, 32)


def forward_multi_gather(g, data, sel, values, dim_origin: int = 256, out=None):
    """Register-accumulator fused forward (maxk_spgemm_forward_multi_gather): the
    destination row's 8 x 256 sums in registers; column-sorted CBSR + per-word
    column bitmasks first (maxk_cbsr_colmask).  Same result as
    MaxKGraph.forward_multi, bit for bit at k = 32."""
    L = load()
    R, k = values.shape[1], data.shape[1]
    if not multi_gather_ok(R, k, dim_origin):
        raise RuntimeError("the gather form needs R = 8, dim_origin = 256 and k in {4, 8, 16, 32}")
    if out is None:
        out = torch.empty((R, g.num_rows, dim_origin), dtype=torch.float32, device=g.device)
    sd = torch.empty((g.num_cols, k), dtype=torch.float32, device=g.device)
    mr = torch.empty((g.num_cols, 16), dtype=torch.int32, device=g.device)
    _lib.check(L.maxk_cbsr_colmask(data.data_ptr(), sel.data_ptr(), g.num_cols, k, sd.data_ptr(),
                                   mr.data_ptr(), _stream(out)), "maxk_cbsr_colmask")
    ws = torch.empty(max(1, L.maxk_forward_multi_workspace_bytes(g.num_panels, dim_origin, R)),
                     dtype=torch.uint8, device=g.device)
    vals = values if g.num_edges > 0 else torch.zeros((1, R), device=g.device)
    _lib.check(L.maxk_spgemm_forward_multi_gather(
        g.sched.data_ptr(), g.num_panels, g.indptr.data_ptr(), g.indices.data_ptr(),
        vals.data_ptr(), R, sd.data_ptr(), mr.data_ptr(), g.num_rows, dim_origin, k,
        out.data_ptr(), ws.data_ptr(), ws.numel(), _stream(out)), "maxk_spgemm_forward_multi_gather")
    return out


def backward_multi_form(g, grad, sel, values, form: str, edge_order: bool = False, out=None):
    """Multi-relation STAGED backward with phase 1 in "gather" (register: R = 8,
    h = 256, k in {8, 16, 32}) or "banked" (bank-ordered selectors: R = 8, k = 32)
    form; phase 2 as the product's.  Same FMAs in the same order as
    MaxKGraph.backward_multi's LDS form: the same bits."""
    L = load()
    R, k, h = values.shape[1], sel.shape[1], grad.shape[2]
    if form == "gather" and not (R == 8 and h == 256 and k in (8, 16, 32)):
        raise RuntimeError("the gather form needs R = 8, h = 256 and k in {8, 16, 32}")
    if form == "banked" and not (R == 8 and k == 32):
        raise RuntimeError("the banked form needs R = 8 and k = 32")
    if form not in ("gather", "banked"):
        raise RuntimeError(f"unknown form {form!r}")
    if out is None:
        out = torch.empty((g.num_cols, k), dtype=torch.float32, device=g.device)
    cabi = _lib.MAXK_BWD_EDGE_GATHER if edge_order else _lib.MAXK_BWD_STAGED
    csc_pos, csc_indptr, csc_sched, CP = g.csc()
    if edge_order:
        csc_pos = g.csc_perm()
    ws = torch.empty(max(1, L.maxk_backward_workspace_bytes(cabi, g.num_edges, k, CP)),
                     dtype=torch.uint8, device=g.device)
    fn, sel_arg = L.maxk_sspmm_backward_multi_gather, sel
    if form == "banked":
        # this call's selectors bank-ordered, each | its original entry << 8
        sp = torch.empty((g.num_cols, k), dtype=torch.int16, device=g.device)
        _lib.check(L.maxk_cbsr_bank_order_ex(None, sel.data_ptr(), g.num_cols, k, R, None, None,
                                             sp.data_ptr(), _stream(out)), "maxk_cbsr_bank_order_ex")
        fn, sel_arg = L.maxk_sspmm_backward_multi_banked, sp
    _lib.check(fn(
        cabi, g.bwd_sched.data_ptr(), g.bwd_num_panels, g.indptr.data_ptr(), g.indices.data_ptr(),
        values.data_ptr(), R, grad.data_ptr(), sel_arg.data_ptr(), g.num_rows, g.num_cols,
        g.num_edges, h, k, out.data_ptr(), csc_pos.data_ptr(), csc_sched.data_ptr(), CP,
        csc_indptr.data_ptr(), ws.data_ptr(), ws.numel(), _stream(out)),
        "maxk_sspmm_backward_multi_" + form)
    return out


def bin_plan(g):
    """Plan of the BINNED backward (maxk_bin_plan_build on the graph's device; one
    host read of the slot count), or None when the graph has no edges or its
    destination windows would need more than BIN_MAX_SLOTS_PER_EDGE slots per
    edge plus the partly filled windows that end each bin.  Tied to bwd_sched."""
    L = load()
    E, C = g.num_edges, g.num_cols
    if E == 0:
        return None
    ws = torch.empty(max(1, L.maxk_bin_plan_workspace_bytes(E, C)), dtype=torch.uint8,
                     device=g.device)
    st = _stream(ws)
    n = ctypes.c_int64(0)
    args = (g.bwd_sched.data_ptr(), g.bwd_num_panels, g.indices.data_ptr(), E, C)
    _lib.check(L.maxk_bin_plan_build(*args, None, None, None, 0, ctypes.byref(n), ws.data_ptr(),
                                     ws.numel(), st), "maxk_bin_plan_build(count)")
    slots = int(n.value)
    nb = -(-C // MAXK_BIN_DESTS)
    if slots > BIN_MAX_SLOTS_PER_EDGE * E + nb * 8 * MAXK_BIN_WINDOW:
        return None
    pos = torch.empty(E, dtype=torch.int32, device=g.device)
    ptr = torch.empty(nb + 1, dtype=torch.int32, device=g.device)
    dst = torch.empty(slots, dtype=torch.uint8, device=g.device)
    _lib.check(L.maxk_bin_plan_build(*args, pos.data_ptr(), ptr.data_ptr(), dst.data_ptr(), slots,
                                     ctypes.byref(n), ws.data_ptr(), ws.numel(), st),
               "maxk_bin_plan_build")
    return {"bin_pos": pos, "bin_ptr": ptr, "bin_dst": dst, "num_bins": nb, "num_slots": slots}


def backward_binned(g, grad, sel, plan, edge: bool = False, values=None, out=None):
    """BINNED backward (maxk_sspmm_backward_binned): phase 1 appends each edge's
    k products into its destination bin, phase 2 sums each bin in LDS.  edge:
    read the edge selectors the graph's last esel forward wrote (as STAGED_EDGE)."""
    L = load()
    k, h = sel.shape[1], grad.shape[1]
    if k not in (8, 16, 32) or plan is None:
        raise RuntimeError("BINNED backward unsupported for this graph / shape (k in {8, 16, 32})")
    values = g.values if values is None else values
    if out is None:
        out = torch.empty((g.num_cols, k), dtype=torch.float32, device=g.device)
    sel_arg = g.make_edge_selectors(sel) if edge else sel
    ws = torch.empty(max(1, L.maxk_backward_binned_workspace_bytes(plan["num_slots"], k)),
                     dtype=torch.uint8, device=g.device)
    _lib.check(L.maxk_sspmm_backward_binned(
        g.bwd_sched.data_ptr(), g.bwd_num_panels, g.indptr.data_ptr(), g.indices.data_ptr(),
        values.data_ptr(), grad.data_ptr(), sel_arg.data_ptr(), int(edge), g.num_rows, g.num_cols,
        g.num_edges, h, k, out.data_ptr(), plan["bin_pos"].data_ptr(), plan["bin_ptr"].data_ptr(),
        plan["bin_dst"].data_ptr(), plan["num_bins"], plan["num_slots"], ws.data_ptr(), ws.numel(),
        _stream(out)), "maxk_sspmm_backward_binned")
    return out
