"""ctypes binding of the C ABI declared in include/maxk_spgemm.h.

This is the thin shim that replaces the reference's pybind11/torch extension
(cuda_kernel_bindings.cpp:429-490).  The shared library is built in-tree by
``__graft_entry__.build()`` (hipcc --offload-arch=gfx950) into
``spgemm_new_amd/lib/libmaxk_spgemm.so``.  There is no fallback: if the library
is missing every entry point raises.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  -- must be imported first so its HIP runtime is the one we bind to

_HERE = os.path.dirname(os.path.abspath(__file__))
# MAXK_LIB overrides the library path (variant builds in development tools)
LIB_PATH = os.environ.get("MAXK_LIB") or os.path.join(_HERE, "lib", "libmaxk_spgemm.so")
SOURCES = [os.path.join(_HERE, "csrc", "maxk_spgemm.hip")]
HEADER = os.path.join(os.path.dirname(_HERE), "include", "maxk_spgemm.h")

MAXK_OK = 0
MAXK_E_ARG = -1
MAXK_E_DIM = -2
MAXK_E_WORKSPACE = -3
MAXK_BWD_AUTO = 0
MAXK_BWD_ATOMIC = 1
MAXK_BWD_STAGED = 2
MAXK_BWD_LOCAL = 3
MAXK_BWD_TILE = 4
MAXK_BWD_STAGED_EDGE = 5
MAXK_BWD_EDGE_GATHER = 6
MAXK_BWD_APPEND = 7     # write-combined propagation blocking (non-deterministic order)
# Python level: APPEND reading the forward's edge selectors (the C entry's edge_sel = 1)
MAXK_BWD_APPEND_EDGE = 8
# backward_multi only (Python level; the C entry is maxk_sspmm_backward_multi with
# MAXK_BWD_STAGED / MAXK_BWD_EDGE_GATHER): relations summed per edge in phase 1
MAXK_BWD_MULTI_STAGED = 16
MAXK_BWD_MULTI_EDGE_GATHER = 17
MAXK_BWD_MULTI_APPEND = 18   # maxk_sspmm_backward_append with num_rel > 1
MAXK_TOPK_ORDER_COLUMN = 0
MAXK_TOPK_ORDER_VALUE = 1
MAXK_TOPK_ORDER_LANE = 2
MAXK_FWD_ACCUMULATE = 1
MAXK_FWD_CACHED_GATHER = 2
DEFAULT_PANEL_COST = 2048
DEFAULT_ROW_COST = 16

# include/maxk_spgemm.h MAXK_ABI_VERSION: the library must report the same
ABI_VERSION = 6

_ERRORS = {MAXK_E_ARG: "invalid argument", MAXK_E_DIM: "invalid dimension (dim_origin must be "
           "<= 256 and 1 <= dim_k <= dim_origin)", MAXK_E_WORKSPACE: "workspace too small"}

# name -> (restype, argtypes); every symbol here is declared in include/maxk_spgemm.h
_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_int64
_S = ctypes.c_size_t
SIGNATURES = {
    "maxk_version": (ctypes.c_char_p, []),
    "maxk_abi_version": (_I, []),
    "maxk_schedule_num_panels": (_I, [_L, _L, _I, _I, ctypes.POINTER(ctypes.c_int64)]),
    "maxk_schedule_build": (_I, [_P, _I, _I, _I, _P, _L, _P]),
    "maxk_warp4_build": (_I, [_P, _I, _I, _P, _P, _L, ctypes.POINTER(ctypes.c_int64), _P]),
    "maxk_forward_workspace_bytes": (_S, [_L, _I]),
    "maxk_spgemm_forward": (_I, [_P, _L, _P, _P, _P, _P, _P, _I, _I, _I, _P, _P, _S, _P]),
    "maxk_spgemm_forward_ex": (_I, [_P, _L, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P, _P, _S, _P]),
    "maxk_backward_workspace_bytes": (_S, [_I, _L, _I, _L]),
    "maxk_sspmm_backward": (_I, [_I, _P, _L, _P, _P, _P, _P, _P, _I, _I, _L, _I, _I, _P, _P, _P,
                                 _L, _P, _P, _S, _P]),
    "maxk_backward_local_lds_bytes": (_S, [_I, _I]),
    "maxk_sspmm_backward_local": (_I, [_P, _I, _P, _I, _I, _P, _P, _P, _P, _I, _I, _I, _P, _P]),
    "maxk_grad_interleave": (_I, [_P, _I, _I, _I, _P, _P]),
    "maxk_sspmm_backward_local_rel8": (_I, [_P, _I, _P, _I, _I, _P, _P, _P, _P, _I, _I, _I, _P,
                                            _P]),
    "maxk_append_bins": (_I, [_I, _I, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "maxk_append_plan_build": (_I, [_P, _L, _P, _P, _I, _I, _I, _P, _I, _I, _P]),
    "maxk_backward_append_workspace_bytes": (_S, [_L, _I, _I]),
    "maxk_sspmm_backward_append": (_I, [_P, _L, _P, _P, _P, _I, _P, _P, _I, _I, _I, _L, _I, _I,
                                        _P, _I, _I, _P, _P, _S, _P]),
    "maxk_sspmm_backward_multi": (_I, [_I, _P, _L, _P, _P, _P, _I, _P, _P, _I, _I, _L, _I, _I, _P,
                                       _P, _P, _L, _P, _P, _S, _P]),
    "maxk_sspmm_backward_tile": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _P, _P, _P, _I, _I, _I, _I,
                                      _P, _P, _P]),
    "maxk_tile_format": (_I, [ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    "maxk_tile_record_words": (_I, []),
    "maxk_blocked_plan_workspace_bytes": (_S, [_L, _I, _I]),
    "maxk_blocked_plan_build": (_I, [_P, _P, _P, _I, _I, _L, _I, _P, _P, _P, _P, _P, _S, _P]),
    "maxk_permute_f32": (_I, [_P, _P, _L, _P, _P]),
    "maxk_rows_sum": (_I, [_P, _I, _L, _P, _P]),
    "maxk_spgemm_forward_sum_parts": (_I, [_P, _L, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P, _I, _P, _P, _S, _P]),
    "maxk_tile_plan_shape": (_I, [_I, _I, _I, _I, ctypes.POINTER(_I), ctypes.POINTER(_I),
                                  ctypes.POINTER(_I)]),
    "maxk_tile_plan_workspace_bytes": (_S, [_L, _I, _I]),
    "maxk_tile_part_planes": (_I, [_I, _I, _I]),
    "maxk_tile_plan_build": (_I, [_P, _P, _P, _I, _I, _L, _I, _I, _I, _I, _P, _L, _P, _P, _L, _P,
                                  _P, _P, ctypes.POINTER(ctypes.c_int64), _P, _S, _P]),
    "maxk_tile_plan_set_values": (_I, [_P, _P, _L, _P, _P]),
    "maxk_cbsr_packed_row_bytes": (_S, [_I]),
    "maxk_cbsr_pack": (_I, [_P, _P, _I, _I, _P, _P]),
    "maxk_spgemm_forward_esel": (_I, [_P, _L, _P, _P, _P, _P, _P, _P, _I, _I, _I, _P, _P, _P, _S,
                                      _P]),
    "maxk_spgemm_forward_packed": (_I, [_P, _L, _P, _P, _P, _P, _I, _I, _I, _P, _P, _S, _P]),
    "maxk_csc_workspace_bytes": (_S, [_L, _I]),
    "maxk_csc_build": (_I, [_P, _L, _I, _P, _P, _P, _S, _P]),
    "maxk_csc_perm_build": (_I, [_P, _L, _P, _P]),
    "maxk_local_plan_workspace_bytes": (_S, [_L, _I, _I]),
    "maxk_local_plan_build": (_I, [_P, _P, _P, _I, _I, _L, _P, _I, _I, _P, _P, _P, _P, _P, _P, _P,
                                   _S, _P]),
    "maxk_local_bands_build": (_I, [_P, _P, _I, _I, _I, _P, _P]),
    "maxk_spmm_dense_forward": (_I, [_P, _L, _P, _P, _P, _P, _I, _I, _P, _P, _S, _P]),
    "maxk_spmm_gnna_sag": (_I, [_P, _L, _P, _P, _P, _I, _P, _P]),
    "maxk_forward_multi_workspace_bytes": (_S, [_L, _I, _I]),
    "maxk_spgemm_forward_multi": (_I, [_P, _L, _P, _P, _P, _I, _P, _P, _I, _I, _I, _P, _P, _S, _P]),
    "maxk_records_sel_gather": (_I, [_P, _I, _P, _L, _P, _P]),
    "maxk_cbsr_gather_records": (_I, [_P, _P, _P, _L, _I, _P, _P]),
    "maxk_spgemm_forward_records": (_I, [_P, _L, _P, _P, _P, _P, _I, _I, _I, _I, _P, _P, _S, _P]),
    "maxk_cbsr_bank_order": (_I, [_P, _P, _I, _I, _I, _P, _P, _P]),
    "maxk_segment_rows_add": (_I, [_P, _I, _P, _P, _P, _L, _P, _P]),
    "maxk_topk_cbsr": (_I, [_P, _I, _I, _L, _I, _I, _P, _P, _P, _P]),
    "maxk_cbsr_scatter": (_I, [_P, _P, _I, _I, _I, _P, _P]),
    "maxk_cbsr_mask": (_I, [_P, _P, _I, _I, _I, _P, _P]),
    "maxk_spmm_forward_warp4": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P]),
    "maxk_spmm_backward_warp4": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P]),
}

_lib = None


class MaxKError(RuntimeError):
    pass


def _stale(why):
    return MaxKError(f"{LIB_PATH} was built from other sources than these bindings ({why}); "
                     "rebuild it with `python -c 'import __graft_entry__ as g; g.build()'`")


def load():
    """Load the HIP library (raises if it has not been built, or if it was built
    from sources whose ABI differs from these bindings: an entry point whose
    arguments changed would otherwise bind without error and be called wrongly)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise MaxKError(
                f"MI355X HIP library not found at {LIB_PATH}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
        L = ctypes.CDLL(LIB_PATH)
        try:
            abi = L.maxk_abi_version
        except AttributeError:
            raise _stale("no maxk_abi_version: older than ABI 5") from None
        abi.restype, abi.argtypes = _I, []
        if abi() != ABI_VERSION:
            raise _stale(f"library ABI {abi()}, bindings ABI {ABI_VERSION}")
        for name, (res, args) in SIGNATURES.items():
            try:
                f = getattr(L, name)
            except AttributeError:
                raise _stale(f"{name} missing") from None
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc: int, what: str) -> None:
    if rc != MAXK_OK:
        if rc < 0:
            raise MaxKError(f"{what}: {_ERRORS.get(rc, 'error')} ({rc})")
        raise MaxKError(f"{what}: HIP error {rc}")


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()
