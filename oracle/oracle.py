"""CPU oracle for the MaxK-GNN aggregation hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg
may import this module.  The product package (``spgemm_new_amd``) never does.

Two independent restatements of the reference math are provided and checked
against each other in ``tests/test_oracle.py``:

* ``c_*``   -- ctypes wrappers around ``libmaxk_oracle.so`` (maxk_oracle.c,
  main_inputs.cpp), which follow kernels/spmm_maxk.cu:17-106,
  kernels/spmm_maxk_backward.cu:15-115, kernels/generate_meta.py:26-48 and
  kernels/main.cu:74-146 line by line;
* ``np_*``  -- vectorised numpy restatements of the same equations
  (SURVEY.md §2.3), accumulated in float64 so that they also serve as the
  high-precision reference for tolerance checks.

Parity pinning: the reference ships no golden vectors for this path; the
oracle is pinned by fixtures generated from the reference's own Python code
(``tests/golden/make_golden.py`` imports reference ``utils/models.py`` MaxK
and replays its CPU aggregation op torch.sparse.mm, utils/models.py:281-287).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libmaxk_oracle.so")
_lib = None


def build(force: bool = False) -> str:
    """Compile libmaxk_oracle.so with the committed Makefile (gcc/g++ only)."""
    if force or not os.path.exists(_LIB_PATH):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        L.oracle_warp4_count.restype = ctypes.c_longlong
        L.oracle_warp4_count.argtypes = [P, ctypes.c_int, ctypes.c_int]
        L.oracle_warp4_fill.restype = ctypes.c_longlong
        L.oracle_warp4_fill.argtypes = [P, ctypes.c_int, ctypes.c_int, P]
        I = ctypes.c_int
        L.oracle_spmm_forward.restype = I
        L.oracle_spmm_forward.argtypes = [P, ctypes.c_longlong, P, P, P, P, I, I, I, P]
        L.oracle_spmm_backward.restype = I   # rows, cols (a rectangular block), dim, k
        L.oracle_spmm_backward.argtypes = [P, ctypes.c_longlong, P, P, P, P, I, I, I, I, P]
        L.oracle_spmm_forward_csr.restype = I
        L.oracle_spmm_forward_csr.argtypes = [P, P, P, P, P, I, I, I, P]
        L.oracle_spmm_backward_csr.restype = I
        L.oracle_spmm_backward_csr.argtypes = [P, P, P, P, P, I, I, I, I, P]
        L.oracle_main_inputs.restype = ctypes.c_int
        L.oracle_main_inputs.argtypes = [ctypes.c_int, ctypes.c_longlong, ctypes.c_int,
                                         P, P, P, P]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.c_void_p)


# ----------------------------------------------------------------------------
# C restatement (ctypes)
# ----------------------------------------------------------------------------
def c_warp4(indptr: np.ndarray, warp_max_nz: int = 64) -> np.ndarray:
    """generate_meta.py:26-48 -> int32[W,4] (row, loc, len, 0)."""
    indptr = np.ascontiguousarray(indptr, dtype=np.int32)
    n = len(indptr) - 1
    w = lib().oracle_warp4_count(_p(indptr), n, warp_max_nz)
    out = np.zeros((int(w), 4), dtype=np.int32)
    w2 = lib().oracle_warp4_fill(_p(indptr), n, warp_max_nz, _p(out))
    assert w2 == w
    return out


def c_forward(warp4, indices, values, data, sel, dim_origin: int) -> np.ndarray:
    """spmm_maxk.cu:17-106 over a warp4 schedule; returns fp32[V, dim_origin]."""
    warp4 = np.ascontiguousarray(warp4, dtype=np.int32).reshape(-1, 4)
    data = np.ascontiguousarray(data, dtype=np.float32)
    sel = np.ascontiguousarray(sel, dtype=np.uint8)
    v, k = data.shape
    out = np.zeros((v, dim_origin), dtype=np.float32)
    rc = lib().oracle_spmm_forward(_p(warp4), len(warp4), _p(np.ascontiguousarray(indices, np.int32)),
                                   _p(np.ascontiguousarray(values, np.float32)), _p(data), _p(sel),
                                   v, dim_origin, k, _p(out))
    if rc != 0:
        raise ValueError(f"oracle_spmm_forward failed ({rc})")
    return out


def c_backward(warp4, indices, values, grad, sel) -> np.ndarray:
    """spmm_maxk_backward.cu:15-115 over a warp4 schedule; returns fp32[V, k]."""
    warp4 = np.ascontiguousarray(warp4, dtype=np.int32).reshape(-1, 4)
    grad = np.ascontiguousarray(grad, dtype=np.float32)
    sel = np.ascontiguousarray(sel, dtype=np.uint8)
    v, h = grad.shape
    c, k = sel.shape          # dXs rows = A's columns (a rank's block has halo columns)
    out = np.zeros((c, k), dtype=np.float32)
    rc = lib().oracle_spmm_backward(_p(warp4), len(warp4), _p(np.ascontiguousarray(indices, np.int32)),
                                    _p(np.ascontiguousarray(values, np.float32)), _p(grad), _p(sel),
                                    v, c, h, k, _p(out))
    if rc != 0:
        raise ValueError(f"oracle_spmm_backward failed ({rc})")
    return out


def c_forward_csr(indptr, indices, values, data, sel, dim_origin: int) -> np.ndarray:
    data = np.ascontiguousarray(data, dtype=np.float32)
    sel = np.ascontiguousarray(sel, dtype=np.uint8)
    v, k = data.shape
    out = np.empty((v, dim_origin), dtype=np.float32)
    lib().oracle_spmm_forward_csr(_p(np.ascontiguousarray(indptr, np.int32)),
                                  _p(np.ascontiguousarray(indices, np.int32)),
                                  _p(np.ascontiguousarray(values, np.float32)), _p(data), _p(sel),
                                  v, dim_origin, k, _p(out))
    return out


def c_backward_csr(indptr, indices, values, grad, sel) -> np.ndarray:
    grad = np.ascontiguousarray(grad, dtype=np.float32)
    sel = np.ascontiguousarray(sel, dtype=np.uint8)
    v, h = grad.shape
    c, k = sel.shape          # dXs rows = A's columns
    out = np.empty((c, k), dtype=np.float32)
    rc = lib().oracle_spmm_backward_csr(_p(np.ascontiguousarray(indptr, np.int32)),
                                        _p(np.ascontiguousarray(indices, np.int32)),
                                        _p(np.ascontiguousarray(values, np.float32)), _p(grad),
                                        _p(sel), v, c, h, k, _p(out))
    if rc != 0:
        raise ValueError(f"oracle_spmm_backward_csr failed ({rc})")
    return out


def c_main_inputs(num_rows: int, num_edges: int, dim_k: int, densify: bool = False):
    """main.cu:74-146 -> (values fp32[E], data fp32[V,k], sel uint8[V,k], dense|None)."""
    values = np.empty(num_edges, dtype=np.float32)
    data = np.empty((num_rows, dim_k), dtype=np.float32)
    sel = np.empty((num_rows, dim_k), dtype=np.uint8)
    dense = np.empty((num_rows, 256), dtype=np.float32) if densify else None
    rc = lib().oracle_main_inputs(num_rows, num_edges, dim_k, _p(values), _p(data), _p(sel),
                                  _p(dense) if dense is not None else None)
    if rc != 0:
        raise ValueError(f"oracle_main_inputs failed ({rc})")
    return values, data, sel, dense


# ----------------------------------------------------------------------------
# numpy restatement (float64 accumulation)
# ----------------------------------------------------------------------------
def np_warp4(indptr: np.ndarray, warp_max_nz: int = 64) -> np.ndarray:
    indptr = np.asarray(indptr, dtype=np.int64)
    deg = np.diff(indptr)
    nch = (deg + warp_max_nz - 1) // warp_max_nz
    rows = np.repeat(np.arange(len(deg)), nch)
    first = np.repeat(np.cumsum(nch) - nch, nch)
    j = np.arange(len(rows)) - first
    loc = indptr[rows] + j * warp_max_nz
    ln = np.minimum(warp_max_nz, indptr[rows + 1] - loc)
    return np.stack([rows, loc, ln, np.zeros_like(rows)], axis=1).astype(np.int32)


def densify(data: np.ndarray, sel: np.ndarray, dim_origin: int) -> np.ndarray:
    """scatter(CBSR) -> dense [V, dim_origin] (main.cu:135-146)."""
    v, k = data.shape
    dense = np.zeros((v, dim_origin), dtype=np.float64)
    np.put_along_axis(dense, sel.astype(np.int64), data.astype(np.float64), axis=1)
    return dense


def np_forward(indptr, indices, values, data, sel, dim_origin: int) -> np.ndarray:
    """Y = A . scatter(CBSR) in float64."""
    indptr = np.asarray(indptr, dtype=np.int64)
    v = len(indptr) - 1
    xs = densify(data, sel, dim_origin)
    rows = np.repeat(np.arange(v), np.diff(indptr))
    out = np.zeros((v, dim_origin), dtype=np.float64)
    np.add.at(out, rows, np.asarray(values, np.float64)[:, None] * xs[np.asarray(indices)])
    return out


def np_backward(indptr, indices, values, grad, sel) -> np.ndarray:
    """dXs[c,l] = sum_{e: idx[e]=c} val[e] * G[row(e), sel[c,l]] in float64."""
    indptr = np.asarray(indptr, dtype=np.int64)
    v = len(indptr) - 1
    rows = np.repeat(np.arange(v), np.diff(indptr))
    cols = np.asarray(indices, dtype=np.int64)
    agt = np.zeros((sel.shape[0], grad.shape[1]), dtype=np.float64)   # A^T G (A may be v x C)
    np.add.at(agt, cols, np.asarray(values, np.float64)[:, None] * np.asarray(grad, np.float64)[rows])
    return np.take_along_axis(agt, sel.astype(np.int64), axis=1)


def np_spmm_dense(indptr, indices, values, x) -> np.ndarray:
    """Dense SpMM Y = A . X in float64: cuSPARSE SpMM (kernels/spmm_cusparse.cu:6-62)
    and, with values = 1, GNNAdvisor's SAG aggregation (kernels/spmm_gnna.cu:60-140)."""
    indptr = np.asarray(indptr, dtype=np.int64)
    v = len(indptr) - 1
    rows = np.repeat(np.arange(v), np.diff(indptr))
    out = np.zeros((v, x.shape[1]), dtype=np.float64)
    np.add.at(out, rows, np.asarray(values, np.float64)[:, None] *
              np.asarray(x, np.float64)[np.asarray(indices)])
    return out


def np_cbsr(x: np.ndarray, k: int):
    """Top-k CBSR producer (torch.topk semantics: descending values)."""
    idx = np.argsort(-x, axis=1, kind="stable")[:, :k]
    return np.take_along_axis(x, idx, axis=1).astype(np.float32), idx.astype(np.uint8)


def parity_error(got: np.ndarray, ref: np.ndarray) -> float:
    """max |got-ref| / max(1, |ref|) -- the per-element 1e-4 criterion."""
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    if got.shape != ref.shape:
        raise ValueError(f"shape mismatch {got.shape} vs {ref.shape}")
    if got.size == 0:
        return 0.0
    return float(np.max(np.abs(got - ref) / np.maximum(1.0, np.abs(ref))))
