"""Functional module mirroring the reference's ``maxk_cuda_kernels`` extension
(cuda_kernel_bindings.cpp:429-490), on MI355X.

Same names, argument meaning and error behaviour (RuntimeError on a bad
device / dtype, like TORCH_CHECK).  Differences, all deliberate:

* launches are asynchronous on the current HIP stream (the reference used the
  legacy default stream, cuda_kernel_wrappers.cu:46,66);
* the reference's defects are not reproduced: every k works,
  the top-k is exact (torch.topk semantics, not the lossy uint8 kernel of
  cuda_kernel_bindings.cpp:203-238).

A reference caller switches with ``sys.modules["maxk_cuda_kernels"] =
spgemm_new_amd.maxk_cuda_kernels``.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import _lib
from .ops import MaxKGraph, check_tensor, topk_cbsr, warp4_build

FULL_DIM = 256  # cuda_kernel_bindings.cpp:70


def _warp4_checks(warp4_metadata, indices, values, input_data, sparse_selector):
    check_tensor(warp4_metadata, "warp4_metadata", torch.int32)
    check_tensor(indices, "indices", torch.int32)
    check_tensor(values, "values", torch.float32)
    check_tensor(input_data, "input_data", torch.float32)
    check_tensor(sparse_selector, "sparse_selector", torch.uint8)


_W4_GRAPHS: "OrderedDict" = None


def _warp4_graph(warp4, indices, values, num_v: int, num_warps: int):
    """The CSR graph behind a warp4 chunk list, or None.

    generate_meta.py:26-48 cuts each row's edges, in order, into chunks
    (row, loc, len, 0); so indptr follows from the lengths, and the fast
    panel-scheduled kernels (no pre-zeroing, LOCAL backward) give the same
    result as the chunk kernels.  Used only when all chunks are processed
    (num_warps covers the list) and the list is exactly such a cut of the
    edges (rows non-decreasing and < V, loc = running edge offset, lengths sum
    to E); otherwise the caller keeps the warp4 kernels.  Cached per
    (warp4, indices, values) tensor state."""
    global _W4_GRAPHS
    from collections import OrderedDict
    if _W4_GRAPHS is None:
        _W4_GRAPHS = OrderedDict()
    n_chunks = warp4.numel() // 4
    if num_warps != n_chunks or warp4.numel() % 4:
        return None
    key = tuple((t.data_ptr(), t.numel(), t._version) for t in (warp4, indices, values)) + (num_v,)
    if key in _W4_GRAPHS:
        _W4_GRAPHS.move_to_end(key)
        return _W4_GRAPHS[key][0]
    w = warp4.view(-1, 4).long()
    rows, loc, ln = w[:, 0], w[:, 1], w[:, 2]
    E = indices.numel()
    ok = True
    if n_chunks:
        start = torch.cumsum(ln, 0) - ln
        ok = bool(((rows >= 0) & (rows < num_v) & (ln >= 0)).all()) \
            and bool((rows[1:] >= rows[:-1]).all()) and torch.equal(loc, start) \
            and int(ln.sum()) == E
    else:
        ok = E == 0
    g = None
    if ok:
        counts = torch.zeros(num_v, dtype=torch.int64, device=warp4.device)
        if n_chunks:
            counts.index_add_(0, rows, ln)
        indptr = torch.zeros(num_v + 1, dtype=torch.int32, device=warp4.device)
        indptr[1:] = torch.cumsum(counts, 0).to(torch.int32)
        g = MaxKGraph(indptr, indices, values)
    # the entry keeps warp4/indices/values alive, so their addresses are not reused
    _W4_GRAPHS[key] = (g, warp4, indices, values)
    while len(_W4_GRAPHS) > 8:
        _W4_GRAPHS.popitem(last=False)
    return g


def spmm_maxk_forward(warp4_metadata, indices, values, input_data, sparse_selector, num_warps,
                      dim_sparse):
    """cuda_kernel_bindings.cpp:42-104 -> fp32[V, 256]."""
    _warp4_checks(warp4_metadata, indices, values, input_data, sparse_selector)
    num_v = input_data.size(0)
    g = _warp4_graph(warp4_metadata, indices, values, num_v, int(num_warps))
    if g is not None and sparse_selector.size(1) == int(dim_sparse):
        return g.forward(input_data, sparse_selector, FULL_DIM)
    output = torch.zeros((num_v, FULL_DIM), dtype=torch.float32, device=input_data.device)
    num_warps = min(int(num_warps), warp4_metadata.numel() // 4)
    L = _lib.load()
    _lib.check(L.maxk_spmm_forward_warp4(
        warp4_metadata.data_ptr(), indices.data_ptr(), values.data_ptr(), input_data.data_ptr(),
        sparse_selector.data_ptr(), output.data_ptr(), num_v, indices.numel(), FULL_DIM,
        int(dim_sparse), num_warps, _lib.stream_ptr(input_data.device)), "CUDA kernel failed")
    return output


def spmm_maxk_backward(warp4_metadata, indices, values, grad_output, sparse_selector, num_warps,
                       dim_sparse):
    """cuda_kernel_bindings.cpp:106-161 -> fp32[V, dim_sparse]."""
    check_tensor(warp4_metadata, "warp4_metadata", torch.int32)
    check_tensor(indices, "indices", torch.int32)
    check_tensor(values, "values", torch.float32)
    check_tensor(grad_output, "grad_output", torch.float32)
    check_tensor(sparse_selector, "sparse_selector", torch.uint8)
    num_v, feat_in = grad_output.size(0), grad_output.size(1)
    g = _warp4_graph(warp4_metadata, indices, values, num_v, int(num_warps))
    if g is not None and sparse_selector.size(1) == int(dim_sparse) \
            and sparse_selector.size(0) == num_v:
        return g.backward(grad_output, sparse_selector)
    grad_input = torch.zeros((num_v, int(dim_sparse)), dtype=torch.float32,
                             device=grad_output.device)
    num_warps = min(int(num_warps), warp4_metadata.numel() // 4)
    L = _lib.load()
    _lib.check(L.maxk_spmm_backward_warp4(
        warp4_metadata.data_ptr(), indices.data_ptr(), values.data_ptr(), grad_output.data_ptr(),
        sparse_selector.data_ptr(), grad_input.data_ptr(), num_v, indices.numel(), feat_in,
        int(dim_sparse), num_warps, _lib.stream_ptr(grad_output.device)), "CUDA kernel failed")
    return grad_input


def load_warp4_metadata(graph_name: str, num_warps: int = 12, warp_max_nz: int = 64):
    """cuda_kernel_bindings.cpp:287-317: read kernels/w{nw}_nz{nz}_warp_4/<g>.warp4."""
    path = os.path.join("kernels", f"w{num_warps}_nz{warp_max_nz}_warp_4", graph_name + ".warp4")
    if not os.path.exists(path):
        raise RuntimeError("Cannot open warp4 file: " + path)
    arr = np.fromfile(path, dtype=np.int32)
    return torch.from_numpy(arr).cuda()


def build_warp4_metadata(indptr, warp_max_nz: int = 64):
    """On-device replacement of kernels/generate_meta.py (no file round trip)."""
    return warp4_build(indptr, warp_max_nz)


class CudaTimer:
    """cuda_kernel_bindings.cpp:343-369 (events on the current stream)."""

    def __init__(self):
        self._s = torch.cuda.Event(enable_timing=True)
        self._e = torch.cuda.Event(enable_timing=True)

    def start(self):
        self._s.record()

    def stop(self) -> float:
        self._e.record()
        self._e.synchronize()
        return float(self._s.elapsed_time(self._e))


def benchmark_spmm_maxk(warp4_metadata, indices, values, input_data, sparse_selector, num_warps,
                        dim_sparse, num_runs: int = 4):
    """cuda_kernel_bindings.cpp:372-402: num_runs warm-up + num_runs timed (ms each)."""
    for _ in range(num_runs):
        spmm_maxk_forward(warp4_metadata, indices, values, input_data, sparse_selector, num_warps,
                          dim_sparse)
    torch.cuda.synchronize()
    t = CudaTimer()
    times = []
    for _ in range(num_runs):
        t.start()
        spmm_maxk_forward(warp4_metadata, indices, values, input_data, sparse_selector, num_warps,
                          dim_sparse)
        times.append(t.stop())
    return times


def validate_spmm_maxk(warp4_metadata, indices, values, input_data, sparse_selector,
                       reference_output, num_warps, dim_sparse, tolerance: float = 0.001):
    """cuda_kernel_bindings.cpp:405-427: mean |diff| < tolerance."""
    out = spmm_maxk_forward(warp4_metadata, indices, values, input_data, sparse_selector,
                            num_warps, dim_sparse)
    diff = (out - reference_output).abs()
    max_diff, avg_diff = float(diff.max()), float(diff.mean())
    print(f"Validation - Max diff: {max_diff}, Avg diff: {avg_diff}")
    return avg_diff < tolerance


# --------------------------------------------------------------------- top-k
def cuda_topk_maxk_float(input, k: int):
    """Top-k with the contract of cuda_kernel_bindings.cpp:203-238: float32 in ->
    (fp32 values[V,k], int32 indices[V,k]), exact (the HIP CBSR producer in
    torch.topk's order, not the lossy uint8-quantised kernel);
    uint8 in -> (uint8 values, int32 indices) through the uint8 path."""
    check_tensor(input, "Input", dim=2)
    if not (0 < k <= input.size(1)):
        raise RuntimeError("Invalid k value")
    if input.dtype == torch.uint8:
        vals, idx = cuda_topk_maxk(input, k)
        return vals, idx.to(torch.int32)
    if input.dtype != torch.float32:
        raise RuntimeError("Input must be float32 or uint8")
    vals, idx = topk_cbsr(input.contiguous(), k, order="value")  # HIP producer (dim <= 256)
    return vals, idx.to(torch.int32)


def cuda_topk_maxk(input, k: int):
    """uint8 top-k (cuda_kernel_bindings.cpp:164-200) -> (uint8 values, uint8 indices)."""
    check_tensor(input, "Input", torch.uint8, dim=2)
    if not (0 < k <= input.size(1)):
        raise RuntimeError("Invalid k value")
    vals, idx = torch.topk(input.int(), k, dim=1)
    return vals.to(torch.uint8), idx.to(torch.uint8)


def prepare_cbsr_format_maxk(features, maxk: int):
    """cuda_kernel_bindings.cpp:240-252 -> (fp32[V,k], int32[V,k])."""
    return cuda_topk_maxk_float(features, maxk)


def generate_sparse_selector(num_v: int, dim_origin: int, dim_sparse: int):
    """cuda_kernel_bindings.cpp:320-340: k distinct random columns per row (uint8)."""
    g = torch.Generator(device="cuda")
    g.manual_seed(123)
    r = torch.rand((num_v, dim_origin), generator=g, device="cuda")
    return torch.argsort(r, dim=1)[:, :dim_sparse].to(torch.uint8).contiguous()


def cusparse_spmm(indptr, indices, values, input_features, timing: bool = False):
    """Vendor dense-SpMM cross-check (cuda_kernel_bindings.cpp:254-284): rocSPARSE via
    torch.sparse on the GPU.  A checker, not the hot path."""
    n = indptr.numel() - 1
    a = torch.sparse_csr_tensor(indptr.long(), indices.long(), values, size=(n, n))
    return torch.sparse.mm(a, input_features)


def spmm_maxk_forward_graph(graph: MaxKGraph, input_data, sparse_selector, dim_origin=FULL_DIM):
    """Fast path (merge-path panels, no pre-zeroing) for callers that hold indptr."""
    return graph.forward(input_data, sparse_selector, dim_origin)


def spmm_maxk_backward_graph(graph: MaxKGraph, grad_output, sparse_selector, algo=0):
    return graph.backward(grad_output, sparse_selector, algo=algo)
