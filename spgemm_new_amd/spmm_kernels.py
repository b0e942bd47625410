"""Class module mirroring the reference's ``spmm_kernels`` extension
(kernels/spmm_bindings.cpp:209-262): ``SpmmMaxK``, ``SpmmMaxKBackward``,
``prepare_cbsr_format``, ``topk_nonlinearity``.

Unlike the reference, ``set_sparse_params`` takes effect and
the schedule is derived from ``indptr`` on the device -- no ``.warp4`` file.
``run_kernel(timing, dim)`` keeps SPMM_BASE::timing_body's protocol
(kernels/spmm_base.h:48-77): untimed = one launch + device sync, returns 0;
timed = 4 warm-up + 4 timed launches, mean wall seconds.
"""
from __future__ import annotations

import time

import torch

from .graph_cache import graph_for
from .ops import check_tensor, topk_cbsr


def _sel_u8(sparse_selector):
    check_tensor(sparse_selector, "sparse_selector")
    if sparse_selector.dtype == torch.uint8:
        return sparse_selector
    if sparse_selector.dtype not in (torch.int32, torch.int64):
        raise RuntimeError("sparse_selector must be int32")
    return sparse_selector.to(torch.uint8).contiguous()


class _SpmmBase:
    def __init__(self, graph_name, indptr, indices, values, input_features, output_features):
        for t, n in ((indptr, "indptr"), (indices, "indices"), (values, "values"),
                     (input_features, "input_features"), (output_features, "output_features")):
            check_tensor(t, n)
        self._graph_name = graph_name
        self._graph = graph_for(indptr, indices, values)
        self._vin, self._vout = input_features, output_features
        self._sel = None
        self._k = None

    def update_input_output(self, input_features, output_features):
        check_tensor(input_features, "input_features")
        check_tensor(output_features, "output_features")
        self._vin, self._vout = input_features, output_features

    def set_sparse_params(self, sparse_selector, maxk):
        self._sel = _sel_u8(sparse_selector)
        self._k = int(maxk)

    def get_graph_name(self):
        return self._graph_name

    def _run(self, dim):
        raise NotImplementedError

    def run_kernel(self, timing: bool = False, dim: int = -1) -> float:
        if self._sel is None:
            raise RuntimeError("set_sparse_params() must be called before run_kernel()")
        if not timing:
            self._run(dim)
            torch.cuda.synchronize()
            return 0.0
        for _ in range(4):
            self._run(dim)
        torch.cuda.synchronize()
        total = 0.0
        for _ in range(4):
            t0 = time.perf_counter()
            self._run(dim)
            torch.cuda.synchronize()
            total += time.perf_counter() - t0
        return total / 4


class SpmmMaxK(_SpmmBase):
    """Forward SpGEMM (kernels/spmm_maxk.cu): vout[V,h] = A . scatter(vin[V,k], sel)."""

    def _run(self, dim):
        dim = self._vout.size(1) if dim is None or dim < 0 else dim
        if dim != self._vout.size(1):
            raise RuntimeError("dim must equal output_features.size(1)")
        self._graph.forward(self._vin, self._sel, dim, out=self._vout)


class SpmmMaxKBackward(_SpmmBase):
    """Backward SSpMM (kernels/spmm_maxk_backward.cu): vout[V,k] from vin = G[V,h]."""

    def _run(self, dim):
        if dim is not None and dim >= 0 and dim != self._vin.size(1):
            raise RuntimeError("dim must equal input_features.size(1)")
        self._graph.backward(self._vin, self._sel, out=self._vout)


def prepare_cbsr_format(features, maxk: int):
    """spmm_bindings.cpp:163-184 -> (fp32[V,k], int32[V,k]) via exact top-k."""
    check_tensor(features, "Features", dim=2)
    if not (0 < maxk <= features.size(1)):
        raise RuntimeError("Invalid maxk value")
    if features.dtype == torch.float32 and features.size(1) <= 256:
        vals, idx = topk_cbsr(features.contiguous(), maxk, order="value")  # HIP producer
        return vals, idx.to(torch.int32)
    vals, idx = torch.topk(features, maxk, dim=1)  # dim > 256: outside the kernels' range
    return vals.contiguous(), idx.to(torch.int32).contiguous()


def topk_nonlinearity(input, k: int):
    """spmm_bindings.cpp:189-204: keep the k largest entries of each row."""
    check_tensor(input, "Input", dim=2)
    if not (0 < k <= input.size(1)):
        raise RuntimeError("Invalid k value")
    if input.dtype == torch.float32 and input.size(1) <= 256:
        return topk_cbsr(input.contiguous(), k, dense=True)[2]  # HIP producer, dense form
    vals, idx = torch.topk(input, k, dim=1)
    out = torch.zeros_like(input)
    out.scatter_(1, idx, vals)
    return out
