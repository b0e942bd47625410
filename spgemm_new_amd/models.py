"""Autograd surface mirroring the op part of the reference's utils/models.py:28-149.

``MaxK.apply(x, k)`` and ``SpGEMMFunction.apply(features, (indptr, indices,
values), maxk)`` have the reference's names, arguments and return values, so
the training loop (maxk_gnn_integrated.py, SAGE.forward utils/models.py:230)
calls them unchanged.  The hot path is the HIP SpGEMM / SSpMM; the CBSR
producer is torch.topk (SURVEY.md §8f1 lists a fused HIP top-k as next).

Fixed relative to the reference: the kernel path actually runs,
there is no per-layer debug copy, and the sparse->dense gradient scatter is a
single on-device scatter instead of a V*k Python loop (utils/models.py:136-141).
No fallback: if the HIP library is missing the call raises.
"""
from __future__ import annotations

import torch
from torch.autograd import Function

from .graph_cache import graph_for


class MaxK(Function):
    """utils/models.py:28-59: keep the k largest entries per row; gradient masked."""

    @staticmethod
    def forward(ctx, input, k=1):
        _, indices = input.topk(k, dim=1)
        mask = torch.zeros_like(input)
        mask.scatter_(1, indices, 1)
        ctx.save_for_backward(mask)
        return input * mask

    @staticmethod
    def backward(ctx, grad_output):
        (mask,) = ctx.saved_tensors
        return grad_output * mask, None


def cbsr_topk(features: torch.Tensor, maxk: int):
    """(data fp32[V,k], sel uint8[V,k]) = top-k of each row (direct_kernel_interface.py:79-83)."""
    vals, idx = torch.topk(features, maxk, dim=1)
    return vals.contiguous(), idx.to(torch.uint8).contiguous()


class SpGEMMFunction(Function):
    """utils/models.py:61-149: forward Y = A . topk_k(X), backward mask . (A^T G)."""

    @staticmethod
    def forward(ctx, features, graph_data, maxk):
        indptr, indices, values = graph_data
        if features.dim() != 2:
            raise RuntimeError("features must be 2D")
        x = features.contiguous()
        data, sel = cbsr_topk(x, maxk)
        g = graph_for(indptr.contiguous(), indices.contiguous(), values.contiguous())
        out = g.forward(data, sel, dim_origin=x.size(1))
        ctx.graph = g
        ctx.sparse_selector = sel
        ctx.maxk = maxk
        ctx.features_shape = x.shape
        return out

    @staticmethod
    def backward(ctx, grad_output):
        g = ctx.graph
        sel = ctx.sparse_selector
        dxs = g.backward(grad_output.contiguous(), sel)
        grad_input = torch.zeros(ctx.features_shape, dtype=grad_output.dtype,
                                 device=grad_output.device)
        grad_input.scatter_(1, sel.long(), dxs)
        return grad_input, None, None
