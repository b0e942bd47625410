"""Autograd surface mirroring the op part of the reference's utils/models.py:28-149.

``MaxK.apply(x, k)`` and ``SpGEMMFunction.apply(features, (indptr, indices,
values), maxk)`` have the reference's names, arguments and return values, so
the training loop (maxk_gnn_integrated.py, SAGE.forward utils/models.py:230)
calls them unchanged.  Every step runs in the HIP library: the top-k CBSR
producer (maxk_topk_cbsr, replacing torch.topk), the SpGEMM / SSpMM, and the
sparse->dense gradient scatter / MaxK mask (maxk_cbsr_scatter / _mask).

Fixed relative to the reference: the kernel path actually runs,
there is no per-layer debug copy, and the sparse->dense gradient scatter is a
single device kernel instead of a V*k Python loop (utils/models.py:136-141).
No fallback: if the HIP library is missing the call raises.
"""
from __future__ import annotations

import torch
from torch.autograd import Function

from .graph_cache import graph_for
from .ops import cbsr_mask, cbsr_scatter, topk_cbsr


class MaxK(Function):
    """utils/models.py:28-59: keep the k largest entries per row; gradient masked."""

    @staticmethod
    def forward(ctx, input, k=1):
        # the HIP producer's domain; no fallback outside it (a CPU or fp64 tensor raises)
        if input.dim() != 2 or input.size(1) > 256:
            raise RuntimeError("MaxK: input must be 2-D with at most 256 columns")
        _, sel, out = topk_cbsr(input.contiguous(), k, dense=True)
        ctx.save_for_backward(sel)
        return out

    @staticmethod
    def backward(ctx, grad_output):
        (sel,) = ctx.saved_tensors
        return cbsr_mask(grad_output.contiguous(), sel), None


def cbsr_topk(features: torch.Tensor, maxk: int, order: str = "value"):
    """(data fp32[V,k], sel uint8[V,k]) = top-k of each row (direct_kernel_interface.py:79-83),
    by the HIP producer; order="value" is torch.topk's sorted order."""
    return topk_cbsr(features.contiguous(), maxk, order=order)


class SpGEMMFunction(Function):
    """utils/models.py:61-149: forward Y = A . topk_k(X), backward mask . (A^T G)."""

    @staticmethod
    def forward(ctx, features, graph_data, maxk):
        indptr, indices, values = graph_data
        if features.dim() != 2:
            raise RuntimeError("features must be 2D")
        x = features.contiguous()
        data, sel = topk_cbsr(x, maxk, order="column")
        g = graph_for(indptr.contiguous(), indices.contiguous(), values.contiguous())
        # edge selectors only when this forward's backward will run
        out = g.forward(data, sel, dim_origin=x.size(1),
                        edge_sel="auto" if ctx.needs_input_grad[0] else False)
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
        return cbsr_scatter(dxs, sel, ctx.features_shape[1]), None, None


class SpGEMMMultiFunction(Function):
    """Multi-relation aggregation (BASELINE config 5, ogbn-proteins' 8 edge
    features; no reference counterpart -- the reference sums the edge features
    into node features, utils/proteins_loader.py:41-44): Y[q] = A_q . topk_k(X)
    for the relations q of values fp32[E, R].  forward -> fp32[R, V, h]
    (fused kernel); backward -> mask . sum_q A_q^T G_q."""

    @staticmethod
    def forward(ctx, features, graph_data, values, maxk):
        indptr, indices = graph_data[0], graph_data[1]
        x = features.contiguous()
        data, sel = topk_cbsr(x, maxk, order="column")
        g = graph_for(indptr.contiguous(), indices.contiguous(), None)
        vals = values.contiguous()
        out = g.forward_multi(data, sel, vals, dim_origin=x.size(1))
        ctx.graph, ctx.sparse_selector, ctx.values = g, sel, vals
        ctx.features_shape = x.shape
        return out

    @staticmethod
    def backward(ctx, grad_output):
        g, sel = ctx.graph, ctx.sparse_selector
        dxs = g.backward_multi(grad_output.contiguous(), sel, ctx.values)
        return cbsr_scatter(dxs, sel, ctx.features_shape[1]), None, None, None


class PartitionedSpGEMMFunction(Function):
    """SpGEMMFunction for one rank of a 1-D row-partitioned graph
    (spgemm_new_amd.distributed.PartitionedMaxK): the rank holds
    its own rows' features; forward = top-k of the own rows, halo exchange of
    their CBSR, local SpGEMM -> Y for the own rows; backward = local SSpMM,
    reverse exchange of the halo partial sums, dense scatter of the own rows'
    dXs.  Every rank calls it in the same order (the exchanges are collective).

        y_own = PartitionedSpGEMMFunction.apply(x_own, model, maxk)
    """

    @staticmethod
    def forward(ctx, features_own, model, maxk):
        if features_own.dim() != 2 or features_own.shape[0] != model.plan.num_own:
            raise RuntimeError("features must be the rank's own rows [num_own, h]")
        x = features_own.contiguous()
        data, sel = topk_cbsr(x, maxk, order="column")
        out = model.forward(data, sel, x.size(1))
        # the halo selectors of THIS forward (a later layer's forward reuses the buffers)
        ctx.model, ctx.sel, ctx.h = model, sel, x.size(1)
        ctx.halo_sel = model.last_halo_selectors()
        return out

    @staticmethod
    def backward(ctx, grad_output):
        dxs = ctx.model.backward(grad_output.contiguous(), ctx.sel, halo_sel=ctx.halo_sel)
        return cbsr_scatter(dxs, ctx.sel, ctx.h), None, None


class PartitionedSpGEMMMultiFunction(Function):
    """SpGEMMMultiFunction for one rank of a row-partitioned graph whose
    PartitionedMaxK holds the relations' values fp32[E, R]: forward = top-k of
    the own rows, one halo exchange shared by the R relations, fused local
    forward -> [R, own rows, h]; backward = local multi-relation SSpMM, one
    reverse exchange, dense scatter.

        y_own = PartitionedSpGEMMMultiFunction.apply(x_own, model, maxk)
    """

    @staticmethod
    def forward(ctx, features_own, model, maxk):
        if features_own.dim() != 2 or features_own.shape[0] != model.plan.num_own:
            raise RuntimeError("features must be the rank's own rows [num_own, h]")
        x = features_own.contiguous()
        data, sel = topk_cbsr(x, maxk, order="column")
        out = model.forward_multi(data, sel, x.size(1))
        ctx.model, ctx.sel, ctx.h = model, sel, x.size(1)
        ctx.halo_sel = model.last_halo_selectors()
        return out

    @staticmethod
    def backward(ctx, grad_output):
        dxs = ctx.model.backward_multi(grad_output.contiguous(), ctx.sel, halo_sel=ctx.halo_sel)
        return cbsr_scatter(dxs, ctx.sel, ctx.h), None, None
