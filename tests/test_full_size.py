"""Parity at BASELINE.json's full sizes (GPU).

The oracle finishes in seconds only on small graphs (test_gpu_parity.py), so
at full size the checks are size-independent properties and a vendor fp32
reference on the same device:

* forward vs rocSPARSE SpMM (torch.sparse.mm on the densified masked input),
  per element |got - ref| / max(1, |ref|) <= 1e-4;
* backward via the exact adjoint identity <A . X^, G> = <X^_s, dXs> (both
  sides summed in fp64), every backward algorithm agreeing within 1e-4, and
  bit-exact linearity of the deterministic LOCAL path (dXs(2G) == 2 dXs(G));
* config 1 (Flickr h=64 k=16, the reference's own CPU case) against the fp64
  oracle at full size.
"""
import numpy as np
import pytest
import torch

import spgemm_new_amd as S
from spgemm_new_amd import _lib
from spgemm_new_amd.graphs import CONFIGS, synthetic_csr_gpu

pytestmark = pytest.mark.gpu
TOL = 1e-4


def _rel(a, b):
    return float(((a - b).abs() / b.abs().clamp_min(1)).max())


@pytest.mark.parametrize("graph,k", [("reddit", 32), ("products", 8), ("products", 64)])
def test_full_size_properties(dev, graph, k):
    V, E = CONFIGS[graph]
    h = 256
    indptr, indices = synthetic_csr_gpu(V, E, device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(11)
    values = torch.rand(indices.numel(), generator=gen, device=dev)
    X = torch.rand((V, h), generator=gen, device=dev)
    Gr = torch.rand((V, h), generator=gen, device=dev)
    data, sel = S.topk_cbsr(X, k)
    g = S.MaxKGraph(indptr, indices, values)
    y = g.forward(data, sel, h)
    # forward vs the vendor SpMM
    a = torch.sparse_csr_tensor(indptr.long(), indices.long(), values, size=(V, V))
    xm = torch.zeros_like(X).scatter_(1, sel.long(), data)
    ref = torch.sparse.mm(a, xm)
    assert _rel(y, ref) <= TOL
    del a, ref
    # backward: adjoint identity, algorithms agree
    algos = [_lib.MAXK_BWD_STAGED, _lib.MAXK_BWD_ATOMIC]
    if g.local_plan(k) is not None:   # slow on products (78 source bands) but must be right
        algos.append(_lib.MAXK_BWD_LOCAL)
    outs = {a_: g.backward(Gr, sel, algo=a_) for a_ in algos}
    lhs = float((y.double() * Gr.double()).sum())
    for a_, dx in outs.items():
        rhs = float((data.double() * dx.double()).sum())
        assert abs(lhs - rhs) / abs(lhs) <= 1e-6, (a_, lhs, rhs)
        assert _rel(dx, outs[_lib.MAXK_BWD_STAGED]) <= TOL, a_
    if _lib.MAXK_BWD_LOCAL in outs:
        dx2 = g.backward(2 * Gr, sel, algo=_lib.MAXK_BWD_LOCAL)
        assert torch.equal(dx2, 2 * outs[_lib.MAXK_BWD_LOCAL])


def test_flickr_config1_full(dev, oracle):
    """BASELINE config 1 shape (Flickr + self-loops, h=64, k=16) against the
    fp64 oracle at full size."""
    V, E = CONFIGS["flickr"]
    h, k = 64, 16
    indptr, indices = synthetic_csr_gpu(V, E, device=dev, self_loops=True)
    gen = torch.Generator(device=dev)
    gen.manual_seed(4)
    values = torch.ones(indices.numel(), device=dev)
    X = torch.rand((V, h), generator=gen, device=dev)
    Gr = torch.rand((V, h), generator=gen, device=dev)
    data, sel = S.topk_cbsr(X, k)
    g = S.MaxKGraph(indptr, indices, values)
    y = g.forward(data, sel, h)
    dx = g.backward(Gr, sel)
    ip, ix, vv = indptr.cpu().numpy(), indices.cpu().numpy(), values.cpu().numpy()
    dn, sn = data.cpu().numpy(), sel.cpu().numpy()
    assert oracle.parity_error(y.cpu().numpy(), oracle.np_forward(ip, ix, vv, dn, sn, h)) <= TOL
    assert oracle.parity_error(dx.cpu().numpy(),
                               oracle.np_backward(ip, ix, vv, Gr.cpu().numpy(), sn)) <= TOL
