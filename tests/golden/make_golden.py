#!/usr/bin/env python3
"""Generate golden vectors by running the REFERENCE's own Python code.

Run in the build container (the reference is not present on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What is executed from the reference (read-only, /root/reference):
  * utils/models.py ``MaxK`` autograd Function (28-59): top-k mask forward and
    masked backward, composed with torch.sparse.mm on the COO adjacency the
    reference's CPU path builds (utils/models.py:281-287, sum form -- the
    kernel path's values, utils/models.py:227).
  * Not usable: SAGE.forward's non-kernel branch itself raises on torch 2.10
    (utils/models.py:287, ``adj.sum(dim=1, keepdim=True) + 1e-6`` adds a dense
    scalar to a sparse tensor: "add(sparse, dense) is not supported"), an
    ordinary error of the reference code, so no SAGE-level golden is made.

How it is loaded:
  * utils/models.py is loaded by file path; /root/reference is NOT put on
    sys.path, and ``spmm_kernels`` is pre-set to None in sys.modules, so the
    reference's prebuilt CUDA extension (spmm_kernels.so) is never searched
    for or loaded -- the module takes its documented ImportError fallback.
  * ``import dgl`` / ``import dgl.nn`` (module top, utils/models.py:6-7) are
    satisfied by empty placeholder modules: DGL is not installed and no DGL
    function is provided or called on this path.

Outputs (tests/golden/*.npz, numpy, no pickle):
  inputs.npz       indptr, indices, values, x, G  (V=300, h=128, seeded)
  kernel_k{K}.npz  from reference code: mask_bits = packbits(MaxK.apply(x,K) != 0),
                   Y = sparse.mm(adj, MaxK(x)), grad_x = d<Y, G>/dx through
                   MaxK.backward and sparse.mm
  inputs_h256.npz  the SURVEY.md §8(c) shape: V=2048, h=256, degrees 0/1/63/64/
                   65/129/257/700/1500 among Poisson-ish ones (> 13 blocks of
                   12 warp4 chunks), seeded
  kernel_h256_k{K}.npz  (K = 32, 64: the shapes of the TILE backward and the
                   north-star config) mask_bits, Y, and grad_x compacted to the
                   selected positions (grad_sel[r, j] = grad_x[r, j-th selected
                   column], row-major column order) -- grad_x is zero elsewhere
                   because MaxK.backward masks it (utils/models.py:52-59)
"""
from __future__ import annotations

import importlib.util
import os
import sys
import types

import numpy as np
import torch

REF = os.environ.get("MAXK_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)


def load_reference_models():
    sys.modules["spmm_kernels"] = None          # never load the prebuilt CUDA .so
    dgl = types.ModuleType("dgl")
    dgl.nn = types.ModuleType("dgl.nn")
    sys.modules.setdefault("dgl", dgl)
    sys.modules.setdefault("dgl.nn", dgl.nn)
    spec = importlib.util.spec_from_file_location("reference_utils_models",
                                                  os.path.join(REF, "utils", "models.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert mod.KERNELS_AVAILABLE is False
    return mod


def graph(v, seed):
    from spgemm_new_amd.graphs import small_csr
    return small_csr(v, seed=seed, extra_degrees=(0, 1, 63, 64, 65, 129, min(257, v - 1)))


def main():
    ref = load_reference_models()
    torch.manual_seed(123)
    rng = np.random.default_rng(123)

    # ---- raw aggregation goldens: V=300, h=128 ----------------------------
    v, h = 300, 128
    indptr, indices = graph(v, 11)
    values = rng.random(len(indices), dtype=np.float32)
    x = rng.random((v, h), dtype=np.float32)
    G = rng.random((v, h), dtype=np.float32)
    rows = np.repeat(np.arange(v), np.diff(indptr))
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.stack([rows, indices]).astype(np.int64)),
                                  torch.from_numpy(values), (v, v)).coalesce()
    np.savez(os.path.join(HERE, "inputs.npz"), indptr=indptr, indices=indices, values=values,
             x=x, G=G)
    for k in (8, 16, 32, 64):
        xt = torch.from_numpy(x).requires_grad_(True)
        xm = ref.MaxK.apply(xt, k)                       # reference MaxK (utils/models.py:28-59)
        y = torch.sparse.mm(adj, xm)                     # reference CPU aggregation op
        y.backward(torch.from_numpy(G))
        np.savez(os.path.join(HERE, f"kernel_k{k}.npz"),
                 mask_bits=np.packbits(xm.detach().numpy() != 0, axis=1),
                 Y=y.detach().numpy(), grad_x=xt.grad.numpy(), k=np.int32(k))

    # ---- SURVEY.md §8(c) shape: V=2048, h=256 (TILE / north-star k) --------
    rng = np.random.default_rng(256)
    v, h = 2048, 256
    from spgemm_new_amd.graphs import small_csr
    indptr, indices = small_csr(v, seed=29, extra_degrees=(0, 1, 63, 64, 65, 129, 257, 700, 1500))
    values = rng.random(len(indices), dtype=np.float32)
    x = rng.random((v, h), dtype=np.float32)
    G = rng.random((v, h), dtype=np.float32)
    rows = np.repeat(np.arange(v), np.diff(indptr))
    adj = torch.sparse_coo_tensor(torch.from_numpy(np.stack([rows, indices]).astype(np.int64)),
                                  torch.from_numpy(values), (v, v)).coalesce()
    np.savez_compressed(os.path.join(HERE, "inputs_h256.npz"), indptr=indptr, indices=indices,
                        values=values, x=x, G=G)
    for k in (32, 64):
        xt = torch.from_numpy(x).requires_grad_(True)
        xm = ref.MaxK.apply(xt, k)
        y = torch.sparse.mm(adj, xm)
        y.backward(torch.from_numpy(G))
        mask = xm.detach().numpy() != 0
        gx = xt.grad.numpy()
        assert np.all(gx[~mask] == 0) and np.all(mask.sum(1) == k)
        np.savez_compressed(os.path.join(HERE, f"kernel_h256_k{k}.npz"),
                            mask_bits=np.packbits(mask, axis=1), Y=y.detach().numpy(),
                            grad_sel=gx[mask].reshape(v, k), k=np.int32(k))
    print("golden vectors written to", HERE)


if __name__ == "__main__":
    main()
