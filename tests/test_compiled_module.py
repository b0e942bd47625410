"""The compiled `maxk_cuda_kernels` extension (csrc/maxk_bindings.cpp, the
pybind11 shim replacing the reference's cuda_kernel_bindings.cpp:429-490):
importable under the reference's module name, same function set as the
reference module definition, same results as the Python mirror and the oracle."""
import os
import sys

import numpy as np
import pytest
import torch

LIBDIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                      "spgemm_new_amd", "lib")
# cuda_kernel_bindings.cpp:429-490, in order
REFERENCE_NAMES = ["spmm_maxk_forward", "spmm_maxk_backward", "cuda_topk_maxk",
                   "cuda_topk_maxk_float", "prepare_cbsr_format_maxk", "load_warp4_metadata",
                   "generate_sparse_selector", "benchmark_spmm_maxk", "validate_spmm_maxk",
                   "cusparse_spmm", "CudaTimer"]


def _module():
    if LIBDIR not in sys.path:
        sys.path.insert(0, LIBDIR)
    import maxk_cuda_kernels
    assert os.path.dirname(os.path.abspath(maxk_cuda_kernels.__file__)) == LIBDIR
    return maxk_cuda_kernels


def test_compiled_module_exports_reference_names():
    m = _module()
    for n in REFERENCE_NAMES:
        assert hasattr(m, n), n
    assert m.spmm_maxk_forward.__doc__.startswith("spmm_maxk_forward(warp4_metadata")


@pytest.mark.gpu
@pytest.mark.parametrize("k", [16, 32])
def test_compiled_module_matches_oracle(dev, oracle, k):
    from spgemm_new_amd import maxk_cuda_kernels as py_mod
    from spgemm_new_amd.graphs import random_cbsr, small_csr
    from spgemm_new_amd.ops import warp4_build
    m = _module()
    indptr, indices = small_csr(2000, seed=8)
    v, h = len(indptr) - 1, 256
    values = np.random.default_rng(1).random(len(indices), dtype=np.float32)
    data, sel = random_cbsr(v, k, h, seed=4)
    grad = np.random.default_rng(2).random((v, h), dtype=np.float32)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    ip, ix, vv, d, s, g = (T(a) for a in (indptr, indices, values, data, sel, grad))
    w4 = warp4_build(ip)
    nw = w4.numel() // 4
    y = m.spmm_maxk_forward(w4, ix, vv, d, s, nw, k)
    dx = m.spmm_maxk_backward(w4, ix, vv, g, s, nw, k)
    torch.cuda.synchronize()
    assert oracle.parity_error(y.cpu().numpy(),
                               oracle.np_forward(indptr, indices, values, data, sel, h)) <= 1e-4
    assert oracle.parity_error(dx.cpu().numpy(),
                               oracle.np_backward(indptr, indices, values, grad, sel)) <= 1e-4
    y_py = py_mod.spmm_maxk_forward(w4, ix, vv, d, s, nw, k)
    assert (y - y_py).abs().max().item() <= 1e-4 * max(1.0, y_py.abs().max().item())
    # exact top-k, torch.topk's set and order.  torch.rand has 2^-24 granularity, so a
    # row of 256 may hold equal values, whose order torch.topk leaves open: the values
    # must match exactly, every index must point at its value, and the index SETS match
    gen = torch.Generator(device=dev)
    gen.manual_seed(11 + k)
    x = torch.rand((500, h), device=dev, generator=gen)
    vals, idx = m.cuda_topk_maxk_float(x, k)
    ref = torch.topk(x, k, dim=1)
    assert torch.equal(vals, ref.values)
    assert torch.equal(x.gather(1, idx.long()), vals)
    assert torch.equal(idx.long().sort(1).values, ref.indices.sort(1).values)
    assert isinstance(m.cuda_topk_maxk_float(x, k), tuple)
    # uint8 input keeps uint8 values, int32 indices (cuda_kernel_bindings.cpp:226-233)
    xu = (x * 255).round().to(torch.uint8)
    for mod in (m, py_mod):
        vu, iu = mod.cuda_topk_maxk_float(xu, k)
        assert vu.dtype == torch.uint8 and iu.dtype == torch.int32
        assert torch.equal(vu, torch.topk(xu.int(), k, dim=1).values.to(torch.uint8))
    t = m.CudaTimer()
    t.start()
    assert t.stop() >= 0.0
    assert len(m.benchmark_spmm_maxk(w4, ix, vv, d, s, nw, k, 2)) == 2
    assert m.validate_spmm_maxk(w4, ix, vv, d, s, y, nw, k)


@pytest.mark.gpu
def test_compiled_module_errors(dev):
    """TORCH_CHECK behaviour of the reference binding: RuntimeError with its messages."""
    m = _module()
    w4 = torch.zeros(4, dtype=torch.int32, device=dev)
    ix = torch.zeros(1, dtype=torch.int32, device=dev)
    vv = torch.zeros(1, device=dev)
    d = torch.zeros((2, 8), device=dev)
    s = torch.zeros((2, 8), dtype=torch.uint8, device=dev)
    with pytest.raises(RuntimeError, match="indices must be CUDA tensor"):
        m.spmm_maxk_forward(w4, ix.cpu(), vv, d, s, 1, 8)
    with pytest.raises(RuntimeError, match="sparse_selector must be uint8"):
        m.spmm_maxk_forward(w4, ix, vv, d, s.int(), 1, 8)
    with pytest.raises(RuntimeError, match="Invalid k value"):
        m.cuda_topk_maxk_float(d, 9)


# ------------------------------------------------ the compiled `spmm_kernels` module
# kernels/spmm_bindings.cpp:209-262
SPMM_CLASS_METHODS = ["update_input_output", "set_sparse_params", "run_kernel", "get_graph_name"]


def _spmm_module():
    if LIBDIR not in sys.path:
        sys.path.insert(0, LIBDIR)
    import spmm_kernels
    assert os.path.dirname(os.path.abspath(spmm_kernels.__file__)) == LIBDIR
    return spmm_kernels


def test_compiled_spmm_kernels_exports_reference_surface():
    m = _spmm_module()
    for cls in ("SpmmMaxK", "SpmmMaxKBackward"):
        for meth in SPMM_CLASS_METHODS:
            assert hasattr(getattr(m, cls), meth), (cls, meth)
    assert callable(m.prepare_cbsr_format) and callable(m.topk_nonlinearity)


@pytest.mark.gpu
@pytest.mark.parametrize("k", [8, 32])
def test_compiled_spmm_kernels_matches_oracle(dev, oracle, k):
    from spgemm_new_amd.graphs import random_cbsr, small_csr
    m = _spmm_module()
    indptr, indices = small_csr(2000, seed=9)
    v, h = len(indptr) - 1, 256
    values = np.random.default_rng(1).random(len(indices), dtype=np.float32)
    data, sel = random_cbsr(v, k, h, seed=5)
    grad = np.random.default_rng(2).random((v, h), dtype=np.float32)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    ip, ix, vv, d, g = (T(a) for a in (indptr, indices, values, data, grad))
    s32 = T(sel.astype(np.int32))             # the reference passes int32 selectors
    y = torch.full((v, h), float("nan"), device=dev)
    fwd = m.SpmmMaxK("g", ip, ix, vv, d, y)
    fwd.set_sparse_params(s32, k)
    assert fwd.run_kernel(False, h) == 0.0 and fwd.get_graph_name() == "g"
    assert oracle.parity_error(y.cpu().numpy(),
                               oracle.np_forward(indptr, indices, values, data, sel, h)) <= 1e-4
    assert fwd.run_kernel(True) > 0.0           # spmm_base.h's 4 + 4 protocol, seconds
    dx = torch.full((v, k), float("nan"), device=dev)
    bwd = m.SpmmMaxKBackward("g", ip, ix, vv, g, dx)
    bwd.set_sparse_params(s32, k)
    bwd.run_kernel()
    assert oracle.parity_error(dx.cpu().numpy(),
                               oracle.np_backward(indptr, indices, values, grad, sel)) <= 1e-4
    x = torch.rand((v, h), device=dev)
    vals, idx = m.prepare_cbsr_format(x, k)
    ref_v, ref_i = torch.topk(x, k, dim=1)
    assert idx.dtype == torch.int32 and torch.equal(vals, ref_v)
    assert torch.equal(torch.sort(idx, 1)[0], torch.sort(ref_i.int(), 1)[0])
    dense = m.topk_nonlinearity(x, k)
    assert torch.equal(dense, torch.zeros_like(x).scatter_(1, ref_i, ref_v))
    with pytest.raises(RuntimeError):
        m.SpmmMaxK("g", ip, ix, vv, d, y).run_kernel()   # no set_sparse_params yet
