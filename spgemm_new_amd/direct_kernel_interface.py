"""Mirror of the reference's benchmarking facade (direct_kernel_interface.py:24-447).

``DirectMaxKKernels`` keeps the reference's method names, arguments and return
values; it drives this package's functional API (``maxk_cuda_kernels``), so
every call runs the MI355X HIP kernels.  ``GraphDataLoader`` replaces the
module the reference imports but does not ship (direct_kernel_interface.py:12);
it reads the raw int32 ``<g>.indptr`` / ``<g>.indices`` files of
kernels/data.h:8-24 from a directory.

Deliberate differences: no emoji progress prints; a missing warp4 file is not
fatal -- ``load_warp4_metadata(..., indptr=...)`` builds the schedule on the
device (generate_meta.py semantics) instead.
"""
from __future__ import annotations

import glob
import os
import time

import numpy as np
import torch

from . import maxk_cuda_kernels as K
from .graphs import read_csr

DIRECT_KERNELS_AVAILABLE = True


class GraphDataLoader:
    def __init__(self, graph_dir: str = "graphs"):
        self.graph_dir = graph_dir

    def get_available_graphs(self):
        return sorted(os.path.basename(p)[: -len(".indptr")]
                      for p in glob.glob(os.path.join(self.graph_dir, "*.indptr")))

    def load_graph(self, name: str, seed: int = 123):
        indptr, indices = read_csr(os.path.join(self.graph_dir, name))
        rng = np.random.default_rng(seed)
        return {"indptr": torch.from_numpy(indptr), "indices": torch.from_numpy(indices),
                "values": torch.from_numpy(rng.random(len(indices), dtype=np.float32)),
                "v_num": len(indptr) - 1, "e_num": len(indices)}

    @staticmethod
    def to_cuda_tensors(graph_data, device="cuda"):
        out = dict(graph_data)
        for k in ("indptr", "indices", "values"):
            out[k] = graph_data[k].to(device).contiguous()
        return out


class DirectMaxKKernels:
    """direct_kernel_interface.py:24-382."""

    def __init__(self, graph_name: str = ""):
        self.graph_name = graph_name
        self.warp4_metadata = None
        self.num_warps = 0

    def load_warp4_metadata(self, graph_name=None, num_warps=12, warp_max_nz=64, indptr=None):
        graph_name = self.graph_name if graph_name is None else graph_name
        try:
            self.warp4_metadata = K.load_warp4_metadata(graph_name, num_warps, warp_max_nz)
        except RuntimeError:
            if indptr is None:
                return False
            self.warp4_metadata = K.build_warp4_metadata(indptr.cuda().int(), warp_max_nz)
        self.num_warps = self.warp4_metadata.numel() // 4
        return True

    def generate_maxk_sparse_data(self, input_features, dim_k, use_cuda_topk=True):
        """(data fp32[V,k], selector uint8[V,k]) by exact top-k (:58-85)."""
        vals, idx = K.cuda_topk_maxk_float(input_features, dim_k)
        return vals, idx.to(torch.uint8)

    def _require(self):
        if self.warp4_metadata is None:
            raise RuntimeError("Warp4 metadata not loaded. Call load_warp4_metadata() first")

    def run_forward_kernel(self, graph_data, input_features, dim_k, timing=True,
                           use_cuda_topk=True):
        """(:87-153) -> (output fp32[V,256], mean ms or 0.0)."""
        self._require()
        data, sel = self.generate_maxk_sparse_data(input_features, dim_k, use_cuda_topk)
        args = (self.warp4_metadata, graph_data["indices"], graph_data["values"], data, sel,
                self.num_warps, dim_k)
        t = float(np.mean(K.benchmark_spmm_maxk(*args, num_runs=4))) if timing else 0.0
        return K.spmm_maxk_forward(*args), t

    def run_backward_kernel(self, graph_data, grad_output, dim_k, timing=True,
                            use_cuda_topk=True, sparse_selector=None):
        """(:155-213).  Like the reference, the selector defaults to top-k of
        grad_output (benchmark semantics); pass the forward's
        ``sparse_selector`` for training semantics."""
        self._require()
        if sparse_selector is None:
            _, sparse_selector = self.generate_maxk_sparse_data(grad_output, dim_k, use_cuda_topk)
        args = (self.warp4_metadata, graph_data["indices"], graph_data["values"], grad_output,
                sparse_selector, self.num_warps, dim_k)
        if not timing:
            return K.spmm_maxk_backward(*args), 0.0
        timer = K.CudaTimer()
        times = []
        for i in range(8):
            timer.start()
            out = K.spmm_maxk_backward(*args)
            ms = timer.stop()
            if i >= 4:
                times.append(ms)
        return out, float(np.mean(times))

    def validate_against_cusparse(self, graph_data, input_features, dim_k, tolerance=0.001,
                                  use_cuda_topk=True):
        """(:215-298): compare against the vendor sparse library on the same top-k
        input, at the positions where the input was non-zero."""
        self._require()
        data, sel = self.generate_maxk_sparse_data(input_features, dim_k, use_cuda_topk)
        sparse_input = torch.zeros_like(input_features)
        sparse_input.scatter_(1, sel.long(), data)
        out = K.spmm_maxk_forward(self.warp4_metadata, graph_data["indices"],
                                  graph_data["values"], data, sel, self.num_warps, dim_k)
        ref = K.cusparse_spmm(graph_data["indptr"], graph_data["indices"], graph_data["values"],
                              sparse_input)
        if out.shape != ref.shape:
            return False
        diff = (out - ref).abs()[sparse_input != 0]
        max_error = float(diff.max()) if diff.numel() else 0.0
        return max_error < tolerance

    def benchmark_all_k_values(self, graph_data, dim_origin=256, k_values=(16, 32, 64),
                               num_runs=4, use_cuda_topk=True):
        """(:300-382) -> {k: {'forward_time': ms, 'backward_time': ms}}."""
        self._require()
        v_num = graph_data["indptr"].size(0) - 1
        torch.manual_seed(123)
        x = torch.rand(v_num, dim_origin, device="cuda", dtype=torch.float32)
        results = {}
        for k in k_values:
            if k > 64:
                continue
            _, tf = self.run_forward_kernel(graph_data, x, k, True, use_cuda_topk)
            g = torch.rand_like(x)
            _, tb = self.run_backward_kernel(graph_data, g, k, True, use_cuda_topk)
            results[k] = {"forward_time": tf, "backward_time": tb}
            print(f"1/1 {self.graph_name} {dim_origin} {k} maxk {tf:.3f}")
            print(f"1/1 {self.graph_name} {dim_origin} {k} maxk_backward {tb:.3f}")
        return results


def test_direct_kernels(graph_dir="graphs"):
    """(:384-447): validate + benchmark every graph found in graph_dir."""
    loader = GraphDataLoader(graph_dir)
    ok = True
    for name in loader.get_available_graphs():
        gd = loader.to_cuda_tensors(loader.load_graph(name))
        kern = DirectMaxKKernels(name)
        kern.load_warp4_metadata(indptr=gd["indptr"])
        x = torch.rand(gd["v_num"], 256, device="cuda")
        valid = kern.validate_against_cusparse(gd, x, dim_k=32, use_cuda_topk=False)
        ok &= valid
        if valid:
            t0 = time.time()
            kern.benchmark_all_k_values(gd, 256, (16, 32), num_runs=2)
            print(f"{name}: benchmarked in {time.time() - t0:.1f}s")
    return ok
