// maxk_bindings.cpp -- the compiled `maxk_cuda_kernels` extension module:
// the pybind11 shim that replaces the reference's cuda_kernel_bindings.cpp
// (module definition :429-490), on the MI355X C ABI (include/maxk_spgemm.h).
//
// Same module name, function names, argument names / defaults and
// TORCH_CHECK error messages as the reference, so `import maxk_cuda_kernels`
// (spgemm_new_amd/lib on sys.path) works for its callers unchanged
// (direct_kernel_interface.py, utils/models.py).  Differences, deliberate:
//  * launches go to the current HIP stream and stay asynchronous (the
//    reference used the legacy default stream, cuda_kernel_wrappers.cu:46,66);
//  * every k works and the top-k is exact (the reference's uint8-quantised
//    float top-k, :203-238, is replaced by the library's exact CBSR producer);
//  * cusparse_spmm is torch.sparse.mm on the device (rocSPARSE).
// This file is host code only: all compute is in libmaxk_spgemm.so.
#include <torch/extension.h>

#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <fstream>
#include <string>
#include <vector>

#include "../../include/maxk_spgemm.h"

namespace {

constexpr int kFullDim = 256;  // cuda_kernel_bindings.cpp:70

void *cur_stream() { return (void *)c10::hip::getCurrentHIPStream().stream(); }

void check_rc(int rc, const char *what)
{
    TORCH_CHECK(rc == MAXK_OK, what, " failed: ",
                rc < 0 ? "invalid argument (MAXK_E " + std::to_string(rc) + ")"
                       : std::string(hipGetErrorString((hipError_t)rc)));
}

void check_cuda(const torch::Tensor &t, const char *name)
{
    TORCH_CHECK(t.is_cuda(), name, " must be CUDA tensor");
    TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

torch::Tensor spmm_maxk_forward(torch::Tensor warp4_metadata, torch::Tensor indices,
                                torch::Tensor values, torch::Tensor input_data,
                                torch::Tensor sparse_selector, int num_warps, int dim_sparse)
{
    check_cuda(warp4_metadata, "warp4_metadata");
    check_cuda(indices, "indices");
    check_cuda(values, "values");
    check_cuda(input_data, "input_data");
    check_cuda(sparse_selector, "sparse_selector");
    TORCH_CHECK(warp4_metadata.dtype() == torch::kInt32, "warp4_metadata must be int32");
    TORCH_CHECK(indices.dtype() == torch::kInt32, "indices must be int32");
    TORCH_CHECK(values.dtype() == torch::kFloat32, "values must be float32");
    TORCH_CHECK(input_data.dtype() == torch::kFloat32, "input_data must be float32");
    TORCH_CHECK(sparse_selector.dtype() == torch::kUInt8, "sparse_selector must be uint8");
    const int num_v = (int)input_data.size(0);
    auto output = torch::zeros({num_v, kFullDim}, input_data.options());
    const int nw = std::min<int64_t>(num_warps, warp4_metadata.numel() / 4);
    check_rc(maxk_spmm_forward_warp4(warp4_metadata.data_ptr<int32_t>(), indices.data_ptr<int32_t>(),
                                     values.data_ptr<float>(), input_data.data_ptr<float>(),
                                     sparse_selector.data_ptr<uint8_t>(), output.data_ptr<float>(),
                                     num_v, (int)indices.numel(), kFullDim, dim_sparse, nw,
                                     cur_stream()),
             "CUDA kernel");
    return output;
}

torch::Tensor spmm_maxk_backward(torch::Tensor warp4_metadata, torch::Tensor indices,
                                 torch::Tensor values, torch::Tensor grad_output,
                                 torch::Tensor sparse_selector, int num_warps, int dim_sparse)
{
    check_cuda(warp4_metadata, "warp4_metadata");
    check_cuda(indices, "indices");
    check_cuda(values, "values");
    check_cuda(grad_output, "grad_output");
    check_cuda(sparse_selector, "sparse_selector");
    TORCH_CHECK(warp4_metadata.dtype() == torch::kInt32, "warp4_metadata must be int32");
    TORCH_CHECK(indices.dtype() == torch::kInt32, "indices must be int32");
    TORCH_CHECK(values.dtype() == torch::kFloat32, "values must be float32");
    TORCH_CHECK(grad_output.dtype() == torch::kFloat32, "grad_output must be float32");
    TORCH_CHECK(sparse_selector.dtype() == torch::kUInt8, "sparse_selector must be uint8");
    const int num_v = (int)grad_output.size(0), feat_in = (int)grad_output.size(1);
    auto grad_input = torch::zeros({num_v, dim_sparse}, grad_output.options());
    const int nw = std::min<int64_t>(num_warps, warp4_metadata.numel() / 4);
    check_rc(maxk_spmm_backward_warp4(warp4_metadata.data_ptr<int32_t>(), indices.data_ptr<int32_t>(),
                                      values.data_ptr<float>(), grad_output.data_ptr<float>(),
                                      sparse_selector.data_ptr<uint8_t>(),
                                      grad_input.data_ptr<float>(), num_v, (int)indices.numel(),
                                      feat_in, dim_sparse, nw, cur_stream()),
             "CUDA kernel");
    return grad_input;
}

std::tuple<torch::Tensor, torch::Tensor> cuda_topk_maxk(torch::Tensor input, int k)
{
    TORCH_CHECK(input.is_cuda(), "Input must be on CUDA");
    TORCH_CHECK(input.dim() == 2, "Input must be 2D tensor");
    TORCH_CHECK(input.dtype() == torch::kUInt8, "Input must be uint8 tensor");
    TORCH_CHECK(k > 0 && k <= input.size(1), "Invalid k value");
    auto r = torch::topk(input.to(torch::kInt32), k, 1);
    return std::make_tuple(std::get<0>(r).to(torch::kUInt8), std::get<1>(r).to(torch::kUInt8));
}

// cuda_kernel_bindings.cpp:203-238's contract: float32 in -> (float32 values,
// int32 indices); uint8 in -> (uint8 values, int32 indices) through the uint8
// path.  The float32 top-k is exact (the library's CBSR producer in torch.topk's
// order) instead of the reference's uint8-quantised one.
std::tuple<torch::Tensor, torch::Tensor> cuda_topk_maxk_float(torch::Tensor input, int k)
{
    TORCH_CHECK(input.is_cuda(), "Input must be on CUDA");
    TORCH_CHECK(input.dim() == 2, "Input must be 2D tensor");
    TORCH_CHECK(k > 0 && k <= input.size(1), "Invalid k value");
    if (input.dtype() == torch::kUInt8) {
        auto r = cuda_topk_maxk(input, k);
        return std::make_tuple(std::get<0>(r), std::get<1>(r).to(torch::kInt32));
    }
    TORCH_CHECK(input.dtype() == torch::kFloat32, "Input must be float32 or uint8");
    auto x = input.contiguous();
    const int V = (int)x.size(0), h = (int)x.size(1);
    TORCH_CHECK(h <= kFullDim, "Input rows must have at most 256 columns");
    auto vals = torch::empty({V, k}, x.options());
    auto sel = torch::empty({V, k}, x.options().dtype(torch::kUInt8));
    check_rc(maxk_topk_cbsr(x.data_ptr<float>(), V, h, h, k, MAXK_TOPK_ORDER_VALUE,
                            vals.data_ptr<float>(), sel.data_ptr<uint8_t>(), nullptr, cur_stream()),
             "maxk_topk_cbsr");
    return std::make_tuple(vals, sel.to(torch::kInt32));
}

std::tuple<torch::Tensor, torch::Tensor> prepare_cbsr_format_maxk(torch::Tensor features, int maxk)
{
    return cuda_topk_maxk_float(features, maxk);
}

// cuda_kernel_bindings.cpp:287-317: kernels/w{nw}_nz{nz}_warp_4/<graph>.warp4
torch::Tensor load_warp4_metadata(const std::string &graph_name, int num_warps, int warp_max_nz)
{
    const std::string path = "kernels/w" + std::to_string(num_warps) + "_nz" +
                             std::to_string(warp_max_nz) + "_warp_4/" + graph_name + ".warp4";
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    TORCH_CHECK(f.good(), "Cannot open warp4 file: ", path);
    const std::streamsize bytes = f.tellg();
    f.seekg(0);
    auto host = torch::empty({(int64_t)(bytes / 4)}, torch::kInt32);
    f.read(reinterpret_cast<char *>(host.data_ptr<int32_t>()), (bytes / 4) * 4);
    return host.to(torch::kCUDA);
}

torch::Tensor generate_sparse_selector(int num_v, int dim_origin, int dim_sparse)
{
    TORCH_CHECK(dim_sparse > 0 && dim_sparse <= dim_origin && dim_origin <= 256,
                "need 0 < dim_sparse <= dim_origin <= 256");
    auto gen = at::make_generator<at::CPUGeneratorImpl>(123);
    auto r = torch::rand({num_v, dim_origin}, gen, torch::kFloat32);
    auto s = torch::argsort(r, (int64_t)1, false).narrow(1, 0, dim_sparse).to(torch::kUInt8).contiguous();
    return s.to(torch::kCUDA);
}

torch::Tensor cusparse_spmm(torch::Tensor indptr, torch::Tensor indices, torch::Tensor values,
                            torch::Tensor input_features, bool timing)
{
    (void)timing;
    const int64_t n = indptr.numel() - 1;
    auto a = torch::sparse_csr_tensor(indptr.to(torch::kInt64), indices.to(torch::kInt64), values,
                                      {n, n}, values.options().layout(torch::kSparseCsr));
    return torch::mm(a, input_features);
}

class CudaTimer {  // cuda_kernel_bindings.cpp:343-369, events on the current stream
  public:
    CudaTimer()
    {
        TORCH_CHECK(hipEventCreate(&s_) == hipSuccess && hipEventCreate(&e_) == hipSuccess,
                    "hipEventCreate failed");
    }
    ~CudaTimer()
    {
        (void)hipEventDestroy(s_);
        (void)hipEventDestroy(e_);
    }
    void start() { TORCH_CHECK(hipEventRecord(s_, (hipStream_t)cur_stream()) == hipSuccess); }
    float stop()
    {
        float ms = 0.f;
        TORCH_CHECK(hipEventRecord(e_, (hipStream_t)cur_stream()) == hipSuccess &&
                        hipEventSynchronize(e_) == hipSuccess &&
                        hipEventElapsedTime(&ms, s_, e_) == hipSuccess,
                    "CudaTimer: event failed");
        return ms;
    }

  private:
    hipEvent_t s_ = nullptr, e_ = nullptr;
};

std::vector<float> benchmark_spmm_maxk(torch::Tensor warp4_metadata, torch::Tensor indices,
                                       torch::Tensor values, torch::Tensor input_data,
                                       torch::Tensor sparse_selector, int num_warps,
                                       int dim_sparse, int num_runs)
{
    for (int i = 0; i < num_runs; ++i)
        spmm_maxk_forward(warp4_metadata, indices, values, input_data, sparse_selector, num_warps,
                          dim_sparse);
    TORCH_CHECK(hipDeviceSynchronize() == hipSuccess, "hipDeviceSynchronize failed");
    std::vector<float> times;
    CudaTimer t;
    for (int i = 0; i < num_runs; ++i) {
        t.start();
        spmm_maxk_forward(warp4_metadata, indices, values, input_data, sparse_selector, num_warps,
                          dim_sparse);
        times.push_back(t.stop());
    }
    return times;
}

bool validate_spmm_maxk(torch::Tensor warp4_metadata, torch::Tensor indices, torch::Tensor values,
                        torch::Tensor input_data, torch::Tensor sparse_selector,
                        torch::Tensor reference_output, int num_warps, int dim_sparse,
                        float tolerance)
{
    auto out = spmm_maxk_forward(warp4_metadata, indices, values, input_data, sparse_selector,
                                 num_warps, dim_sparse);
    auto diff = (out - reference_output).abs();
    const float max_diff = diff.max().item<float>(), avg_diff = diff.mean().item<float>();
    std::printf("Validation - Max diff: %g, Avg diff: %g\n", max_diff, avg_diff);
    return avg_diff < tolerance;
}

}  // namespace

PYBIND11_MODULE(maxk_cuda_kernels, m)
{
    namespace py = pybind11;
    m.doc() = "MI355X MaxK-GNN SpGEMM / SSpMM bindings (drop-in for cuda_kernel_bindings.cpp)";
    m.def("spmm_maxk_forward", &spmm_maxk_forward, "MaxK-GNN forward SPMM kernel",
          py::arg("warp4_metadata"), py::arg("indices"), py::arg("values"), py::arg("input_data"),
          py::arg("sparse_selector"), py::arg("num_warps"), py::arg("dim_sparse"));
    m.def("spmm_maxk_backward", &spmm_maxk_backward, "MaxK-GNN backward SPMM kernel",
          py::arg("warp4_metadata"), py::arg("indices"), py::arg("values"), py::arg("grad_output"),
          py::arg("sparse_selector"), py::arg("num_warps"), py::arg("dim_sparse"));
    m.def("cuda_topk_maxk", &cuda_topk_maxk, "TopK for uint8 tensors", py::arg("input"),
          py::arg("k"));
    m.def("cuda_topk_maxk_float", &cuda_topk_maxk_float, "Exact TopK for float tensors",
          py::arg("input"), py::arg("k"));
    m.def("prepare_cbsr_format_maxk", &prepare_cbsr_format_maxk, "CBSR format via the MaxK TopK",
          py::arg("features"), py::arg("maxk"));
    m.def("load_warp4_metadata", &load_warp4_metadata, "Load warp4 metadata from file",
          py::arg("graph_name"), py::arg("num_warps") = 12, py::arg("warp_max_nz") = 64);
    m.def("generate_sparse_selector", &generate_sparse_selector, "Random sparse selector",
          py::arg("num_v"), py::arg("dim_origin"), py::arg("dim_sparse"));
    m.def("benchmark_spmm_maxk", &benchmark_spmm_maxk, "Benchmark the forward kernel",
          py::arg("warp4_metadata"), py::arg("indices"), py::arg("values"), py::arg("input_data"),
          py::arg("sparse_selector"), py::arg("num_warps"), py::arg("dim_sparse"),
          py::arg("num_runs") = 4);
    m.def("validate_spmm_maxk", &validate_spmm_maxk, "Validate the forward against a reference",
          py::arg("warp4_metadata"), py::arg("indices"), py::arg("values"), py::arg("input_data"),
          py::arg("sparse_selector"), py::arg("reference_output"), py::arg("num_warps"),
          py::arg("dim_sparse"), py::arg("tolerance") = 0.001f);
    m.def("cusparse_spmm", &cusparse_spmm, "Vendor (rocSPARSE) dense SpMM reference",
          py::arg("indptr"), py::arg("indices"), py::arg("values"), py::arg("input_features"),
          py::arg("timing") = false);
    py::class_<CudaTimer>(m, "CudaTimer")
        .def(py::init<>())
        .def("start", &CudaTimer::start)
        .def("stop", &CudaTimer::stop);
}
