// spmm_bindings.cpp -- the compiled `spmm_kernels` extension module: the
// class-based surface of the reference's kernels/spmm_bindings.cpp (module
// definition :209-262) on the MI355X C ABI (include/maxk_spgemm.h).
//
// Same module name, classes (SpmmMaxK, SpmmMaxKBackward), methods, argument
// names / defaults and free functions (prepare_cbsr_format, topk_nonlinearity),
// so `import spmm_kernels` (spgemm_new_amd/lib on sys.path) works for the
// reference's callers unchanged.  Differences, deliberate:
//  * set_sparse_params takes effect (the selector and k are the ones used);
//  * the schedule is derived from indptr on the device (merge-path panels), no
//    .warp4 file; the backward is the deterministic STAGED algorithm (CSC plan
//    built once per object) -- the measured per-shape choice lives in the
//    Python API (spgemm_new_amd.MaxKGraph);
//  * launches go to the current HIP stream.
// run_kernel keeps SPMM_BASE::timing_body's protocol (kernels/spmm_base.h:48-77):
// untimed = one launch + device synchronise, returns 0; timed = 4 warm-up + 4
// timed launches each closed by a synchronise, returns the mean in seconds.
// Host code only: all compute is in libmaxk_spgemm.so.
#include <torch/extension.h>

#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <string>

#include "../../include/maxk_spgemm.h"

namespace {

void *cur_stream() { return (void *)c10::hip::getCurrentHIPStream().stream(); }

void check_rc(int rc, const char *what)
{
    TORCH_CHECK(rc == MAXK_OK, what, " failed: ",
                rc < 0 ? "invalid argument (MAXK_E " + std::to_string(rc) + ")"
                       : std::string(hipGetErrorString((hipError_t)rc)));
}

void check_dev(const torch::Tensor &t, const char *name)
{
    TORCH_CHECK(t.is_cuda(), name, " must be a CUDA tensor");
    TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

torch::Tensor workspace(const torch::Tensor &like, size_t bytes)
{
    return torch::empty({(int64_t)std::max<size_t>(bytes, 1)},
                        like.options().dtype(torch::kUInt8));
}

// the graph part both classes share: CSR, panel schedule
struct Csr {
    torch::Tensor indptr, indices, values, sched;
    int64_t P = 0;
    int V = 0;
    int64_t E = 0;

    Csr(torch::Tensor ip, torch::Tensor ix, torch::Tensor vv)
    {
        check_dev(ip, "indptr");
        check_dev(ix, "indices");
        check_dev(vv, "values");
        TORCH_CHECK(ip.dtype() == torch::kInt32, "indptr must be int32");
        TORCH_CHECK(ix.dtype() == torch::kInt32, "indices must be int32");
        TORCH_CHECK(vv.dtype() == torch::kFloat32, "values must be float32");
        TORCH_CHECK(ip.dim() == 1 && ip.numel() >= 1, "indptr must be 1-D");
        TORCH_CHECK(ix.numel() == vv.numel(), "indices and values must have the same length");
        indptr = ip;
        indices = ix.numel() ? ix : torch::zeros({1}, ix.options());
        values = vv.numel() ? vv : torch::zeros({1}, vv.options());
        V = (int)(ip.numel() - 1);
        E = ix.numel();
        check_rc(maxk_schedule_num_panels(V, E, MAXK_DEFAULT_PANEL_COST, MAXK_DEFAULT_ROW_COST, &P),
                 "maxk_schedule_num_panels");
        sched = torch::empty({2 * (P + 1)}, ip.options());
        check_rc(maxk_schedule_build(ip.data_ptr<int32_t>(), V, MAXK_DEFAULT_PANEL_COST,
                                     MAXK_DEFAULT_ROW_COST, sched.data_ptr<int32_t>(), P,
                                     cur_stream()),
                 "maxk_schedule_build");
    }
};

torch::Tensor selector_u8(const torch::Tensor &s)
{
    check_dev(s, "sparse_selector");
    if (s.dtype() == torch::kUInt8) return s;
    TORCH_CHECK(s.dtype() == torch::kInt32 || s.dtype() == torch::kInt64,
                "sparse_selector must be int32");
    return s.to(torch::kUInt8).contiguous();
}

class SpmmBase {
  public:
    SpmmBase(const std::string &graph_name, torch::Tensor indptr, torch::Tensor indices,
             torch::Tensor values, torch::Tensor input_features, torch::Tensor output_features)
        : name_(graph_name), g_(indptr, indices, values)
    {
        update_input_output(input_features, output_features);
    }
    virtual ~SpmmBase() = default;

    void update_input_output(torch::Tensor input_features, torch::Tensor output_features)
    {
        check_dev(input_features, "input_features");
        check_dev(output_features, "output_features");
        TORCH_CHECK(input_features.dtype() == torch::kFloat32, "input_features must be float32");
        TORCH_CHECK(output_features.dtype() == torch::kFloat32, "output_features must be float32");
        vin_ = input_features;
        vout_ = output_features;
    }

    void set_sparse_params(torch::Tensor sparse_selector, int maxk)
    {
        TORCH_CHECK(maxk >= 1, "maxk must be positive");
        sel_ = selector_u8(sparse_selector);
        TORCH_CHECK(sel_.dim() == 2 && sel_.size(1) == maxk, "sparse_selector must be [V, maxk]");
        k_ = maxk;
    }

    std::string get_graph_name() const { return name_; }

    float run_kernel(bool timing, int dim)
    {
        TORCH_CHECK(sel_.defined(), "set_sparse_params() must be called before run_kernel()");
        if (!timing) {
            run(dim);
            TORCH_CHECK(hipDeviceSynchronize() == hipSuccess, "device synchronise failed");
            return 0.f;
        }
        for (int i = 0; i < 4; ++i) run(dim);
        TORCH_CHECK(hipDeviceSynchronize() == hipSuccess, "device synchronise failed");
        double total = 0;
        for (int i = 0; i < 4; ++i) {
            const auto t0 = std::chrono::steady_clock::now();
            run(dim);
            TORCH_CHECK(hipDeviceSynchronize() == hipSuccess, "device synchronise failed");
            total += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        }
        return (float)(total / 4);
    }

  protected:
    virtual void run(int dim) = 0;
    std::string name_;
    Csr g_;
    torch::Tensor vin_, vout_, sel_;
    int k_ = 0;
};

// forward SpGEMM (kernels/spmm_maxk.cu): vout[V, dim] = A . scatter(vin[V, k], sel)
class SpmmMaxK : public SpmmBase {
  public:
    using SpmmBase::SpmmBase;

  protected:
    void run(int dim) override
    {
        if (dim < 0) dim = (int)vout_.size(1);
        TORCH_CHECK(dim == vout_.size(1), "dim must equal output_features.size(1)");
        TORCH_CHECK(vout_.size(0) == g_.V && vin_.size(0) == g_.V && sel_.size(0) == g_.V,
                    "features must have one row per node");
        TORCH_CHECK(vin_.dim() == 2 && vin_.size(1) == k_, "input_features must be [V, maxk]");
        const size_t wb = maxk_forward_workspace_bytes(g_.P, dim);
        if (!ws_.defined() || (size_t)ws_.numel() < wb) ws_ = workspace(vin_, wb);
        check_rc(maxk_spgemm_forward(g_.sched.data_ptr<int32_t>(), g_.P, g_.indptr.data_ptr<int32_t>(),
                                     g_.indices.data_ptr<int32_t>(), g_.values.data_ptr<float>(),
                                     vin_.data_ptr<float>(), sel_.data_ptr<uint8_t>(), g_.V, dim, k_,
                                     vout_.data_ptr<float>(), ws_.data_ptr(), (size_t)ws_.numel(),
                                     cur_stream()),
                 "maxk_spgemm_forward");
    }

  private:
    torch::Tensor ws_;
};

// backward SSpMM (kernels/spmm_maxk_backward.cu): vout[V, k] from vin = G[V, dim]
class SpmmMaxKBackward : public SpmmBase {
  public:
    using SpmmBase::SpmmBase;

  protected:
    void run(int dim) override
    {
        if (dim < 0) dim = (int)vin_.size(1);
        TORCH_CHECK(dim == vin_.size(1), "dim must equal input_features.size(1)");
        TORCH_CHECK(vin_.size(0) == g_.V && vout_.size(0) == g_.V && sel_.size(0) == g_.V,
                    "features must have one row per node");
        TORCH_CHECK(vout_.dim() == 2 && vout_.size(1) == k_, "output_features must be [V, maxk]");
        plan();
        const size_t wb = maxk_backward_workspace_bytes(MAXK_BWD_STAGED, g_.E, k_, cp_);
        if (!ws_.defined() || (size_t)ws_.numel() < wb) ws_ = workspace(vin_, wb);
        check_rc(maxk_sspmm_backward(MAXK_BWD_STAGED, g_.sched.data_ptr<int32_t>(), g_.P,
                                     g_.indptr.data_ptr<int32_t>(), g_.indices.data_ptr<int32_t>(),
                                     g_.values.data_ptr<float>(), vin_.data_ptr<float>(),
                                     sel_.data_ptr<uint8_t>(), g_.V, g_.V, g_.E, dim, k_,
                                     vout_.data_ptr<float>(), csc_pos_.data_ptr<int32_t>(),
                                     csc_sched_.data_ptr<int32_t>(), cp_,
                                     csc_indptr_.data_ptr<int32_t>(), ws_.data_ptr(),
                                     (size_t)ws_.numel(), cur_stream()),
                 "maxk_sspmm_backward");
    }

  private:
    void plan()  // CSC transpose + its panel schedule, once
    {
        if (csc_pos_.defined()) return;
        auto opt = g_.indptr.options();
        csc_pos_ = torch::empty({std::max<int64_t>(g_.E, 1)}, opt);
        csc_indptr_ = torch::empty({(int64_t)g_.V + 1}, opt);
        auto ws = workspace(g_.indptr, maxk_csc_workspace_bytes(g_.E, g_.V));
        check_rc(maxk_csc_build(g_.indices.data_ptr<int32_t>(), g_.E, g_.V,
                                csc_indptr_.data_ptr<int32_t>(), csc_pos_.data_ptr<int32_t>(),
                                ws.data_ptr(), (size_t)ws.numel(), cur_stream()),
                 "maxk_csc_build");
        check_rc(maxk_schedule_num_panels(g_.V, g_.E, MAXK_DEFAULT_PANEL_COST,
                                          MAXK_DEFAULT_ROW_COST, &cp_),
                 "maxk_schedule_num_panels");
        csc_sched_ = torch::empty({2 * (cp_ + 1)}, opt);
        check_rc(maxk_schedule_build(csc_indptr_.data_ptr<int32_t>(), g_.V, MAXK_DEFAULT_PANEL_COST,
                                     MAXK_DEFAULT_ROW_COST, csc_sched_.data_ptr<int32_t>(), cp_,
                                     cur_stream()),
                 "maxk_schedule_build (CSC)");
    }
    torch::Tensor ws_, csc_pos_, csc_indptr_, csc_sched_;
    int64_t cp_ = 0;
};

// spmm_bindings.cpp:163-184: (values fp32[V, k], indices int32[V, k]) of the row-wise top-k,
// torch.topk's order (descending value)
std::tuple<torch::Tensor, torch::Tensor> prepare_cbsr_format(torch::Tensor features, int maxk)
{
    TORCH_CHECK(features.dim() == 2, "Features must be 2D");
    TORCH_CHECK(maxk > 0 && maxk <= features.size(1), "Invalid maxk value");
    if (features.is_cuda() && features.dtype() == torch::kFloat32 && features.size(1) <= 256) {
        auto x = features.contiguous();
        const int V = (int)x.size(0), h = (int)x.size(1);
        auto vals = torch::empty({V, maxk}, x.options());
        auto sel = torch::empty({V, maxk}, x.options().dtype(torch::kUInt8));
        check_rc(maxk_topk_cbsr(x.data_ptr<float>(), V, h, h, maxk, MAXK_TOPK_ORDER_VALUE,
                                vals.data_ptr<float>(), sel.data_ptr<uint8_t>(), nullptr,
                                cur_stream()),
                 "maxk_topk_cbsr");
        return {vals, sel.to(torch::kInt32)};
    }
    auto r = torch::topk(features, maxk, 1);   // wider rows: outside the kernels' range
    return {std::get<0>(r).contiguous(), std::get<1>(r).to(torch::kInt32).contiguous()};
}

// spmm_bindings.cpp:189-204: keep the k largest entries of each row, zero the rest
torch::Tensor topk_nonlinearity(torch::Tensor input, int k)
{
    TORCH_CHECK(input.dim() == 2, "Input must be 2D");
    TORCH_CHECK(k > 0 && k <= input.size(1), "Invalid k value");
    if (input.is_cuda() && input.dtype() == torch::kFloat32 && input.size(1) <= 256) {
        auto x = input.contiguous();
        const int V = (int)x.size(0), h = (int)x.size(1);
        auto vals = torch::empty({V, k}, x.options());
        auto sel = torch::empty({V, k}, x.options().dtype(torch::kUInt8));
        auto dense = torch::empty_like(x);
        check_rc(maxk_topk_cbsr(x.data_ptr<float>(), V, h, h, k, MAXK_TOPK_ORDER_COLUMN,
                                vals.data_ptr<float>(), sel.data_ptr<uint8_t>(),
                                dense.data_ptr<float>(), cur_stream()),
                 "maxk_topk_cbsr");
        return dense;
    }
    auto r = torch::topk(input, k, 1);
    return torch::zeros_like(input).scatter_(1, std::get<1>(r), std::get<0>(r));
}

}  // namespace

PYBIND11_MODULE(spmm_kernels, m)
{
    m.doc() = "MaxK-GNN SpMM kernels on MI355X (spmm_bindings.cpp surface, C ABI underneath)";
    pybind11::class_<SpmmMaxK>(m, "SpmmMaxK")
        .def(pybind11::init<const std::string &, torch::Tensor, torch::Tensor, torch::Tensor,
                            torch::Tensor, torch::Tensor>(),
             "Initialize SPMM_MAXK kernel", pybind11::arg("graph_name"), pybind11::arg("indptr"),
             pybind11::arg("indices"), pybind11::arg("values"), pybind11::arg("input_features"),
             pybind11::arg("output_features"))
        .def("update_input_output", &SpmmMaxK::update_input_output,
             "Update input and output tensor pointers", pybind11::arg("input_features"),
             pybind11::arg("output_features"))
        .def("set_sparse_params", &SpmmMaxK::set_sparse_params,
             "Set sparse selector and maxk parameters", pybind11::arg("sparse_selector"),
             pybind11::arg("maxk"))
        .def("run_kernel", &SpmmMaxK::run_kernel, "Execute the SPMM kernel",
             pybind11::arg("timing") = false, pybind11::arg("dim") = -1)
        .def("get_graph_name", &SpmmMaxK::get_graph_name, "Get the graph name");
    pybind11::class_<SpmmMaxKBackward>(m, "SpmmMaxKBackward")
        .def(pybind11::init<const std::string &, torch::Tensor, torch::Tensor, torch::Tensor,
                            torch::Tensor, torch::Tensor>(),
             "Initialize SPMM_MAXK_BACKWARD kernel", pybind11::arg("graph_name"),
             pybind11::arg("indptr"), pybind11::arg("indices"), pybind11::arg("values"),
             pybind11::arg("input_features"), pybind11::arg("output_features"))
        .def("update_input_output", &SpmmMaxKBackward::update_input_output,
             "Update input and output tensor pointers", pybind11::arg("input_features"),
             pybind11::arg("output_features"))
        .def("set_sparse_params", &SpmmMaxKBackward::set_sparse_params,
             "Set sparse selector and maxk parameters", pybind11::arg("sparse_selector"),
             pybind11::arg("maxk"))
        .def("run_kernel", &SpmmMaxKBackward::run_kernel, "Execute the backward SPMM kernel",
             pybind11::arg("timing") = false, pybind11::arg("dim") = -1)
        .def("get_graph_name", &SpmmMaxKBackward::get_graph_name, "Get the graph name");
    m.def("prepare_cbsr_format", &prepare_cbsr_format, "Convert dense features to CBSR format",
          pybind11::arg("features"), pybind11::arg("maxk"));
    m.def("topk_nonlinearity", &topk_nonlinearity, "Apply top-k nonlinearity function",
          pybind11::arg("input"), pybind11::arg("k"));
    m.attr("__version__") = "1.0.0";
}
