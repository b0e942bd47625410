// maxk_kernel_test -- the reference's kernel benchmark executable
// (kernels/main.cu:50-220, timing protocol kernels/spmm_base.h:48-77) on the
// MI355X library, through the C ABI only (include/maxk_spgemm.h; no torch).
//
//   maxk_kernel_test [graph] [--dir DIR] [--check]
//
// With a graph name it reads DIR/<graph>.indptr and DIR/<graph>.indices
// (raw int32, kernels/data.h:8-24); without one it runs every *.indptr in DIR
// (default ../graphs/, as main.cu).  Inputs follow main.cu:74-146: minstd_rand0
// seeded 123 drawing U(0,1) floats for the edge values, the two bulk buffers,
// then per k in {16, 32, 64} a std::sample of k columns and k values per row;
// the densified input doubles as the backward's upstream gradient (main.cu:103).
// Output lines match main.cu: "<i>/<n> <graph> 256 <k> <kernel> <ms>", kernels
//   dense_spmm      the dense SpMM comparison (main.cu times cuSPARSE here;
//                   this is the library's HIP dense SpMM on the same input)
//   maxk            forward SpGEMM (merge-path schedule, no pre-zeroing)
//   maxk_backward   backward SSpMM, the fastest of the algorithms below
//   maxk_backward_{atomic,staged,staged_edge,append,append_edge,local,tile}
//                   (staged_edge / append_edge: the edge selectors written by
//                   maxk_spgemm_forward_esel; append: its plan from
//                   maxk_append_plan_build; tile: k in {32, 64}; its plan
//                   from maxk_tile_plan_build, as MaxKGraph.tile_plan builds it)
// Each time is the mean of 4 runs after 4 warm-ups, each run followed by a
// device synchronise (spmm_base.h:58-75).  --check compares the forward
// with the dense SpMM of the densified input (main.cu:18-48's check_err) and
// every backward algorithm with ATOMIC's result.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <functional>
#include <numeric>
#include <random>
#include <string>
#include <vector>

#include "../../include/maxk_spgemm.h"

namespace {

constexpr int kDimOrigin = 256;
constexpr int kDimKLimit = 64;
const int kDimKList[] = {16, 32, 64};

#define HIPCHECK(x)                                                                       \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            std::fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, \
                         __LINE__);                                                       \
            std::exit(2);                                                                 \
        }                                                                                 \
    } while (0)

#define MAXKCHECK(x)                                                                      \
    do {                                                                                  \
        int rc_ = (x);                                                                    \
        if (rc_ != 0) {                                                                   \
            std::fprintf(stderr, "%s failed: %d at %s:%d\n", #x, rc_, __FILE__, __LINE__); \
            std::exit(3);                                                                 \
        }                                                                                 \
    } while (0)

template <typename T>
std::vector<T> read_array(const std::string &path)
{
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    if (!f) {
        std::fprintf(stderr, "cannot open %s\n", path.c_str());
        std::exit(1);
    }
    const std::streamsize bytes = f.tellg();
    f.seekg(0);
    std::vector<T> v((size_t)bytes / sizeof(T));
    f.read(reinterpret_cast<char *>(v.data()), (std::streamsize)(v.size() * sizeof(T)));
    return v;
}

template <typename T>
T *to_device(const std::vector<T> &h)
{
    T *d = nullptr;
    HIPCHECK(hipMalloc(&d, std::max<size_t>(h.size(), 1) * sizeof(T)));
    if (!h.empty()) HIPCHECK(hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    return d;
}

template <typename T>
T *dev_alloc(size_t n)
{
    T *d = nullptr;
    HIPCHECK(hipMalloc(&d, std::max<size_t>(n, 1) * sizeof(T)));
    return d;
}

// spmm_base.h:58-75: 4 warm-ups, then 4 runs each closed by a synchronise; mean ms
double time_ms(const std::function<void()> &run)
{
    const int times = 4;
    for (int i = 0; i < times; ++i) run();
    HIPCHECK(hipDeviceSynchronize());
    double total = 0;
    for (int i = 0; i < times; ++i) {
        const auto t0 = std::chrono::steady_clock::now();
        run();
        HIPCHECK(hipDeviceSynchronize());
        const auto t1 = std::chrono::steady_clock::now();
        total += std::chrono::duration<double, std::milli>(t1 - t0).count();
    }
    return total / times;
}

struct Local {  // LOCAL backward plan and its bands
    int32_t *dstart = nullptr, *woff = nullptr, *erc = nullptr, *perm = nullptr, *seg = nullptr;
    float *ev = nullptr;
    int W = 0, dmax = 0, bands = 0;
};

void test_graph(const std::string &dir, const std::string &graph, int idx, int count, bool check)
{
    const std::vector<int32_t> h_indptr = read_array<int32_t>(dir + graph + ".indptr");
    const std::vector<int32_t> h_indices = read_array<int32_t>(dir + graph + ".indices");
    const int V = (int)h_indptr.size() - 1;
    const int64_t E = (int64_t)h_indices.size();
    if (V < 1 || h_indptr[0] != 0 || h_indptr[V] != E) {
        std::fprintf(stderr, "%s: malformed CSR\n", graph.c_str());
        std::exit(1);
    }
    // main.cu:74-96
    std::default_random_engine engine;
    engine.seed(123);
    std::uniform_real_distribution<float> rd(0, 1);
    std::vector<float> h_val(E), h_data((size_t)V * kDimKLimit), h_dense((size_t)V * kDimOrigin);
    std::generate(h_val.begin(), h_val.end(), [&] { return rd(engine); });
    std::generate(h_data.begin(), h_data.end(), [&] { return rd(engine); });
    std::generate(h_dense.begin(), h_dense.end(), [&] { return rd(engine); });
    std::vector<uint8_t> h_sel((size_t)V * kDimKLimit);
    std::vector<int> sequence(kDimOrigin);
    std::iota(sequence.begin(), sequence.end(), 0);

    hipStream_t st;
    HIPCHECK(hipStreamCreate(&st));
    int32_t *indptr = to_device(h_indptr), *indices = to_device(h_indices);
    float *val = to_device(h_val);
    float *data = dev_alloc<float>((size_t)V * kDimKLimit);
    uint8_t *sel = dev_alloc<uint8_t>((size_t)V * kDimKLimit);
    float *dense = dev_alloc<float>((size_t)V * kDimOrigin);
    float *y = dev_alloc<float>((size_t)V * kDimOrigin), *y_ref = dev_alloc<float>((size_t)V * kDimOrigin);
    float *dxs = dev_alloc<float>((size_t)V * kDimKLimit);

    // schedule + forward workspace (one per graph)
    int64_t P = 0;
    MAXKCHECK(maxk_schedule_num_panels(V, E, MAXK_DEFAULT_PANEL_COST, MAXK_DEFAULT_ROW_COST, &P));
    int32_t *sched = dev_alloc<int32_t>(2 * (size_t)(P + 1));
    MAXKCHECK(maxk_schedule_build(indptr, V, MAXK_DEFAULT_PANEL_COST, MAXK_DEFAULT_ROW_COST, sched, P, st));
    const size_t fws_b = maxk_forward_workspace_bytes(P, kDimOrigin);
    void *fws = dev_alloc<char>(fws_b);
    // CSC transpose (STAGED) and its schedule
    int32_t *csc_indptr = dev_alloc<int32_t>((size_t)V + 1), *csc_pos = dev_alloc<int32_t>(E);
    {
        const size_t b = maxk_csc_workspace_bytes(E, V);
        void *ws = dev_alloc<char>(b);
        MAXKCHECK(maxk_csc_build(indices, E, V, csc_indptr, csc_pos, ws, b, st));
        HIPCHECK(hipStreamSynchronize(st));
        HIPCHECK(hipFree(ws));
    }
    int64_t CP = 0;
    MAXKCHECK(maxk_schedule_num_panels(V, E, MAXK_DEFAULT_PANEL_COST, MAXK_DEFAULT_ROW_COST, &CP));
    int32_t *csched = dev_alloc<int32_t>(2 * (size_t)(CP + 1));
    MAXKCHECK(maxk_schedule_build(csc_indptr, V, MAXK_DEFAULT_PANEL_COST, MAXK_DEFAULT_ROW_COST, csched, CP, st));

    hipDeviceProp_t prop;
    HIPCHECK(hipGetDeviceProperties(&prop, 0));

    // column-blocked forward (include/maxk_spgemm.h, maxk_rows_sum): the CSR
    // restacked into kBlocks column blocks, its schedule and workspaces
    constexpr int kBlocks = 4;
    int32_t *b_indptr = dev_alloc<int32_t>((size_t)kBlocks * V + 1);
    int32_t *b_indices = dev_alloc<int32_t>(E > 0 ? E : 1), *b_order = dev_alloc<int32_t>(E > 0 ? E : 1);
    float *b_val = dev_alloc<float>(E > 0 ? E : 1);
    {
        const size_t b = maxk_blocked_plan_workspace_bytes(E, V, kBlocks);
        void *ws = dev_alloc<char>(b);
        MAXKCHECK(maxk_blocked_plan_build(indptr, indices, val, V, V, E, kBlocks, b_indptr, b_indices,
                                          b_val, b_order, ws, b, st));
        HIPCHECK(hipStreamSynchronize(st));
        HIPCHECK(hipFree(ws));
    }
    int64_t BP = 0;
    MAXKCHECK(maxk_schedule_num_panels((int64_t)kBlocks * V, E, MAXK_DEFAULT_PANEL_COST,
                                       MAXK_DEFAULT_ROW_COST, &BP));
    int32_t *b_sched = dev_alloc<int32_t>(2 * (size_t)(BP + 1));
    MAXKCHECK(maxk_schedule_build(b_indptr, kBlocks * V, MAXK_DEFAULT_PANEL_COST,
                                  MAXK_DEFAULT_ROW_COST, b_sched, BP, st));
    const size_t bws_b = maxk_forward_workspace_bytes(BP, kDimOrigin);
    void *bws = dev_alloc<char>(bws_b);
    float *parts = dev_alloc<float>((size_t)kBlocks * V * kDimOrigin);
    float *y_blk = dev_alloc<float>((size_t)V * kDimOrigin);

    std::printf("num graph dim_origin dim_k kernel time(ms)\n");
    for (size_t n = 0; n < sizeof(kDimKList) / sizeof(int); ++n) {
        const int k = kDimKList[n];
        if (k > kDimKLimit) break;
        const std::string out = std::to_string(idx) + "/" + std::to_string(count) + " " + graph + " " +
                                std::to_string(kDimOrigin) + " " + std::to_string(k);
        // main.cu:111-146 (rows stored with stride k, DIM_MUL_N = 1)
        std::vector<int> sample(k);
        for (int i = 0; i < V; ++i) {
            std::sample(sequence.begin(), sequence.end(), sample.begin(), k, engine);
            for (int j = 0; j < k; ++j) {
                h_data[(size_t)i * k + j] = rd(engine);
                h_sel[(size_t)i * k + j] = (uint8_t)sample[j];
            }
        }
        std::fill(h_dense.begin(), h_dense.end(), 0.f);
        for (int i = 0; i < V; ++i)
            for (int j = 0; j < k; ++j)
                h_dense[(size_t)i * kDimOrigin + h_sel[(size_t)i * k + j]] = h_data[(size_t)i * k + j];
        HIPCHECK(hipMemcpy(data, h_data.data(), (size_t)V * k * 4, hipMemcpyHostToDevice));
        HIPCHECK(hipMemcpy(sel, h_sel.data(), (size_t)V * k, hipMemcpyHostToDevice));
        HIPCHECK(hipMemcpy(dense, h_dense.data(), h_dense.size() * 4, hipMemcpyHostToDevice));

        auto dense_spmm = [&] {
            MAXKCHECK(maxk_spmm_dense_forward(sched, P, indptr, indices, val, dense, V, kDimOrigin,
                                              y_ref, fws, fws_b, st));
        };
        if (n == 0) std::printf("%s dense_spmm %g\n", out.c_str(), time_ms(dense_spmm));
        auto fwd = [&] {
            MAXKCHECK(maxk_spgemm_forward(sched, P, indptr, indices, val, data, sel, V, kDimOrigin, k,
                                          y, fws, fws_b, st));
        };
        std::printf("%s maxk %g\n", out.c_str(), time_ms(fwd));
        if (check) {
            dense_spmm();
            fwd();
            HIPCHECK(hipDeviceSynchronize());
            std::vector<float> a((size_t)V * kDimOrigin), b(a.size());
            HIPCHECK(hipMemcpy(a.data(), y, a.size() * 4, hipMemcpyDeviceToHost));
            HIPCHECK(hipMemcpy(b.data(), y_ref, b.size() * 4, hipMemcpyDeviceToHost));
            double err_sum = 0;
            for (size_t i = 0; i < a.size(); ++i) err_sum += std::fabs((double)a[i] - b[i]);
            std::printf("err sum = %g  %s\n", err_sum,
                        err_sum / a.size() < 0.001 ? "validation pass!" : "validation fail!");
        }

        if (k >= 32) {  // the column-blocked forward: same Y up to the fp32 regrouping by block
            auto fwd_blk = [&] {
                MAXKCHECK(maxk_spgemm_forward_ex(b_sched, BP, b_indptr, b_indices, b_val, data, sel,
                                                 kBlocks * V, kDimOrigin, k, MAXK_FWD_CACHED_GATHER,
                                                 parts, bws, bws_b, st));
                MAXKCHECK(maxk_rows_sum(parts, kBlocks, (int64_t)V * kDimOrigin, y_blk, st));
            };
            std::printf("%s maxk_blocked%d %g\n", out.c_str(), kBlocks, time_ms(fwd_blk));
            if (check) {
                fwd();
                fwd_blk();
                HIPCHECK(hipDeviceSynchronize());
                std::vector<float> a((size_t)V * kDimOrigin), b(a.size());
                HIPCHECK(hipMemcpy(a.data(), y_blk, a.size() * 4, hipMemcpyDeviceToHost));
                HIPCHECK(hipMemcpy(b.data(), y, b.size() * 4, hipMemcpyDeviceToHost));
                double worst = 0;
                for (size_t i = 0; i < a.size(); ++i)
                    worst = std::max(worst, std::fabs((double)a[i] - b[i]) / std::max(1.0, std::fabs((double)b[i])));
                std::printf("forward blocked%d vs plain: max rel diff %g  %s\n", kBlocks, worst,
                            worst <= 1e-4 ? "validation pass!" : "validation fail!");
            }
        }

        // backward: every algorithm, then the fastest as maxk_backward; with
        // --check each result is compared with ATOMIC's (same fp32 sums in another
        // order: per element |a - b| <= 1e-4 * max(1, |b|))
        double best = 1e30;
        std::vector<float> dx_ref;
        auto compare = [&](const char *name) {
            if (!check) return;
            HIPCHECK(hipDeviceSynchronize());
            std::vector<float> got((size_t)V * k);
            HIPCHECK(hipMemcpy(got.data(), dxs, got.size() * 4, hipMemcpyDeviceToHost));
            if (dx_ref.empty()) { dx_ref = got; return; }
            double worst = 0;
            for (size_t i = 0; i < got.size(); ++i)
                worst = std::max(worst, std::fabs((double)got[i] - dx_ref[i]) /
                                            std::max(1.0, std::fabs((double)dx_ref[i])));
            std::printf("backward %s vs atomic: max rel diff %g  %s\n", name, worst,
                        worst <= 1e-4 ? "validation pass!" : "validation fail!");
        };
        {
            const size_t b = maxk_backward_workspace_bytes(MAXK_BWD_ATOMIC, E, k, CP);
            void *ws = dev_alloc<char>(b);
            const double t = time_ms([&] {
                MAXKCHECK(maxk_sspmm_backward(MAXK_BWD_ATOMIC, sched, P, indptr, indices, val, dense,
                                              sel, V, V, E, kDimOrigin, k, dxs, nullptr, nullptr, 0,
                                              nullptr, ws, b, st));
            });
            std::printf("%s maxk_backward_atomic %g\n", out.c_str(), t);
            compare("atomic");
            best = std::min(best, t);
            HIPCHECK(hipFree(ws));
        }
        {
            const size_t b = maxk_backward_workspace_bytes(MAXK_BWD_STAGED, E, k, CP);
            void *ws = dev_alloc<char>(b);
            const double t = time_ms([&] {
                MAXKCHECK(maxk_sspmm_backward(MAXK_BWD_STAGED, sched, P, indptr, indices, val, dense,
                                              sel, V, V, E, kDimOrigin, k, dxs, csc_pos, csched, CP,
                                              csc_indptr, ws, b, st));
            });
            std::printf("%s maxk_backward_staged %g\n", out.c_str(), t);
            compare("staged");
            best = std::min(best, t);
            // STAGED_EDGE: the forward stores the edge selectors, the backward reads them
            uint8_t *esel = dev_alloc<uint8_t>((size_t)E * k);
            MAXKCHECK(maxk_spgemm_forward_esel(sched, P, indptr, indices, val, data, sel, nullptr, V,
                                               kDimOrigin, k, y, esel, fws, fws_b, st));
            const double te = time_ms([&] {
                MAXKCHECK(maxk_sspmm_backward(MAXK_BWD_STAGED_EDGE, sched, P, indptr, indices, val,
                                              dense, esel, V, V, E, kDimOrigin, k, dxs, csc_pos,
                                              csched, CP, csc_indptr, ws, b, st));
            });
            std::printf("%s maxk_backward_staged_edge %g\n", out.c_str(), te);
            compare("staged_edge");
            best = std::min(best, te);
            HIPCHECK(hipFree(ws));
            // APPEND (non-deterministic like ATOMIC): plan for the schedule passed
            // below, then node selectors and the edge selectors stored above
            int nb = 0, bs = 0;
            MAXKCHECK(maxk_append_bins(V, k, &nb, &bs));
            int32_t *region_base = dev_alloc<int32_t>((size_t)nb * 8 + 1);
            MAXKCHECK(maxk_append_plan_build(sched, P, indptr, indices, V, V, k, region_base, nb,
                                             bs, st));
            const size_t ab = maxk_backward_append_workspace_bytes(E, k, nb);
            void *aws = dev_alloc<char>(ab);
            for (int es = 0; es < 2; ++es) {
                const double ta = time_ms([&] {
                    MAXKCHECK(maxk_sspmm_backward_append(sched, P, indptr, indices, val, 1, dense,
                                                         es ? esel : sel, es, V, V, E, kDimOrigin, k,
                                                         region_base, nb, bs, dxs, aws, ab, st));
                });
                const char *name = es ? "append_edge" : "append";
                std::printf("%s maxk_backward_%s %g\n", out.c_str(), name, ta);
                compare(name);
                best = std::min(best, ta);
            }
            HIPCHECK(hipFree(aws));
            HIPCHECK(hipFree(region_base));
            HIPCHECK(hipFree(esel));
        }
        if (64 % k == 0 && E > 0) {
            // the plan MaxKGraph.local_plan() builds: ~10 KB of LDS per wave, 16 waves per CU
            Local L;
            L.dmax = std::max(1, std::min(256, 10 * 1024 / (5 * k)));
            const int T = std::max((V + L.dmax - 1) / L.dmax, std::min(prop.multiProcessorCount * 16, V));
            const size_t b = maxk_local_plan_workspace_bytes(E, V, T);
            void *ws = dev_alloc<char>(b);
            MAXKCHECK(maxk_local_plan_build(indptr, indices, val, V, V, E, csc_indptr, L.dmax, T,
                                            nullptr, nullptr, nullptr, nullptr, nullptr, &L.W, ws, b, st));
            L.dstart = dev_alloc<int32_t>((size_t)L.W + 1);
            L.woff = dev_alloc<int32_t>((size_t)L.W + 1);
            L.erc = dev_alloc<int32_t>(E);
            L.perm = dev_alloc<int32_t>(E);
            L.ev = dev_alloc<float>(E);
            MAXKCHECK(maxk_local_plan_build(indptr, indices, val, V, V, E, csc_indptr, L.dmax, T,
                                            L.dstart, L.woff, L.erc, L.perm, L.ev, &L.W, ws, b, st));
            // source bands of about 32 MB of G
            const int64_t gbytes = (int64_t)V * kDimOrigin * 4;
            L.bands = (int)std::min<int64_t>(V, std::max<int64_t>(1, (gbytes + (32 << 20) - 1) >> 25));
            L.seg = dev_alloc<int32_t>((size_t)(L.bands + 1) * L.W);
            MAXKCHECK(maxk_local_bands_build(L.woff, L.erc, L.W, V, L.bands, L.seg, st));
            HIPCHECK(hipStreamSynchronize(st));
            const double t = time_ms([&] {
                MAXKCHECK(maxk_sspmm_backward_local(L.seg, L.bands, L.dstart, L.W, L.dmax, L.erc, L.ev,
                                                    dense, sel, V, kDimOrigin, k, dxs, st));
            });
            std::printf("%s maxk_backward_local %g\n", out.c_str(), t);
            compare("local");
            best = std::min(best, t);
            for (void *p : {(void *)L.dstart, (void *)L.woff, (void *)L.erc, (void *)L.perm,
                            (void *)L.ev, (void *)L.seg, ws})
                HIPCHECK(hipFree(p));
        }
        if ((k == 32 || k == 64) && E > 0) {
            int G = 0, GS = 0, P = 0;
            MAXKCHECK(maxk_tile_plan_shape(V, V, prop.multiProcessorCount, k, &G, &GS, &P));
            const size_t b = maxk_tile_plan_workspace_bytes(E, G, P);
            const int NP = G + P - 1;   // plan pieces
            void *ws = dev_alloc<char>(b);
            int64_t sizes[3] = {0, 0, 0};
            MAXKCHECK(maxk_tile_plan_build(indptr, indices, val, V, V, E, k, G, GS, P, nullptr, 0,
                                           nullptr, nullptr, 0, nullptr, nullptr, nullptr, sizes, ws,
                                           b, st));
            if (sizes[2] <= 0xFFFF) {
                const int nw = NP * 16;
                void *hdrs = dev_alloc<int32_t>((size_t)sizes[0] * 4);
                void *recs = dev_alloc<int32_t>((size_t)sizes[1] * maxk_tile_record_words());
                int64_t *hstart = dev_alloc<int64_t>(nw), *rstart = dev_alloc<int64_t>(nw);
                int32_t *nch = dev_alloc<int32_t>((size_t)NP);
                MAXKCHECK(maxk_tile_plan_build(indptr, indices, val, V, V, E, k, G, GS, P, hdrs,
                                               sizes[0], hstart, recs, sizes[1], rstart, nch, nullptr,
                                               sizes, ws, b, st));
                std::vector<float> zeros(kDimOrigin, 0.f);
                float *zero_row = to_device(zeros);
                const int planes = maxk_tile_part_planes(V, G, P);
                float *part = planes > 0 ? dev_alloc<float>((size_t)planes * V * k) : nullptr;
                const double t = time_ms([&] {
                    MAXKCHECK(maxk_sspmm_backward_tile(hdrs, hstart, recs, rstart, nch, G, P, GS,
                                                       dense, zero_row, sel, V, V, kDimOrigin, k,
                                                       dxs, part, st));
                });
                std::printf("%s maxk_backward_tile %g\n", out.c_str(), t);
                compare("tile");
                best = std::min(best, t);
                for (void *q : {hdrs, recs, (void *)hstart, (void *)rstart, (void *)nch,
                                (void *)zero_row, (void *)part})
                    if (q) HIPCHECK(hipFree(q));
            }
            HIPCHECK(hipFree(ws));
        }
        std::printf("%s maxk_backward %g\n", out.c_str(), best);
        std::fflush(stdout);
    }
    for (void *p : {(void *)indptr, (void *)indices, (void *)val, (void *)data, (void *)sel,
                    (void *)dense, (void *)y, (void *)y_ref, (void *)dxs, (void *)sched, fws,
                    (void *)csc_indptr, (void *)csc_pos, (void *)csched})
        HIPCHECK(hipFree(p));
    HIPCHECK(hipStreamDestroy(st));
}

}  // namespace

int main(int argc, char **argv)
{
    std::string dir = "../graphs/", graph;
    bool check = false;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        if (a == "--dir" && i + 1 < argc) {
            dir = argv[++i];
            if (!dir.empty() && dir.back() != '/') dir += '/';
        } else if (a == "--check") {
            check = true;
        } else if (a == "-h" || a == "--help") {
            std::printf("usage: %s [graph] [--dir DIR] [--check]\n", argv[0]);
            return 0;
        } else {
            graph = a;
        }
    }
    std::printf("%s\n", maxk_version());
    if (!graph.empty()) {
        test_graph(dir, graph, 1, 1, check);
        return 0;
    }
    std::vector<std::string> names;
    for (const auto &f : std::filesystem::directory_iterator(dir))
        if (f.path().extension() == ".indptr") names.push_back(f.path().stem().string());
    std::sort(names.begin(), names.end());
    for (size_t i = 0; i < names.size(); ++i) {
        test_graph(dir, names[i], (int)i + 1, (int)names.size(), check);
        HIPCHECK(hipDeviceSynchronize());
    }
    return 0;
}
