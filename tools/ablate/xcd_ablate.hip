// xcd_ablate.hip -- forward SpGEMM with XCD-aware column classes (development tool).
//
// Columns are split into NC contiguous classes; block b works on class b % NC
// (blocks b and b+8 are observed to share an XCD), so each XCD's L2 sees only
// its class's slice of the CBSR table.  Rows have sorted columns, so a row's
// class-x edges are a contiguous segment [bnd[r][x], bnd[r][x+1]).
// Partial rows go to Y8[x][V][256]; a second kernel sums the NC partials.
//   base : all columns in one pass (current product kernel form), Y written
//   cls  : per-class partial pass (time of the gather phase alone)
//   comb : the combine pass
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)
typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int K = 32, LPE = 8, EPS = 8;

__device__ __forceinline__ void edges(int e0, int e1, const int *__restrict__ idx,
                                      const float *__restrict__ val, const float *__restrict__ data,
                                      const unsigned char *__restrict__ sel, float *acc, int lane)
{
    const int sub = lane % LPE, slot = lane / LPE;
    float *my = acc + slot * 256;
    for (int base = e0; base < e1; base += 64) {
        const int n = min(64, e1 - base);
        int my_c = 0;
        float my_v = 0.f;
        if (lane < n) { my_c = idx[base + lane]; my_v = val[base + lane]; }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int t = u * EPS + slot;
            if (u * EPS >= n) break;
            const int c = __shfl(my_c, t);
            const float v = __shfl(my_v, t);
            if (t < n) {
                const size_t off = (size_t)c * K + sub * 4;
                const f4 d = __builtin_nontemporal_load(reinterpret_cast<const f4 *>(data + off));
                const unsigned sb = *reinterpret_cast<const unsigned *>(sel + off);
                my[sb & 255] += v * d.x; my[(sb >> 8) & 255] += v * d.y;
                my[(sb >> 16) & 255] += v * d.z; my[sb >> 24] += v * d.w;
            }
        }
    }
}

__device__ __forceinline__ void flush(float *acc, float *dst, int lane)
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    f4 a = reinterpret_cast<f4 *>(acc)[lane];
    reinterpret_cast<f4 *>(acc)[lane] = f4{0, 0, 0, 0};
    for (int cp = 1; cp < EPS; ++cp) {
        a += reinterpret_cast<f4 *>(acc + cp * 256)[lane];
        reinterpret_cast<f4 *>(acc + cp * 256)[lane] = f4{0, 0, 0, 0};
    }
    reinterpret_cast<f4 *>(dst)[lane] = a;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// panels: int2 row ranges. CLS: 0 = base, else NC classes.
template <int NC>
__global__ __launch_bounds__(256) void fwd(const int2 *__restrict__ panels, int P,
                                           const int *__restrict__ indptr,
                                           const int *__restrict__ bnd,
                                           const int *__restrict__ idx, const float *__restrict__ val,
                                           const float *__restrict__ data,
                                           const unsigned char *__restrict__ sel,
                                           float *__restrict__ out, int V)
{
    __shared__ __attribute__((aligned(16))) float lds[4 * EPS * 256];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float *acc = lds + wv * EPS * 256;
    for (int i = lane; i < EPS * 256; i += 64) acc[i] = 0.f;
    int x = 0, pidx;
    if constexpr (NC == 0) {
        pidx = blockIdx.x * 4 + wv;
    } else {
        x = blockIdx.x % NC;
        pidx = (blockIdx.x / NC) * 4 + wv;
    }
    if (pidx >= P) return;
    const int2 pr = panels[pidx];
    for (int r = pr.x; r < pr.y; ++r) {
        int e0, e1;
        float *dst;
        if constexpr (NC == 0) {
            e0 = indptr[r]; e1 = indptr[r + 1];
            dst = out + (size_t)r * 256;
        } else {
            e0 = bnd[(size_t)r * (NC + 1) + x]; e1 = bnd[(size_t)r * (NC + 1) + x + 1];
            dst = out + ((size_t)x * V + r) * 256;
        }
        edges(e0, e1, idx, val, data, sel, acc, lane);
        flush(acc, dst, lane);
    }
}

// Sequential classes: one launch per class x, every block on class x; launch 0
// stores rows, later launches add (plain RMW of owned rows).
__global__ __launch_bounds__(256) void fwd_seq(const int2 *__restrict__ panels, int P, int x, int NC,
                                               const int *__restrict__ bnd,
                                               const int *__restrict__ idx, const float *__restrict__ val,
                                               const float *__restrict__ data,
                                               const unsigned char *__restrict__ sel,
                                               float *__restrict__ out)
{
    __shared__ __attribute__((aligned(16))) float lds[4 * EPS * 256];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float *acc = lds + wv * EPS * 256;
    for (int i = lane; i < EPS * 256; i += 64) acc[i] = 0.f;
    const int pidx = blockIdx.x * 4 + wv;
    if (pidx >= P) return;
    const int2 pr = panels[pidx];
    for (int r = pr.x; r < pr.y; ++r) {
        const int e0 = bnd[(size_t)r * (NC + 1) + x], e1 = bnd[(size_t)r * (NC + 1) + x + 1];
        edges(e0, e1, idx, val, data, sel, acc, lane);
        float *dst = out + (size_t)r * 256;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        f4 a = reinterpret_cast<f4 *>(acc)[lane];
        reinterpret_cast<f4 *>(acc)[lane] = f4{0, 0, 0, 0};
        for (int cp = 1; cp < EPS; ++cp) {
            a += reinterpret_cast<f4 *>(acc + cp * 256)[lane];
            reinterpret_cast<f4 *>(acc + cp * 256)[lane] = f4{0, 0, 0, 0};
        }
        if (x > 0) a += reinterpret_cast<f4 *>(dst)[lane];
        reinterpret_cast<f4 *>(dst)[lane] = a;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

template <int NC>
__global__ __launch_bounds__(256) void combine(const float *__restrict__ y8, float *__restrict__ y, size_t n4, int V)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        f4 s = reinterpret_cast<const f4 *>(y8)[i];
#pragma unroll
        for (int x = 1; x < NC; ++x) s += __builtin_nontemporal_load(reinterpret_cast<const f4 *>(y8 + (size_t)x * V * 256) + i);
        reinterpret_cast<f4 *>(y)[i] = s;
    }
}

template <typename F>
float timeit(F f, int reps)
{
    f();
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

template <typename T>
T *up(const std::vector<T> &v)
{
    T *d;
    CK(hipMalloc(&d, std::max<size_t>(1, v.size()) * sizeof(T)));
    CK(hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return d;
}

template <int NC>
void run_cls(int V, const std::vector<int> &indptr, const std::vector<int> &idx, int *d_idx,
             float *d_val, float *d_data, unsigned char *d_sel, int reps, double bytes, float *d_y)
{
    const long long E = indptr[V];
    std::vector<int> bnd((size_t)V * (NC + 1));
    for (int r = 0; r < V; ++r)
        for (int x = 0; x <= NC; ++x) {
            const long long cut = (long long)V * x / NC;
            bnd[(size_t)r * (NC + 1) + x] = (int)(std::lower_bound(idx.begin() + indptr[r], idx.begin() + indptr[r + 1], (int)cut) - idx.begin());
        }
    // row panels per class sized ~2048 edges of that class (same row ranges for every class)
    std::vector<int2> panels;
    int r0 = 0;
    long long acc = 0;
    for (int r = 0; r < V; ++r) {
        acc += (indptr[r + 1] - indptr[r]) / NC + 16;
        if (acc >= 2048) { panels.push_back(make_int2(r0, r + 1)); r0 = r + 1; acc = 0; }
    }
    if (r0 < V) panels.push_back(make_int2(r0, V));
    int *d_bnd = up(bnd);
    int2 *d_p = up(panels);
    const int P = (int)panels.size();
    float *d_y8;
    CK(hipMalloc(&d_y8, (size_t)NC * V * 256 * 4));
    dim3 g((unsigned)(((P + 3) / 4) * NC)), b(256);
    float tc = timeit([&] { hipLaunchKernelGGL((fwd<NC>), g, b, 0, 0, d_p, P, (const int *)nullptr, d_bnd, d_idx, d_val, d_data, d_sel, d_y8, V); }, reps);
    const size_t n4 = (size_t)V * 64;
    float tm = timeit([&] { hipLaunchKernelGGL((combine<NC>), dim3(256 * 16), b, 0, 0, d_y8, d_y, n4, V); }, reps);
    printf("NC=%d: class pass %.3f ms + combine %.3f ms = %.3f ms (%.0f GB/s eff)\n", NC, tc, tm, tc + tm, bytes / (tc + tm) / 1e6);
    fflush(stdout);
    hipFree(d_bnd); hipFree(d_p); hipFree(d_y8);
}

void run_seq(int NC, int V, const std::vector<int> &indptr, const std::vector<int> &idx, int *d_idx,
             float *d_val, float *d_data, unsigned char *d_sel, int reps, double bytes, float *d_y)
{
    std::vector<int> bnd((size_t)V * (NC + 1));
    for (int r = 0; r < V; ++r)
        for (int x = 0; x <= NC; ++x) {
            const long long cut = (long long)V * x / NC;
            bnd[(size_t)r * (NC + 1) + x] = (int)(std::lower_bound(idx.begin() + indptr[r], idx.begin() + indptr[r + 1], (int)cut) - idx.begin());
        }
    std::vector<int2> panels;
    int r0 = 0;
    long long acc = 0;
    for (int r = 0; r < V; ++r) {
        acc += (indptr[r + 1] - indptr[r]) / NC + 16;
        if (acc >= 2048) { panels.push_back(make_int2(r0, r + 1)); r0 = r + 1; acc = 0; }
    }
    if (r0 < V) panels.push_back(make_int2(r0, V));
    int *d_bnd = up(bnd);
    int2 *d_p = up(panels);
    const int P = (int)panels.size();
    float t = timeit([&] {
        for (int x = 0; x < NC; ++x)
            hipLaunchKernelGGL(fwd_seq, dim3((P + 3) / 4), dim3(256), 0, 0, d_p, P, x, NC, d_bnd, d_idx, d_val, d_data, d_sel, d_y);
    }, reps);
    printf("seq NC=%d: %.3f ms (%.0f GB/s eff)\n", NC, t, bytes / t / 1e6);
    fflush(stdout);
    hipFree(d_bnd); hipFree(d_p);
}

int main(int argc, char **argv)
{
    const int V = argc > 1 ? atoi(argv[1]) : 232965;
    const long long Et = argc > 2 ? atoll(argv[2]) : 114615892LL;
    const int reps = 5;
    const int avg = (int)(Et / V);
    std::mt19937_64 rng(123);
    std::vector<int> indptr(V + 1, 0);
    for (int v = 0; v < V; ++v) indptr[v + 1] = indptr[v] + (int)(rng() % (2 * avg + 1));
    const long long E = indptr[V];
    std::vector<int> idx(E);
    for (int v = 0; v < V; ++v) {
        for (int e = indptr[v]; e < indptr[v + 1]; ++e) idx[e] = (int)(rng() % V);
        std::sort(idx.begin() + indptr[v], idx.begin() + indptr[v + 1]);
    }
    std::vector<float> val(E), data((size_t)V * K);
    std::vector<unsigned char> sel((size_t)V * K);
    for (auto &x : val) x = (rng() % 1000) / 1000.f;
    for (auto &x : data) x = (rng() % 1000) / 1000.f;
    std::vector<int> perm(256);
    for (int i = 0; i < 256; ++i) perm[i] = i;
    for (int v = 0; v < V; ++v) {
        for (int j = 0; j < K; ++j) { int q = j + rng() % (256 - j); std::swap(perm[j], perm[q]); }
        for (int j = 0; j < K; ++j) sel[(size_t)v * K + j] = perm[j];
    }
    int *d_ptr = up(indptr), *d_idx = up(idx);
    float *d_val = up(val), *d_data = up(data);
    unsigned char *d_sel = up(sel);
    float *d_y;
    CK(hipMalloc(&d_y, (size_t)V * 256 * 4));
    const double bytes = 8.0 * E + 5.0 * K * E + 4.0 * 256 * V;
    std::vector<int2> panels;
    { int r0 = 0; long long acc = 0;
      for (int r = 0; r < V; ++r) { acc += indptr[r + 1] - indptr[r] + 16; if (acc >= 2048) { panels.push_back(make_int2(r0, r + 1)); r0 = r + 1; acc = 0; } }
      if (r0 < V) panels.push_back(make_int2(r0, V)); }
    int2 *d_p = up(panels);
    const int P = (int)panels.size();
    float tb = timeit([&] { hipLaunchKernelGGL((fwd<0>), dim3((P + 3) / 4), dim3(256), 0, 0, d_p, P, d_ptr, (const int *)nullptr, d_idx, d_val, d_data, d_sel, d_y, V); }, reps);
    printf("V=%d E=%lld base: %.3f ms (%.0f GB/s eff)\n", V, E, tb, bytes / tb / 1e6);
    fflush(stdout);
    for (int nc : {1, 2, 3, 4, 8}) run_seq(nc, V, indptr, idx, d_idx, d_val, d_data, d_sel, reps, bytes, d_y);
    run_cls<8>(V, indptr, idx, d_idx, d_val, d_data, d_sel, reps, bytes, d_y);
    run_cls<4>(V, indptr, idx, d_idx, d_val, d_data, d_sel, reps, bytes, d_y);
    return 0;
}
