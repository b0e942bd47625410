// fwd_ablate.hip -- standalone timing ablation of the forward SpGEMM inner loop
// (development tool, not part of the product library).
//
// Reddit-shaped random graph (uniform degrees in [0, 2*avg], random columns),
// h = 256, k = K.  Each variant is timed with hipEvents over REPS launches.
//   v0  production form: ds_add_f32 into one LDS row per wave
//   v1  gathers only (no LDS): products summed in registers
//   v2  one LDS row copy per edge slot (no same-address collision inside an
//       instruction), ds_add_f32, copies summed at flush
//   v3  LDS adds only (synthetic selectors, no CBSR gathers)
//   v4  like v0 but idx/val read per lane from global (no ds_bpermute)
//   v5  like v0 but ds_read + ds_write (non-atomic RMW, slot copies as v2)
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int kWave = 64;

template <int K, int MODE>
__global__ __launch_bounds__(256) void fwd(const int2 *__restrict__ panels, int P,
                                           const int *__restrict__ indptr,
                                           const int *__restrict__ idx,
                                           const float *__restrict__ val,
                                           const float *__restrict__ data,
                                           const unsigned char *__restrict__ sel,
                                           float *__restrict__ out)
{
    constexpr int LPE = K / 4, EPS = kWave / LPE, STEPS = LPE, U = STEPS < 8 ? STEPS : 8;
    constexpr bool COPIES = (MODE == 2 || MODE == 5);
    constexpr int NC = COPIES ? EPS : 1;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    float *acc = lds + wv * NC * 256;
    const int w = blockIdx.x * 4 + wv;
    if (w >= P) return;
    for (int c = lane; c < NC * 256; c += 64) acc[c] = 0.f;
    __builtin_amdgcn_wave_barrier();
    const int sub = lane % LPE, slot = lane / LPE;
    float *myacc = acc + (COPIES ? slot * 256 : 0);
    float reg = 0.f;
    const int2 pr = panels[w];
    for (int r = pr.x; r < pr.y; ++r) {
        const int e0 = indptr[r], e1 = indptr[r + 1];
        for (int base = e0; base < e1; base += 64) {
            const int n = min(64, e1 - base);
            int my_c = 0;
            float my_v = 0.f;
            if (lane < n) { my_c = idx[base + lane]; my_v = val[base + lane]; }
#pragma unroll
            for (int s0 = 0; s0 < STEPS; s0 += U) {
                if (s0 * EPS >= n) break;
                f4 d[U];
                unsigned sb[U];
                float v[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int t = (s0 + u) * EPS + slot;
                    int c;
                    if constexpr (MODE == 4) {
                        c = t < n ? idx[base + t] : 0;
                        v[u] = t < n ? val[base + t] : 0.f;
                    } else {
                        c = __shfl(my_c, t < 64 ? t : 0);
                        v[u] = __shfl(my_v, t < 64 ? t : 0);
                    }
                    if (t < n) {
                        if constexpr (MODE == 3) {
                            d[u] = f4{v[u], v[u], v[u], v[u]};
                            sb[u] = (unsigned)(c * 2654435761u) ^ (unsigned)(t * 40503u);
                        } else {
                            const size_t off = (size_t)c * K + sub * 4;
                            d[u] = *reinterpret_cast<const f4 *>(data + off);
                            sb[u] = *reinterpret_cast<const unsigned *>(sel + off);
                        }
                    } else {
                        v[u] = 0.f; d[u] = f4{0, 0, 0, 0}; sb[u] = 0;
                    }
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int t = (s0 + u) * EPS + slot;
                    if (t < n) {
                        if constexpr (MODE == 1) {
                            reg += v[u] * (d[u].x + d[u].y + d[u].z + d[u].w) + (float)(sb[u] & 1);
                        } else if constexpr (MODE == 5) {
                            float *p0 = myacc + (sb[u] & 0xff), *p1 = myacc + ((sb[u] >> 8) & 0xff);
                            float *p2 = myacc + ((sb[u] >> 16) & 0xff), *p3 = myacc + (sb[u] >> 24);
                            *p0 += v[u] * d[u].x; *p1 += v[u] * d[u].y;
                            *p2 += v[u] * d[u].z; *p3 += v[u] * d[u].w;
                        } else {
                            __hip_atomic_fetch_add(myacc + (sb[u] & 0xff), v[u] * d[u].x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                            __hip_atomic_fetch_add(myacc + ((sb[u] >> 8) & 0xff), v[u] * d[u].y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                            __hip_atomic_fetch_add(myacc + ((sb[u] >> 16) & 0xff), v[u] * d[u].z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                            __hip_atomic_fetch_add(myacc + (sb[u] >> 24), v[u] * d[u].w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                        }
                    }
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        f4 a = reinterpret_cast<f4 *>(acc)[lane];
        reinterpret_cast<f4 *>(acc)[lane] = f4{0, 0, 0, 0};
        for (int cp = 1; cp < NC; ++cp) {
            a += reinterpret_cast<f4 *>(acc + cp * 256)[lane];
            reinterpret_cast<f4 *>(acc + cp * 256)[lane] = f4{0, 0, 0, 0};
        }
        if constexpr (MODE == 1) a.x += reg;
        reinterpret_cast<f4 *>(out + (size_t)r * 256)[lane] = a;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

template <int K, int MODE>
float run(const int2 *panels, int P, const int *indptr, const int *idx, const float *val,
          const float *data, const unsigned char *sel, float *out, int reps)
{
    constexpr int LPE = K / 4, EPS = 64 / LPE;
    const int nc = (MODE == 2 || MODE == 5) ? EPS : 1;
    const size_t lds = 4 * nc * 256 * sizeof(float);
    if (lds > 160 * 1024) return -1.f;
    dim3 g((P + 3) / 4), b(256);
    hipLaunchKernelGGL((fwd<K, MODE>), g, b, lds, 0, panels, P, indptr, idx, val, data, sel, out);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL((fwd<K, MODE>), g, b, lds, 0, panels, P, indptr, idx, val, data, sel, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

template <int K>
void sweep(int V, long long E, int reps, const int *d_indptr, const int *d_idx, const float *d_val,
           const std::vector<int> &indptr, float *d_out)
{
    std::mt19937 rng(7);
    std::vector<float> data((size_t)V * K);
    std::vector<unsigned char> sel((size_t)V * K);
    std::vector<int> perm(256);
    for (int i = 0; i < 256; ++i) perm[i] = i;
    for (int v = 0; v < V; ++v) {
        for (int j = 0; j < K; ++j) { int q = j + rng() % (256 - j); std::swap(perm[j], perm[q]); }
        for (int j = 0; j < K; ++j) { sel[(size_t)v * K + j] = perm[j]; data[(size_t)v * K + j] = (rng() % 1000) / 1000.f; }
    }
    float *d_data; unsigned char *d_sel;
    CK(hipMalloc(&d_data, data.size() * 4)); CK(hipMalloc(&d_sel, sel.size()));
    CK(hipMemcpy(d_data, data.data(), data.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_sel, sel.data(), sel.size(), hipMemcpyHostToDevice));
    for (int pc : {1024, 2048, 4096}) {
        std::vector<int2> panels;
        int r0 = 0; long long acc = 0;
        for (int r = 0; r < V; ++r) {
            acc += indptr[r + 1] - indptr[r] + 16;
            if (acc >= pc) { panels.push_back(make_int2(r0, r + 1)); r0 = r + 1; acc = 0; }
        }
        if (r0 < V) panels.push_back(make_int2(r0, V));
        int2 *d_p; CK(hipMalloc(&d_p, panels.size() * sizeof(int2)));
        CK(hipMemcpy(d_p, panels.data(), panels.size() * sizeof(int2), hipMemcpyHostToDevice));
        const int P = (int)panels.size();
        const double bytes = 8.0 * E + 5.0 * K * E + 4.0 * 256 * V;
        float t[6] = {run<K, 0>(d_p, P, d_indptr, d_idx, d_val, d_data, d_sel, d_out, reps),
                      run<K, 1>(d_p, P, d_indptr, d_idx, d_val, d_data, d_sel, d_out, reps),
                      run<K, 2>(d_p, P, d_indptr, d_idx, d_val, d_data, d_sel, d_out, reps),
                      run<K, 3>(d_p, P, d_indptr, d_idx, d_val, d_data, d_sel, d_out, reps),
                      run<K, 4>(d_p, P, d_indptr, d_idx, d_val, d_data, d_sel, d_out, reps),
                      run<K, 5>(d_p, P, d_indptr, d_idx, d_val, d_data, d_sel, d_out, reps)};
        printf("K=%d panel_cost=%d P=%d :", K, pc, P);
        for (int i = 0; i < 6; ++i) printf("  v%d %.3f ms (%.0f GB/s)", i, t[i], t[i] > 0 ? bytes / t[i] / 1e6 : 0.0);
        printf("\n");
        fflush(stdout);
        CK(hipFree(d_p));
    }
    CK(hipFree(d_data)); CK(hipFree(d_sel));
}

int main(int argc, char **argv)
{
    const int V = argc > 1 ? atoi(argv[1]) : 232965;
    const long long Etarget = argc > 2 ? atoll(argv[2]) : 114615892LL;
    const int reps = argc > 3 ? atoi(argv[3]) : 5;
    const int avg = (int)(Etarget / V);
    std::mt19937_64 rng(123);
    std::vector<int> indptr(V + 1, 0);
    for (int v = 0; v < V; ++v) indptr[v + 1] = indptr[v] + (int)(rng() % (2 * avg + 1));
    const long long E = indptr[V];
    std::vector<int> idx(E);
    std::vector<float> val(E);
    for (long long e = 0; e < E; ++e) { idx[e] = (int)(rng() % V); val[e] = (rng() % 1000) / 1000.f; }
    printf("V=%d E=%lld\n", V, E);
    int *d_indptr, *d_idx; float *d_val, *d_out;
    CK(hipMalloc(&d_indptr, (V + 1) * 4)); CK(hipMalloc(&d_idx, E * 4)); CK(hipMalloc(&d_val, E * 4));
    CK(hipMalloc(&d_out, (size_t)V * 256 * 4));
    CK(hipMemcpy(d_indptr, indptr.data(), (V + 1) * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_idx, idx.data(), E * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_val, val.data(), E * 4, hipMemcpyHostToDevice));
    sweep<32>(V, E, reps, d_indptr, d_idx, d_val, indptr, d_out);
    sweep<8>(V, E, reps, d_indptr, d_idx, d_val, indptr, d_out);
    sweep<64>(V, E, reps, d_indptr, d_idx, d_val, indptr, d_out);
    return 0;
}
