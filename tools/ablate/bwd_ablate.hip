// bwd_ablate.hip -- standalone timing ablation of the backward SSpMM
// (development tool, not part of the product library).
//
// Reddit-shaped random graph (uniform degrees in [0, 2*avg], random columns),
// h = 256, k = K.
// Phase-1 (push over CSR rows, G row staged in LDS) variants:
//   p0  P[csc_pos[e]] <- k-vector, non-temporal 16 B stores (scattered rows)
//   p1  same, plain stores
//   p2  P[e] (CSR order, sequential) plain stores
//   p3  like p0 without the LDS gather (LDS cost ablation)
//   pA  atomic push: dXs[c,l] += v*G[r,sel[c,l]] (global float atomics)
// Phase-2 (segmented sum per destination) variants:
//   q0  P in CSC order: contiguous rows per destination
//   q1  P in CSR order: rows gathered through the CSC->CSR edge permutation
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)
typedef float f4 __attribute__((ext_vector_type(4)));

template <int K, int MODE>
__global__ __launch_bounds__(256) void phase1(const int2 *__restrict__ panels, int P,
                                              const int *__restrict__ indptr,
                                              const int *__restrict__ idx,
                                              const float *__restrict__ val,
                                              const int *__restrict__ csc_pos,
                                              const float *__restrict__ G,
                                              const unsigned char *__restrict__ sel,
                                              float *__restrict__ Pbuf, float *__restrict__ dxs,
                                              int split = 0)
{
    __shared__ __attribute__((aligned(16))) float lds[4 * 256];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float *gs = lds + wv * 256;
    const int w = blockIdx.x * 4 + wv;
    if (w >= P) return;
    const int2 pr = panels[w];
    for (int r = pr.x; r < pr.y; ++r) {
        const int e0 = indptr[r], e1 = indptr[r + 1];
        if (e0 == e1) continue;
        __builtin_amdgcn_wave_barrier();
        reinterpret_cast<f4 *>(gs)[lane] = reinterpret_cast<const f4 *>(G + (size_t)r * 256)[lane];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (MODE == 9 || (MODE == 10 && w < split)) {   // atomic push, one entry per lane
            constexpr int EPS = 64 / K;
            const int slot = lane / K, l = lane % K;
            for (int base = e0; base < e1; base += 64) {
                const int n = min(64, e1 - base);
                int my_c = lane < n ? idx[base + lane] : 0;
                float my_v = lane < n ? val[base + lane] : 0.f;
                for (int s = 0; s < n; s += EPS) {
                    const int t = s + slot;
                    const int c = __shfl(my_c, t < 64 ? t : 0);
                    const float v = __shfl(my_v, t < 64 ? t : 0);
                    if (t < n) {
                        const size_t off = (size_t)c * K + l;
                        __hip_atomic_fetch_add(dxs + off, v * gs[sel[off]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
            }
        } else {
            constexpr int LPE = K / 4, EPS = 64 / LPE, STEPS = LPE, U = STEPS < 8 ? STEPS : 8;
            const int sub = lane % LPE, slot = lane / LPE;
            for (int base = e0; base < e1; base += 64) {
                const int n = min(64, e1 - base);
                int my_c = 0, my_p = 0;
                float my_v = 0.f;
                if (lane < n) { my_c = idx[base + lane]; my_v = val[base + lane]; my_p = (MODE == 2) ? base + lane : csc_pos[base + lane]; }
#pragma unroll
                for (int s0 = 0; s0 < STEPS; s0 += U) {
                    if (s0 * EPS >= n) break;
                    unsigned sb[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const int t = (s0 + u) * EPS + slot;
                        const int c = __shfl(my_c, t < 64 ? t : 0);
                        if constexpr (MODE == 4) sb[u] = (unsigned)c;
                        else sb[u] = t < n ? *reinterpret_cast<const unsigned *>(sel + (size_t)c * K + sub * 4) : 0u;
                    }
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const int t = (s0 + u) * EPS + slot;
                        const int p = __shfl(my_p, t < 64 ? t : 0);
                        const float v = __shfl(my_v, t < 64 ? t : 0);
                        if (t < n) {
                            f4 o;
                            if constexpr (MODE == 3 || MODE == 4) {
                                o = f4{v, v * (float)(sb[u] & 255), v, v};
                            } else {
                                o.x = v * gs[sb[u] & 0xff];
                                o.y = v * gs[(sb[u] >> 8) & 0xff];
                                o.z = v * gs[(sb[u] >> 16) & 0xff];
                                o.w = v * gs[sb[u] >> 24];
                            }
                            f4 *dst = reinterpret_cast<f4 *>(Pbuf + (size_t)p * K + sub * 4);
                            if constexpr (MODE == 0 || MODE == 3 || MODE == 4 || MODE == 10) __builtin_nontemporal_store(o, dst);
                            else *dst = o;
                        }
                    }
                }
            }
        }
    }
}

template <int K, int MODE>
__global__ __launch_bounds__(256) void phase2(const int2 *__restrict__ panels, int P,
                                              const int *__restrict__ cptr,
                                              const int *__restrict__ csc_eid,
                                              const float *__restrict__ Pbuf,
                                              float *__restrict__ dxs)
{
    constexpr int LPE = K / 4, EPS = 64 / LPE;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int w = blockIdx.x * 4 + wv;
    if (w >= P) return;
    const int sub = lane % LPE, slot = lane / LPE;
    const int2 pr = panels[w];
    for (int c = pr.x; c < pr.y; ++c) {
        const int q0 = cptr[c], q1 = cptr[c + 1];
        f4 s = f4{0, 0, 0, 0};
        int q = q0 + slot;
        for (; q + 3 * EPS < q1; q += 4 * EPS) {
            f4 t[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const size_t row = MODE == 1 ? (size_t)csc_eid[q + u * EPS] : (size_t)(q + u * EPS);
                t[u] = __builtin_nontemporal_load(reinterpret_cast<const f4 *>(Pbuf + row * K + sub * 4));
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) s += t[u];
        }
        for (; q < q1; q += EPS) {
            const size_t row = MODE == 1 ? (size_t)csc_eid[q] : (size_t)q;
            s += __builtin_nontemporal_load(reinterpret_cast<const f4 *>(Pbuf + row * K + sub * 4));
        }
        for (int m = LPE; m < 64; m <<= 1) {
            s.x += __shfl_xor(s.x, m); s.y += __shfl_xor(s.y, m);
            s.z += __shfl_xor(s.z, m); s.w += __shfl_xor(s.w, m);
        }
        if (lane < LPE) reinterpret_cast<f4 *>(dxs + (size_t)c * K)[sub] = s;
    }
}

static std::vector<int2> make_panels(const std::vector<int> &ptr, int V, int pc)
{
    std::vector<int2> panels;
    int r0 = 0;
    long long acc = 0;
    for (int r = 0; r < V; ++r) {
        acc += ptr[r + 1] - ptr[r] + 16;
        if (acc >= pc) { panels.push_back(make_int2(r0, r + 1)); r0 = r + 1; acc = 0; }
    }
    if (r0 < V) panels.push_back(make_int2(r0, V));
    return panels;
}

template <typename T>
T *up(const std::vector<T> &v)
{
    T *d;
    CK(hipMalloc(&d, std::max<size_t>(1, v.size()) * sizeof(T)));
    CK(hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return d;
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

template <int K>
void sweep(int V, const std::vector<int> &indptr, const std::vector<int> &idx, int reps)
{
    const long long E = indptr[V];
    std::mt19937 rng(11);
    std::vector<unsigned char> sel((size_t)V * K);
    std::vector<int> perm(256);
    std::iota(perm.begin(), perm.end(), 0);
    for (int v = 0; v < V; ++v) {
        for (int j = 0; j < K; ++j) { int q = j + rng() % (256 - j); std::swap(perm[j], perm[q]); }
        for (int j = 0; j < K; ++j) sel[(size_t)v * K + j] = perm[j];
    }
    // CSC
    std::vector<int> cptr(V + 1, 0);
    for (long long e = 0; e < E; ++e) cptr[idx[e] + 1]++;
    for (int v = 0; v < V; ++v) cptr[v + 1] += cptr[v];
    std::vector<int> fill(cptr.begin(), cptr.end() - 1), csc_pos(E), csc_eid(E);
    for (long long e = 0; e < E; ++e) { int p = fill[idx[e]]++; csc_pos[e] = p; csc_eid[p] = (int)e; }
    std::vector<float> val(E), G((size_t)V * 256);
    for (auto &x : val) x = (rng() % 1000) / 1000.f;
    for (auto &x : G) x = (rng() % 1000) / 1000.f;
    int *d_ptr = up(indptr), *d_idx = up(idx), *d_cpos = up(csc_pos), *d_ceid = up(csc_eid),
        *d_cptr = up(cptr);
    float *d_val = up(val), *d_G = up(G);
    unsigned char *d_sel = up(sel);
    float *d_P, *d_dxs;
    CK(hipMalloc(&d_P, (size_t)E * K * 4));
    CK(hipMalloc(&d_dxs, (size_t)V * K * 4));
    auto p1 = make_panels(indptr, V, 2048);
    auto p2 = make_panels(cptr, V, 2048);
    int2 *d_p1 = up(p1), *d_p2 = up(p2);
    const int P1 = (int)p1.size(), P2 = (int)p2.size();
    dim3 b(256), g1((P1 + 3) / 4), g2((P2 + 3) / 4);
    const double bytes = 8.0 * E + 5.0 * K * E + 4.0 * 256 * V;
#define P1RUN(M) timeit([&] { hipLaunchKernelGGL((phase1<K, M>), g1, b, 0, 0, d_p1, P1, d_ptr, d_idx, d_val, d_cpos, d_G, d_sel, d_P, d_dxs); }, reps)
#define P2RUN(M) timeit([&] { hipLaunchKernelGGL((phase2<K, M>), g2, b, 0, 0, d_p2, P2, d_cptr, d_ceid, d_P, d_dxs); }, reps)
    float t0 = P1RUN(0), t1 = P1RUN(1), t2 = P1RUN(2), t3 = P1RUN(3);
    float tA = timeit([&] {
        CK(hipMemsetAsync(d_dxs, 0, (size_t)V * K * 4));
        hipLaunchKernelGGL((phase1<K, 9>), g1, b, 0, 0, d_p1, P1, d_ptr, d_idx, d_val, d_cpos, d_G, d_sel, d_P, d_dxs);
    }, reps);
    float q0 = P2RUN(0), q1 = P2RUN(1);
    float t4 = P1RUN(4);
    for (float f : {0.2f, 0.3f, 0.4f, 0.5f}) {
        const int split = (int)(P1 * f);
        float th = timeit([&] {
            CK(hipMemsetAsync(d_dxs, 0, (size_t)V * K * 4));
            hipLaunchKernelGGL((phase1<K, 10>), g1, b, 0, 0, d_p1, P1, d_ptr, d_idx, d_val, d_cpos, d_G, d_sel, d_P, d_dxs, split);
        }, reps);
        printf("   hybrid f=%.1f phase1 %.3f ms (+ phase2 ~%.3f) = %.3f ms\n", f, th, q0 * (1 - f), th + q0 * (1 - f));
    }
    printf("   p4 (pure scattered write, no sel gather, no LDS) %.3f ms\n", t4);
    printf("K=%d E=%lld  p0(nt scat) %.3f  p1(plain scat) %.3f  p2(seq) %.3f  p3(noLDS) %.3f  | q0(seq) %.3f  q1(gather) %.3f | atomic %.3f ms\n",
           K, E, t0, t1, t2, t3, q0, q1, tA);
    printf("   staged best: scat %.3f ms (%.0f GB/s), seq+gather %.3f ms (%.0f GB/s), atomic %.0f GB/s\n",
           std::min(t0, t1) + q0, bytes / (std::min(t0, t1) + q0) / 1e6, t2 + q1, bytes / (t2 + q1) / 1e6,
           bytes / tA / 1e6);
    fflush(stdout);
    hipFree(d_P); hipFree(d_dxs); hipFree(d_ptr); hipFree(d_idx); hipFree(d_cpos); hipFree(d_ceid);
    hipFree(d_cptr); hipFree(d_val); hipFree(d_G); hipFree(d_sel); hipFree(d_p1); hipFree(d_p2);
}

int main(int argc, char **argv)
{
    const int V = argc > 1 ? atoi(argv[1]) : 232965;
    const long long Et = argc > 2 ? atoll(argv[2]) : 114615892LL;
    const int reps = argc > 3 ? atoi(argv[3]) : 5;
    const int avg = (int)(Et / V);
    std::mt19937_64 rng(123);
    std::vector<int> indptr(V + 1, 0);
    for (int v = 0; v < V; ++v) indptr[v + 1] = indptr[v] + (int)(rng() % (2 * avg + 1));
    const long long E = indptr[V];
    std::vector<int> idx(E);
    for (long long e = 0; e < E; ++e) idx[e] = (int)(rng() % V);
    printf("V=%d E=%lld\n", V, E);
    sweep<32>(V, indptr, idx, reps);
    sweep<8>(V, indptr, idx, reps);
    sweep<64>(V, indptr, idx, reps);
    return 0;
}
