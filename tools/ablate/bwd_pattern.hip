// bwd_pattern.hip -- the ceiling of the products backward's per-edge access
// pattern.  Development tool, not product code.
//
// A push backward (edges in CSR order, row r -> destination column c) must, per
// edge, learn which k columns of G it needs (the destination's selector row, a
// random read of k bytes, or a sequential edge-selector stream written by the
// forward) and deliver k products to destination c (a random write / atomic of
// 4k bytes, or a sequential staging stream that a second pass gathers back).
// This times each of those per-edge patterns alone at products size (E = 124 M
// edges, V = 2.45 M, uniform random columns), with the column stream read as
// the real kernels read it (4 B per edge, non-temporal), so the algorithms'
// times can be set against what their irreducible pattern costs:
//
//   sel      random k-byte selector row read (one sector per edge)
//   rw32     sel + a random 4k-byte plain store (a partial sector at k = 8)
//   rw64     sel + a random 64-byte store (a whole sector, k floats + pad)
//   app      sel + a 4k-byte append in edge order (sequential stream)
//   atom     sel + k random global_atomic_add_f32 by ONE lane (64 rows per
//            wave-instruction: the slow shape, for comparison)
//   atom8    sel + the ATOMIC backward's shape: 8 lanes per edge, one 32-B row
//            of no-return float atomics per edge
//   gath     a random 4k-byte read from an E-row staging table by a
//            permutation (EDGE_GATHER's phase 2) + the column stream
//   w64      a random 64-byte store only (no selector read)
//
// Results are not meaningful values (stores of garbage); only time is.  Each
// lane handles one edge (k = 8: a 32-B product = 2 x dwordx4), 8 edges in
// flight per lane.  usage: bwd_pattern <variant> [k=8] [E_M=123.7] [V=2449029] [reps]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned u2 __attribute__((ext_vector_type(2)));

enum { SEL = 0, RW32, RW64, APP, ATOM, GATH, W64 };

template <int V_, int K>
__global__ __launch_bounds__(256) void pattern(const int *__restrict__ col, long n,
                                               const uint8_t *__restrict__ sel,
                                               float *__restrict__ dst, const float *__restrict__ stage,
                                               const int *__restrict__ perm, float *__restrict__ out)
{
    constexpr int U = 8;
    const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const long nth = (long)gridDim.x * blockDim.x;
    float acc = 0.f;
    for (long base = tid; base < n; base += nth * U) {
        int c[U];
        f4 s0[U], s1[U];
        unsigned sv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long e = base + (long)u * nth;
            c[u] = e < n ? __builtin_nontemporal_load(V_ == GATH ? perm + e : col + e) : 0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if constexpr (V_ == GATH) {
                const f4 *p = reinterpret_cast<const f4 *>(stage + (long)c[u] * K);
                s0[u] = p[0];
                if constexpr (K == 8) s1[u] = p[1];
            } else if constexpr (V_ != W64) {
                // the destination's selector row: k bytes (k = 8: one dwordx2)
                const u2 v = *reinterpret_cast<const u2 *>(sel + (long)c[u] * K);
                sv[u] = v.x ^ v.y;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long e = base + (long)u * nth;
            if (e >= n) continue;
            const float x = V_ == GATH || V_ == W64 ? 1.f : (float)(sv[u] & 0xff);
            f4 p = {x, x + 1.f, x + 2.f, x + 3.f};
            if constexpr (V_ == RW32) {
                f4 *d = reinterpret_cast<f4 *>(dst + (long)c[u] * K);
                d[0] = p;
                d[1] = p;
            } else if constexpr (V_ == RW64 || V_ == W64) {
                f4 *d = reinterpret_cast<f4 *>(dst + (long)c[u] * 16);
                d[0] = p;
                d[1] = p;
                d[2] = p;
                d[3] = p;
            } else if constexpr (V_ == APP) {
                f4 *d = reinterpret_cast<f4 *>(dst + e * K);
                __builtin_nontemporal_store(p, d);
                __builtin_nontemporal_store(p, d + 1);
            } else if constexpr (V_ == ATOM) {
                float *d = dst + (long)c[u] * K;
#pragma unroll
                for (int j = 0; j < K; ++j) atomicAdd(d + j, x);
            } else if constexpr (V_ == GATH) {
                acc += s0[u].x + s0[u].y + s0[u].z + s0[u].w;
                if constexpr (K == 8) acc += s1[u].x + s1[u].w;
            } else {
                acc += x;
            }
        }
    }
    if (acc == 12345.678f) out[tid] = acc;   // practically never: keeps the loads
}

// atom8: the ATOMIC backward's real shape -- 8 lanes per edge, each one no-return
// global_atomic_add_f32 into the destination's 32-B row (one 32-B segment per
// edge per wave-instruction: 8 edges x 32 B), plus the selector read
__global__ __launch_bounds__(256) void atom8(const int *__restrict__ col, long n,
                                             const uint8_t *__restrict__ sel, float *__restrict__ dst)
{
    constexpr int U = 8;
    const int lane = threadIdx.x & 63;
    const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const long waves = ((long)gridDim.x * blockDim.x) >> 6;
    for (long base = wave * 8 * U; base < n; base += waves * 8 * U) {
        int c[U];
        unsigned sv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long e = base + u * 8 + (lane >> 3);
            c[u] = e < n ? __builtin_nontemporal_load(col + e) : 0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) sv[u] = sel[(long)c[u] * 8 + (lane & 7)];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long e = base + u * 8 + (lane >> 3);
            if (e < n)
                __hip_atomic_fetch_add(dst + (long)c[u] * 8 + (lane & 7), (float)(sv[u] & 0xff),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

template <int V_>
float launch(int blocks, const int *col, long n, const uint8_t *sel, float *dst, const float *stage,
             const int *perm, float *out, int reps)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    pattern<V_, 8><<<blocks, 256>>>(col, n, sel, dst, stage, perm, out);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) pattern<V_, 8><<<blocks, 256>>>(col, n, sel, dst, stage, perm, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char **argv)
{
    if (argc < 2) {
        printf("usage: %s sel|rw32|rw64|app|atom|gath|w64|all [E_M] [V] [reps]\n", argv[0]);
        return 2;
    }
    const long n = (long)((argc > 2 ? atof(argv[2]) : 123.718280) * 1e6);
    const long V = argc > 3 ? atol(argv[3]) : 2449029;
    const int reps = argc > 4 ? atoi(argv[4]) : 10;
    const int K = 8;
    int *col, *perm;
    uint8_t *sel;
    float *dst, *stage, *out;
    CK(hipMalloc(&col, n * 4));
    CK(hipMalloc(&perm, n * 4));
    CK(hipMalloc(&sel, V * K));
    CK(hipMalloc(&dst, (n > V ? n : V) * K * 4 * 2));   // append stream (E x 32 B) or V x 64 B
    CK(hipMalloc(&stage, n * K * 4));
    CK(hipMalloc(&out, 1 << 26));
    CK(hipMemset(sel, 1, V * K));
    CK(hipMemset(stage, 0, n * K * 4));
    std::vector<int> h(n);
    unsigned x = 12345u;
    for (long i = 0; i < n; ++i) {
        x = x * 1664525u + 1013904223u;
        h[i] = (int)(((unsigned long long)x * (unsigned long long)V) >> 32);
    }
    CK(hipMemcpy(col, h.data(), n * 4, hipMemcpyHostToDevice));
    for (long i = 0; i < n; ++i) {   // a random permutation-like index into the staging rows
        x = x * 1664525u + 1013904223u;
        h[i] = (int)(((unsigned long long)x * (unsigned long long)n) >> 32);
    }
    CK(hipMemcpy(perm, h.data(), n * 4, hipMemcpyHostToDevice));
    const int blocks = 256 * 8;
    const char *names[] = {"sel", "rw32", "rw64", "app", "atom", "gath", "w64"};
    const char *want = argv[1];
    if (!strcmp(want, "all") || !strcmp(want, "atom8")) {
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        atom8<<<blocks, 256>>>(col, n, sel, dst);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        for (int i = 0; i < reps; ++i) atom8<<<blocks, 256>>>(col, n, sel, dst);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("%-5s E=%ld V=%ld k=%d: %.3f ms  (%.1f ps per edge)\n", "atom8", n, V, K, ms / reps,
               ms / reps * 1e9 / n);
        fflush(stdout);
    }
    for (int v = 0; v <= W64; ++v) {
        if (strcmp(want, "all") && strcmp(want, names[v])) continue;
        float ms = 0.f;
        switch (v) {
        case SEL: ms = launch<SEL>(blocks, col, n, sel, dst, stage, perm, out, reps); break;
        case RW32: ms = launch<RW32>(blocks, col, n, sel, dst, stage, perm, out, reps); break;
        case RW64: ms = launch<RW64>(blocks, col, n, sel, dst, stage, perm, out, reps); break;
        case APP: ms = launch<APP>(blocks, col, n, sel, dst, stage, perm, out, reps); break;
        case ATOM: ms = launch<ATOM>(blocks, col, n, sel, dst, stage, perm, out, reps); break;
        case GATH: ms = launch<GATH>(blocks, col, n, sel, dst, stage, perm, out, reps); break;
        case W64: ms = launch<W64>(blocks, col, n, sel, dst, stage, perm, out, reps); break;
        }
        printf("%-5s E=%ld V=%ld k=%d: %.3f ms  (%.1f ps per edge)\n", names[v], n, V, K, ms,
               ms * 1e9 / n);
        fflush(stdout);
    }
    return 0;
}
