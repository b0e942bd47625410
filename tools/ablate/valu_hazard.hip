// valu_hazard.hip -- isolates the wrong results of the TILE "VALU row-address
// shift" variants (DESIGN.md §4 TILE, tools/exp_tile_vshift2_variant.py modes
// alate / anop).  Development tool, not product code.
//
// Each wave runs the instruction sequence of one record group of
// tile_groups2 in a loop, with wave-uniform synthetic records, and checks the
// LDS byte address the sequence computes (no LDS access is made):
//   exec <- half mask (or all lanes)
//   [A] v_lshrrev_b32 a_j, 14, g_j          (VALU row-address shift, record SGPR)
//   s_set_gpr_idx_on s80, gpr_idx(SRC0); v_bfe_u32 t_j, v48, off_j, 8 (x4, idx between)
//   s_set_gpr_idx_off
//   [B] v_lshrrev_b32 a_j, 14, g_j          (the "alate" placement)
//   v_lshl_add_u32 t_j, t_j, 2, a_j          (address = selector * 4 + row)
// Variants (argv[1]):
//   0 shipped form: row address by s_lshr_b32 (SALU), read as an SGPR operand
//   1 "addr": VALU shift at [A]           2 "alate": VALU shift at [B]
//   3 "alate" with full exec               4 [B] without any gpr-index section
//   5 [B] with the shifts under full exec, the section and the adds under the half
//   6 [B] with s_nop 4 between the shifts and the adds
//   7 [B] reading the shifted value as SRC1 (v_add_u32) instead of SRC2
// Output: wrong lane-results per variant (0 = correct), and per lane half.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

typedef unsigned sel16_t __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint32_t rec_of(uint32_t it, uint32_t j, uint32_t wv)
{
    uint32_t x = (it * 2654435761u) ^ (j * 0x9E3779B9u) ^ (wv * 0x85EBCA6Bu);
    x ^= x >> 13; x *= 0xC2B2AE35u; x ^= x >> 16;
    const uint32_t word = x & 15, b = (x >> 4) & 3, row = (x >> 6) & 0x3ffffu;
    return (word << 2) | b | (row << 14);
}

template <int V>
__global__ __launch_bounds__(1024) void probe(int iters, unsigned *__restrict__ bad)
{
    const int lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(blockIdx.x * 16 + (threadIdx.x >> 6));
    sel16_t selv;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        uint32_t w = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) w |= (uint32_t)((j * 4 + b + lane * 7) & 0xff) << (8 * b);
        selv[j] = w;
    }
    const uint64_t lo = 0x00000000ffffffffull, hi = 0xffffffff00000000ull;
    unsigned nbad0 = 0, nbad1 = 0;
    for (int it = 0; it < iters; ++it) {
        uint32_t g[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) g[j] = __builtin_amdgcn_readfirstlane(rec_of(it, j, wv));
        const uint32_t half = __builtin_amdgcn_readfirstlane((it ^ wv) & 1);
        const uint64_t hm = V == 3 ? ~0ull : (half ? hi : lo);
        uint32_t t0, t1, t2, t3, a0, a1, a2, a3;
        uint64_t ex;
#define SEC                                                                         \
        "s_lshr_b32 s80, %[g0], 2\n\t" "s_lshl_b32 s81, %[g0], 3\n\t"            \
        "s_lshr_b32 s83, %[g1], 2\n\t" "s_lshl_b32 s84, %[g1], 3\n\t"            \
        "s_lshr_b32 s86, %[g2], 2\n\t" "s_lshl_b32 s87, %[g2], 3\n\t"            \
        "s_lshr_b32 s89, %[g3], 2\n\t" "s_lshl_b32 s90, %[g3], 3\n\t"            \
        "s_set_gpr_idx_on s80, gpr_idx(SRC0)\n\t"                                  \
        "v_bfe_u32 %[t0], v48, s81, 8\n\t" "s_set_gpr_idx_idx s83\n\t"             \
        "v_bfe_u32 %[t1], v48, s84, 8\n\t" "s_set_gpr_idx_idx s86\n\t"             \
        "v_bfe_u32 %[t2], v48, s87, 8\n\t" "s_set_gpr_idx_idx s89\n\t"             \
        "v_bfe_u32 %[t3], v48, s90, 8\n\t" "s_set_gpr_idx_off\n\t"
#define SEC_PLAIN                                                                   \
        "s_lshl_b32 s81, %[g0], 3\n\t" "s_lshl_b32 s84, %[g1], 3\n\t"            \
        "s_lshl_b32 s87, %[g2], 3\n\t" "s_lshl_b32 s90, %[g3], 3\n\t"            \
        "v_bfe_u32 %[t0], v48, s81, 8\n\t" "v_bfe_u32 %[t1], v48, s84, 8\n\t"     \
        "v_bfe_u32 %[t2], v48, s87, 8\n\t" "v_bfe_u32 %[t3], v48, s90, 8\n\t"
#define VSH                                                                         \
        "v_lshrrev_b32 %[a0], 14, %[g0]\n\t" "v_lshrrev_b32 %[a1], 14, %[g1]\n\t"  \
        "v_lshrrev_b32 %[a2], 14, %[g2]\n\t" "v_lshrrev_b32 %[a3], 14, %[g3]\n\t"
#define ADDS                                                                        \
        "v_lshl_add_u32 %[t0], %[t0], 2, %[a0]\n\t" "v_lshl_add_u32 %[t1], %[t1], 2, %[a1]\n\t" \
        "v_lshl_add_u32 %[t2], %[t2], 2, %[a2]\n\t" "v_lshl_add_u32 %[t3], %[t3], 2, %[a3]\n\t"
#define OUTS [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3), [a0] "=&v"(a0), \
             [a1] "=&v"(a1), [a2] "=&v"(a2), [a3] "=&v"(a3), [ex] "=&s"(ex), "+{v[48:63]}"(selv)
#define INS [hm] "s"(hm), [g0] "s"(g[0]), [g1] "s"(g[1]), [g2] "s"(g[2]), [g3] "s"(g[3])
#define CLOB "memory", "scc", "s80", "s81", "s82", "s83", "s84", "s85", "s86", "s87", "s88", \
             "s89", "s90", "s91"
        if constexpr (V == 0) {
            asm volatile("s_mov_b64 %[ex], exec\n\t" "s_mov_b64 exec, %[hm]\n\t" SEC
                         "s_lshr_b32 s82, %[g0], 14\n\t" "s_lshr_b32 s85, %[g1], 14\n\t"
                         "s_lshr_b32 s88, %[g2], 14\n\t" "s_lshr_b32 s91, %[g3], 14\n\t"
                         "v_mov_b32 %[a0], 0\n\t" "v_mov_b32 %[a1], 0\n\t"
                         "v_mov_b32 %[a2], 0\n\t" "v_mov_b32 %[a3], 0\n\t"
                         "v_lshl_add_u32 %[t0], %[t0], 2, s82\n\t" "v_lshl_add_u32 %[t1], %[t1], 2, s85\n\t"
                         "v_lshl_add_u32 %[t2], %[t2], 2, s88\n\t" "v_lshl_add_u32 %[t3], %[t3], 2, s91\n\t"
                         "s_mov_b64 exec, %[ex]\n\t" : OUTS : INS : CLOB);
        } else if constexpr (V == 1) {
            asm volatile("s_mov_b64 %[ex], exec\n\t" "s_mov_b64 exec, %[hm]\n\t" VSH SEC ADDS
                         "s_mov_b64 exec, %[ex]\n\t" : OUTS : INS : CLOB);
        } else if constexpr (V == 2 || V == 3) {
            asm volatile("s_mov_b64 %[ex], exec\n\t" "s_mov_b64 exec, %[hm]\n\t" SEC VSH ADDS
                         "s_mov_b64 exec, %[ex]\n\t" : OUTS : INS : CLOB);
        } else if constexpr (V == 4) {
            asm volatile("s_mov_b64 %[ex], exec\n\t" "s_mov_b64 exec, %[hm]\n\t" SEC_PLAIN VSH ADDS
                         "s_mov_b64 exec, %[ex]\n\t" : OUTS : INS : CLOB);
        } else if constexpr (V == 5) {
            asm volatile("s_mov_b64 %[ex], exec\n\t" VSH "s_mov_b64 exec, %[hm]\n\t" SEC ADDS
                         "s_mov_b64 exec, %[ex]\n\t" : OUTS : INS : CLOB);
        } else if constexpr (V == 6) {
            asm volatile("s_mov_b64 %[ex], exec\n\t" "s_mov_b64 exec, %[hm]\n\t" SEC VSH
                         "s_nop 4\n\t" ADDS "s_mov_b64 exec, %[ex]\n\t" : OUTS : INS : CLOB);
        } else if constexpr (V == 7) {
            asm volatile("s_mov_b64 %[ex], exec\n\t" "s_mov_b64 exec, %[hm]\n\t" SEC VSH
                         "v_lshlrev_b32 %[t0], 2, %[t0]\n\t" "v_lshlrev_b32 %[t1], 2, %[t1]\n\t"
                         "v_lshlrev_b32 %[t2], 2, %[t2]\n\t" "v_lshlrev_b32 %[t3], 2, %[t3]\n\t"
                         "v_add_u32 %[t0], %[t0], %[a0]\n\t" "v_add_u32 %[t1], %[t1], %[a1]\n\t"
                         "v_add_u32 %[t2], %[t2], %[a2]\n\t" "v_add_u32 %[t3], %[t3], %[a3]\n\t"
                         "s_mov_b64 exec, %[ex]\n\t" : OUTS : INS : CLOB);
        }
        const bool act = V == 3 || (lane >> 5) == (int)half;
        if (act) {
            const uint32_t tt[4] = {t0, t1, t2, t3};
            unsigned wrong = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t w = g[j], word = (w >> 2) & 15, b = w & 3;
                const uint32_t sel = (word * 4 + b + lane * 7) & 0xff;
                wrong += tt[j] != sel * 4 + (w >> 14);
            }
            if (lane < 32) nbad0 += wrong; else nbad1 += wrong;
        }
    }
    atomicAdd(bad + 0, nbad0);
    atomicAdd(bad + 1, nbad1);
}

template <int V>
void run(int iters, int blocks)
{
    unsigned *d, h[2];
    CK(hipMalloc(&d, 8));
    CK(hipMemset(d, 0, 8));
    hipLaunchKernelGGL(probe<V>, dim3(blocks), dim3(1024), 0, 0, iters, d);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h, d, 8, hipMemcpyDeviceToHost));
    const double checks = (double)blocks * 16 * iters * 4 * 32;
    printf("variant %d: wrong %u (half 0) %u (half 1) of %.0f lane-results\n", V, h[0], h[1],
           checks);
    CK(hipFree(d));
}

int main(int argc, char **argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 20000;
    const int blocks = argc > 2 ? atoi(argv[2]) : 256;
    run<0>(iters, blocks);
    run<1>(iters, blocks);
    run<2>(iters, blocks);
    run<3>(iters, blocks);
    run<4>(iters, blocks);
    run<5>(iters, blocks);
    run<6>(iters, blocks);
    run<7>(iters, blocks);
    return 0;
}
