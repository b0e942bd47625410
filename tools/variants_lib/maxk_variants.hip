// maxk_variants.hip -- the ABLATION build (tools/variants_lib/libmaxk_variants.so):
// the product sources plus the kernels that were built, tested bit-exact and
// measured slower on every BASELINE shape, moved out of the product library in
// round 5.  DESIGN.md §4 (config 5: register-accumulator
// forward and backward phase 1, bank-ordered backward phase 1) and §5
// (BINNED: propagation blocking) hold their measurements.  Declarations:
// maxk_variants.h.  Not loaded by the product path (spgemm_new_amd/_lib.py);
// tests/test_variants.py runs them against the oracle and the product kernels.
#include "../../spgemm_new_amd/csrc/maxk_spgemm.hip"
#include "maxk_variants.h"

namespace {

// ---------------------------------------------------------------------------
// Register-accumulator form of the fused R = 8 forward (h = 256, k <= 32):
// the destination row's 8 x 256 sums live in registers, lane l owning columns
// 4l .. 4l+3 of every relation (8 x f4 = 32 VGPRs), so the per-edge LDS
// read-modify-write of the relation-vector kernel (ds_read_b128 + ds_write_b128,
// 17 LDS cycles per edge plus bank conflicts) goes away.  An edge reaches a
// lane's columns as a GATHER, not a scatter: the source's CBSR row is kept
// column-sorted (cbsr_colmask_kernel), with a 256-bit column bitmask and the
// number of selected columns below each 32-column word; lane l tests its four
// bits, their ranks in the row are base + popcount of the lower bits, and
// ds_bpermute fetches the values from the lanes holding the (sorted) CBSR row;
// a column the source did not select reads a lane of the zero half.  Then
// 2 x 8 v_pk_fma_f32 with the edge's 8 values (wave-uniform, scalar loads).
// Per element the FMAs happen in edge order (fma(x, v_q, acc); an unselected
// column adds 0 * v_q), as in the relation-vector kernel at k = 32, which then
// gives the same bits (at k < 32 that kernel sums per-edge-slot row copies).
// ---------------------------------------------------------------------------
typedef float f2 __attribute__((ext_vector_type(2)));

// Column-sorted CBSR + column bitmask records: one wave per row; entry j's rank
// = the number of the row's distinct columns below it; duplicate columns (not a
// valid CBSR, handled anyway) are summed in entry order into one rank.  mrec[r*8 + w]
// = {bits of columns 32w .. 32w+31, selected columns below 32w}.
template <int K>
__global__ __launch_bounds__(kBlock) void cbsr_colmask_kernel(const float *__restrict__ data,
                                                              const uint8_t *__restrict__ sel,
                                                              int num_rows,
                                                              float *__restrict__ sdata,
                                                              uint2 *__restrict__ mrec)
{
    const int lane = lane_id();
    const int64_t nwaves = (int64_t)gridDim.x * kWavesPerBlock;
    for (int64_t r = (int64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave; r < num_rows;
         r += nwaves) {
        const bool on = lane < K;
        const int c = on ? (int)sel[r * K + lane] : 1024;
        const float d = on ? data[r * K + lane] : 0.f;
        int rank = 0;
        float dsum = 0.f;
        bool first = on;
#pragma unroll
        for (int i = 0; i < K; ++i) {
            const int ci = __shfl(c, i);
            const float di = __shfl(d, i);
            rank += ci < c;
            if (ci == c) {
                dsum += di;
                if (i < lane) first = false;
            }
        }
        if (first) sdata[r * K + rank] = dsum;
        const int myw = c >> 5;
        uint32_t mw = 0, pw = 0;
#pragma unroll
        for (int w = 0; w < 8; ++w) {
            uint32_t b = (on && myw == w) ? (1u << (c & 31)) : 0u;
            b |= __shfl_xor(b, 1);
            b |= __shfl_xor(b, 2);
            b |= __shfl_xor(b, 4);
            b |= __shfl_xor(b, 8);
            b |= __shfl_xor(b, 16);
            b |= __shfl_xor(b, 32);
            const uint32_t below = (uint32_t)__builtin_popcountll(__ballot(first && myw < w));
            if (lane == w) {
                mw = b;
                pw = below;
            }
        }
        if (lane < 8) mrec[r * 8 + lane] = make_uint2(mw, pw);
    }
}

// One round of U edges of a destination row (FULL: all U exist).  Per edge:
// the bitmask word of the lane's columns and the rank base (one 8-B load per
// lane from the source's 64-B record), the source's sorted CBSR row in lanes
// 0 .. K-1 (lanes K .. 63 hold zeros), the 8 values by scalar loads.
template <int K, int U, bool FULL>
__device__ __forceinline__ void rel8g_round(int my_c, int ebase, int s0, int n,
                                            const float *__restrict__ val,
                                            const float *__restrict__ sdata,
                                            const uint2 *__restrict__ mrec, f2 (&a)[8][2])
{
    const int lane = lane_id();
    const int wd = lane >> 3;
    const uint32_t sh = (uint32_t)(lane & 7) * 4u;
    const uint32_t low = (1u << sh) - 1u;
    uint2 mr[U];
    float dv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if (!FULL && s0 + u >= n) break;
        const int c = __builtin_amdgcn_readlane(my_c, s0 + u);
        const uint2 *mp = mrec + (size_t)c * 8;      // wave-uniform row pointers
        const float *dp = sdata + (size_t)c * K;
        mr[u] = mp[wd];
        const float x = dp[lane & (K - 1)];
        dv[u] = lane < K ? x : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if (!FULL && s0 + u >= n) break;
        // the edge's 8 values: a uniform address, so scalar loads and SGPR operands
        const int eu = __builtin_amdgcn_readfirstlane(ebase + s0 + u);
        const float *vr = val + (size_t)eu * 8;
        const uint32_t nib = (mr[u].x >> sh) & 15u;
        const uint32_t base = (uint32_t)__builtin_popcount(mr[u].x & low) + mr[u].y;
        // rank of column 4l + i among the source's selected columns (x4: a byte
        // address for ds_bpermute), or lane 63 (a zero) when column 4l + i is not
        // selected: bfi(-hit, rank * 4, 252)
        uint32_t ad[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t p = (uint32_t)__builtin_popcount(nib & ((1u << i) - 1u)) + base;
            const uint32_t hit = (uint32_t)(((int32_t)(nib << (31 - i))) >> 31);
            ad[i] = ((p << 2) & hit) | (((uint32_t)(kWave - 1) << 2) & ~hit);
        }
        const int xb = __float_as_int(dv[u]);
        f2 x01, x23;
        x01.x = __int_as_float(__builtin_amdgcn_ds_bpermute((int)ad[0], xb));
        x01.y = __int_as_float(__builtin_amdgcn_ds_bpermute((int)ad[1], xb));
        x23.x = __int_as_float(__builtin_amdgcn_ds_bpermute((int)ad[2], xb));
        x23.y = __int_as_float(__builtin_amdgcn_ds_bpermute((int)ad[3], xb));
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const float v = vr[q];
            const f2 vv = {v, v};
            a[q][0] = __builtin_elementwise_fma(x01, vv, a[q][0]);
            a[q][1] = __builtin_elementwise_fma(x23, vv, a[q][1]);
        }
    }
}

template <int K>
__device__ __forceinline__ void rel8g_edges(int e0, int e1, const int32_t *__restrict__ idx,
                                            const float *__restrict__ val,
                                            const float *__restrict__ sdata,
                                            const uint2 *__restrict__ mrec, f2 (&a)[8][2])
{
    constexpr int U = 8;
    const int lane = lane_id();
    for (int base = e0; base < e1; base += kWave) {
        const int n = __builtin_amdgcn_readfirstlane((e1 - base) < kWave ? (e1 - base) : kWave);
        const int my_c = lane < n ? __builtin_nontemporal_load(idx + base + lane) : 0;
        int s0 = 0;
        for (; s0 + U <= n; s0 += U) rel8g_round<K, U, true>(my_c, base, s0, n, val, sdata, mrec, a);
        if (s0 < n) rel8g_round<K, U, false>(my_c, base, s0, n, val, sdata, mrec, a);
    }
}

__device__ __forceinline__ void rel8g_store(f2 (&a)[8][2], float *__restrict__ dst, size_t rel_stride)
{
    const int lane = lane_id();
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const f4 s = {a[q][0].x, a[q][0].y, a[q][1].x, a[q][1].y};
        *reinterpret_cast<f4 *>(dst + q * rel_stride + 4 * lane) = s;
        a[q][0] = f2{0.f, 0.f};
        a[q][1] = f2{0.f, 0.f};
    }
}

template <int K>
__global__ __launch_bounds__(kBlock) void fwd_rel8_gather_kernel(
    const int2 *__restrict__ sched, int64_t num_panels, const int32_t *__restrict__ indptr,
    const int32_t *__restrict__ idx, const float *__restrict__ val,
    const float *__restrict__ sdata, const uint2 *__restrict__ mrec, int num_rows,
    float *__restrict__ out, float *__restrict__ carry, int32_t *__restrict__ carry_row)
{
    const int64_t w = (int64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave;
    if (w >= num_panels) return;
    f2 a[8][2];
#pragma unroll
    for (int q = 0; q < 8; ++q) a[q][0] = a[q][1] = f2{0.f, 0.f};
    const size_t rs = (size_t)num_rows * kMaxDim;
    const int2 s0 = sched[w], s1 = sched[w + 1];
    const int i0 = s0.x, j0 = s0.y, i1 = s1.x, j1 = s1.y;
    int e = j0;
    for (int r = i0; r < i1; ++r) {
        const int re = indptr[r + 1];
        if (e < re) rel8g_edges<K>(e, re, idx, val, sdata, mrec, a);
        rel8g_store(a, out + (size_t)r * kMaxDim, rs);
        e = re;
    }
    int has_carry = 0;
    if (i1 < num_rows) {
        const int eb = e > indptr[i1] ? e : indptr[i1];
        if (eb < j1) {
            rel8g_edges<K>(eb, j1, idx, val, sdata, mrec, a);
            has_carry = 1;
        }
    }
    if (has_carry) {
        rel8g_store(a, carry + (size_t)w * 8 * kMaxDim, kMaxDim);
        if (lane_id() == 0) carry_row[w] = i1;
    } else if (lane_id() == 0) {
        carry_row[w] = -1;
    }
}

// R = 8, k = 32 with bank-ordered selectors (round 4): one edge per
// wave-instruction, lane 2p + q reads quad q of the edge's p-th (bank-ordered)
// column -- a ds_read_b128 16-lane group then covers 8 columns x both quads,
// conflict-free iff the 8 columns differ mod 8, which the bank order (mode 2,
// maxk_cbsr_bank_order) arranges wherever the row allows (a conflict model:
// 11.9 -> 7.7 LDS cycles per edge against the 8-lanes-per-edge layout above,
// whose 16-lane groups mix four destinations' columns).  Lane 2p + 1 hands its
// quad to lane 2p (DPP), which adds the 8 relations in order -- the same FMAs
// as bwd_multi_edges, so the same bits -- and pushes the product to the lane of
// the column's ORIGINAL entry (ds_permute; sp = bank-ordered selector |
// original entry << 8), so lanes 0..31 store the row as one contiguous line.
template <int PM>
__device__ __forceinline__ void bwd_multi_edges_banked(int e0, int e1,
                                                       const int32_t *__restrict__ idx,
                                                       const float *__restrict__ val,
                                                       const int32_t *__restrict__ csc_pos,
                                                       const uint16_t *__restrict__ sp,
                                                       const char *gs, float *__restrict__ P)
{
    constexpr bool CSRP = PM == kPmEdge;
    constexpr int K = 32, KP = 32, U = 8;
    const int lane = lane_id();
    const int ent = lane >> 1, q = lane & 1;
    for (int base = e0; base < e1; base += kWave) {
        const int n = __builtin_amdgcn_readfirstlane((e1 - base) < kWave ? (e1 - base) : kWave);
        int my_c = 0, my_p = 0;
        f4 v0 = f4{0.f, 0.f, 0.f, 0.f}, v1 = v0;
        if (lane < n) {
            my_c = __builtin_nontemporal_load(idx + base + lane);
            my_p = CSRP ? base + lane : __builtin_nontemporal_load(csc_pos + base + lane);
            const f4 *vp = reinterpret_cast<const f4 *>(val + (size_t)(base + lane) * 8);
            v0 = __builtin_nontemporal_load(vp);
            v1 = __builtin_nontemporal_load(vp + 1);
        }
        // straight-line per group of U edges (the tail clamped to the last edge,
        // its stores skipped): U selector loads, U LDS reads, then per edge its 8
        // values by readlane (scalar loads would share the LDS reads' counter)
        // the next group's selectors are loaded while this group computes (one
        // gather round trip per U edges would otherwise stall the wave)
        uint32_t wn[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int c = __builtin_amdgcn_readlane(my_c, u < n ? u : n - 1);
            wn[u] = sp[(size_t)c * K + ent];
        }
        for (int s0 = 0; s0 < n; s0 += U) {
            uint32_t w[U];
            f4 g[U];
#pragma unroll
            for (int u = 0; u < U; ++u) w[u] = wn[u];
            if (s0 + U < n) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int t = s0 + U + u;
                    const int c = __builtin_amdgcn_readlane(my_c, t < n ? t : n - 1);
                    wn[u] = sp[(size_t)c * K + ent];
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
                g[u] = *reinterpret_cast<const f4 *>(gs + RelLds<8>::off(w[u] & 0xffu, q));
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int uu = s0 + u < n ? s0 + u : n - 1;
                // quad 1 of the column from the odd lane (DPP quad_perm [1,0,3,2])
                f4 h;
                h.x = __uint_as_float(dpp_xor1(__float_as_uint(g[u].x)));
                h.y = __uint_as_float(dpp_xor1(__float_as_uint(g[u].y)));
                h.z = __uint_as_float(dpp_xor1(__float_as_uint(g[u].z)));
                h.w = __uint_as_float(dpp_xor1(__float_as_uint(g[u].w)));
                const auto rl = [uu](float x) {
                    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), uu));
                };
                float acc = 0.f;
                acc = fmaf(rl(v0.x), g[u].x, acc);
                acc = fmaf(rl(v0.y), g[u].y, acc);
                acc = fmaf(rl(v0.z), g[u].z, acc);
                acc = fmaf(rl(v0.w), g[u].w, acc);
                acc = fmaf(rl(v1.x), h.x, acc);
                acc = fmaf(rl(v1.y), h.y, acc);
                acc = fmaf(rl(v1.z), h.z, acc);
                acc = fmaf(rl(v1.w), h.w, acc);
                // each even lane pushes its product to the lane of the column's
                // original entry (odd lanes to the unused upper half), so lanes
                // 0..31 store the row as one contiguous 128-B line
                const int dst = q == 0 ? (int)(w[u] >> 8) : 32 + ent;
                const float o = __int_as_float(__builtin_amdgcn_ds_permute(dst << 2, __float_as_int(acc)));
                const int p = __builtin_amdgcn_readlane(my_p, uu);
                if (lane < 32 && s0 + u < n)
                    __builtin_nontemporal_store(o, P + (size_t)p * KP + lane);
            }
        }
    }
}

// the multi-relation STAGED phase 1 over bank-ordered selectors (R = 8, k = 32)
template <int PM>
__global__ __launch_bounds__(kBlock) void bwd_multi_stage_banked_kernel(
    const int2 *__restrict__ sched, int64_t num_panels, const int32_t *__restrict__ indptr,
    const int32_t *__restrict__ idx, const float *__restrict__ val,
    const float *__restrict__ grad, int64_t plane, const int32_t *__restrict__ csc_pos,
    int num_rows, int dim, float *__restrict__ P, const uint16_t *__restrict__ sp)
{
    extern __shared__ __attribute__((aligned(16))) float lds[];
    char *gs = reinterpret_cast<char *>(lds + (threadIdx.x / kWave) * (kMaxDim * 8));
    const int64_t w = (int64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave;
    if (w >= num_panels) return;
    const int2 a = sched[w], b = sched[w + 1];
    const int i0 = a.x, j0 = a.y, i1 = b.x, j1 = b.y;
    const int rlast = i1 < num_rows ? i1 : num_rows - 1;
    for (int r = i0; r <= rlast; ++r) {
        const int rb = indptr[r], re = indptr[r + 1];
        const int eb = rb > j0 ? rb : j0;
        const int ee = re < j1 ? re : j1;
        if (eb >= ee) continue;
        stage_rel_rows<8>(gs, grad, plane, r, dim);
        bwd_multi_edges_banked<PM>(eb, ee, idx, val, csc_pos, sp, gs, P);
    }
}

// Register form of the multi-relation STAGED phase 1 for R = 8, h = 256, k <= 32
// (proteins): the source row's 8 gradient rows stay in registers, lane l holding
// columns 4l .. 4l+3 of every relation (8 x f4), loaded once per (row, panel).
// Per edge the lane first folds the relations for ALL of its columns,
// t = sum_q val[e, q] * G_q[r, 4l .. 4l+3] (8 v_pk_fma_f32 pairs, relation order,
// so the same FMAs as the LDS kernel's per-column sum), then entry j (lane j <
// k) fetches t at its selected column c_j by ds_bpermute from lane c_j / 4 and
// keeps component c_j % 4.  No LDS array is touched: the LDS kernel's 2 x
// ds_read_b128 per entry at random columns (bank conflicts ~47 % of its LDS
// cycles) become 4 bpermutes per edge.  P rows as the LDS kernel writes them.
template <int K, int PM>
__global__ __launch_bounds__(kBlock) void bwd_rel8_gather_stage_kernel(
    const int2 *__restrict__ sched, int64_t num_panels, const int32_t *__restrict__ indptr,
    const int32_t *__restrict__ idx, const float *__restrict__ val,
    const float *__restrict__ grad, int64_t plane, const uint8_t *__restrict__ sel,
    const int32_t *__restrict__ csc_pos, int num_rows, float *__restrict__ P)
{
    constexpr bool CSRP = PM == kPmEdge;
    constexpr int KP = PM == kPmCsc ? PRow<K>::KP : K;
    constexpr int U = 4;
    const int64_t w = (int64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave;
    if (w >= num_panels) return;
    const int lane = lane_id();
    const int2 a = sched[w], b = sched[w + 1];
    const int i0 = a.x, j0 = a.y, i1 = b.x, j1 = b.y;
    const int rlast = i1 < num_rows ? i1 : num_rows - 1;
    for (int r = i0; r <= rlast; ++r) {
        const int rb = indptr[r], re = indptr[r + 1];
        const int eb = rb > j0 ? rb : j0;
        const int ee = re < j1 ? re : j1;
        if (eb >= ee) continue;
        f2 g[8][2];
        const float *gr = grad + (size_t)r * kMaxDim + 4 * lane;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const f4 v = *reinterpret_cast<const f4 *>(gr + (size_t)q * plane);
            g[q][0] = f2{v.x, v.y};
            g[q][1] = f2{v.z, v.w};
        }
        for (int base = eb; base < ee; base += kWave) {
            const int n = __builtin_amdgcn_readfirstlane((ee - base) < kWave ? (ee - base) : kWave);
            int my_c = 0, my_p = 0;
            if (lane < n) {
                my_c = __builtin_nontemporal_load(idx + base + lane);
                my_p = CSRP ? base + lane : __builtin_nontemporal_load(csc_pos + base + lane);
            }
            for (int s0 = 0; s0 < n; s0 += U) {
                uint32_t cb[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int c = __builtin_amdgcn_readlane(my_c, s0 + u < n ? s0 + u : s0);
                    const uint8_t *sp = sel + (size_t)c * K;
                    cb[u] = sp[lane & (K - 1)];
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    if (s0 + u >= n) break;
                    const int eu = __builtin_amdgcn_readfirstlane(base + s0 + u);
                    const float *vr = val + (size_t)eu * 8;
                    f2 t0 = {0.f, 0.f}, t1 = {0.f, 0.f};
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        const float v = vr[q];
                        const f2 vv = {v, v};
                        t0 = __builtin_elementwise_fma(vv, g[q][0], t0);
                        t1 = __builtin_elementwise_fma(vv, g[q][1], t1);
                    }
                    const int src = (int)(cb[u] >> 2) << 2;
                    const float x = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(t0.x)));
                    const float y = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(t0.y)));
                    const float z = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(t1.x)));
                    const float ww = __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(t1.y)));
                    const uint32_t cc = cb[u] & 3u;
                    const float lo = (cc & 1u) ? y : x, hi = (cc & 1u) ? ww : z;
                    const float o = (cc & 2u) ? hi : lo;
                    const int p = __builtin_amdgcn_readlane(my_p, s0 + u);
                    if (lane < K) __builtin_nontemporal_store(o, P + (size_t)p * KP + lane);
                    else if (KP > K && lane < KP) __builtin_nontemporal_store(0.f, P + (size_t)p * KP + lane);
                }
            }
        }
    }
}

// BINNED phase 2 (propagation blocking): destination bin b = columns
// [b*255, b*255 + 255) is summed by one wave in LDS (255 x K floats).  Its
// slots P[bin_ptr[b] .. bin_ptr[b+1]) come in windows of 64 whose destinations
// are distinct (maxk_bin_plan_build packs them so), so one lane per slot adds
// its row into the destination's LDS row with a plain read-add-write: no two
// lanes of an instruction touch one row, and the wave's LDS operations are in
// order.  Padding slots carry destination 0xFF.  U windows of rows are loaded
// before their adds.  Summation order per destination = slot order, fixed by
// the plan: deterministic.
constexpr int kBinDests = MAXK_BIN_DESTS;

template <int K>
__global__ __launch_bounds__(kWave) void bwd_bin_sum_kernel(const int32_t *__restrict__ bin_ptr,
                                                           int num_bins,
                                                           const uint8_t *__restrict__ bin_dst,
                                                           const float *__restrict__ P,
                                                           int num_cols, float *__restrict__ dxs)
{
    constexpr int Q = K / 4;                       // float4 per row
    constexpr int QS = Q + 1;                      // LDS row stride in float4: a pad quad
                                                   // spreads a window's rows over the banks
    constexpr int U = K == 32 ? 2 : K == 16 ? 4 : 6;   // windows per register batch
    extern __shared__ __attribute__((aligned(16))) float lds[];   // one wave per block
    const int lane = lane_id();
    f4 *acc = reinterpret_cast<f4 *>(lds);
    for (int i = lane; i < kBinDests * QS; i += kWave) acc[i] = f4{0.f, 0.f, 0.f, 0.f};
    const int64_t b = blockIdx.x;
    if (b >= num_bins) return;
    const int q0 = bin_ptr[b];
    const int nw = (bin_ptr[b + 1] - q0) / kWave;  // windows of 64 slots
    if (nw > 0) {
    const f4 *P4 = reinterpret_cast<const f4 *>(P) + (size_t)q0 * Q;
    const uint8_t *D = bin_dst + q0;
    // two batches of U windows in registers: batch i + 1 is loaded before
    // batch i is added, so a wave always has U windows of loads in flight;
    // batches past the end reload the last window (no branch around loads)
    const int last = nw - 1;
    uint32_t da[U], db[U];
    f4 va[U][Q], vb[U][Q];
    auto load = [&](uint32_t (&d)[U], f4 (&v)[U][Q], int w0) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int w = w0 + u < last ? w0 + u : last;
            d[u] = __builtin_nontemporal_load(D + w * kWave + lane);
#pragma unroll
            for (int j = 0; j < Q; ++j)
                v[u][j] = __builtin_nontemporal_load(P4 + (size_t)(w * kWave + lane) * Q + j);
        }
    };
    auto add = [&](const uint32_t (&d)[U], const f4 (&v)[U][Q], int w0) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (w0 + u < nw && d[u] != 0xFFu) {
                f4 *a = acc + d[u] * QS;
#pragma unroll
                for (int j = 0; j < Q; ++j) {
                    f4 t = a[j];
                    t.x += v[u][j].x; t.y += v[u][j].y; t.z += v[u][j].z; t.w += v[u][j].w;
                    a[j] = t;
                }
            }
        }
    };
    load(da, va, 0);
    for (int w0 = 0; w0 < nw; w0 += 2 * U) {
        load(db, vb, w0 + U);
        add(da, va, w0);
        if (w0 + U >= nw) break;
        load(da, va, w0 + 2 * U);
        add(db, vb, w0 + U);
    }
    }
    const int64_t c0 = b * kBinDests;
    const int rows = (int)((num_cols - c0) < kBinDests ? (num_cols - c0) : kBinDests);
    f4 *out = reinterpret_cast<f4 *>(dxs + c0 * K);
    for (int i = lane; i < rows * Q; i += kWave) out[i] = acc[(i / Q) * QS + i % Q];
}

// the register-accumulator R = 8 forward (h = 256) and its CBSR preparation, k <= 32
template <int K>
struct CbsrColmask {
    static int run(const float *data, const uint8_t *sel, int V, float *sdata, uint2 *mrec,
                   hipStream_t st)
    {
        if constexpr (K == 0 || K > 32) {
            return MAXK_E_DIM;
        } else {
            const int64_t blocks = ceil_div(V, kWavesPerBlock);
            hipLaunchKernelGGL(cbsr_colmask_kernel<K>, dim3((unsigned)(blocks < 8192 ? blocks : 8192)),
                               dim3(kBlock), 0, st, data, sel, V, sdata, mrec);
            return launch_status();
        }
    }
};

template <int K>
struct FwdRel8Gather {
    static int run(const int32_t *sched, int64_t P, const int32_t *indptr, const int32_t *idx,
                   const float *val, const float *sdata, const uint2 *mrec, int V, float *out,
                   float *carry, int32_t *carry_row, hipStream_t st)
    {
        if constexpr (K == 0 || K > 32) {
            return MAXK_E_DIM;
        } else {
            const int64_t blocks = ceil_div(P, kWavesPerBlock);
            hipLaunchKernelGGL(fwd_rel8_gather_kernel<K>, dim3((unsigned)blocks), dim3(kBlock), 0, st,
                               reinterpret_cast<const int2 *>(sched), P, indptr, idx, val, sdata,
                               mrec, V, out, carry, carry_row);
            int rc = launch_status();
            if (rc) return rc;
            hipLaunchKernelGGL(carry_fixup_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, st, P,
                               carry, carry_row, out, kMaxDim, kMaxDim, 8, (size_t)V * kMaxDim);
            return launch_status();
        }
    }
};

// register form of the multi-relation phase 1 (R = 8, h = 256, k <= 32)
template <int K>
struct BwdRel8Gather {
    static int run(bool edge_order, const int32_t *sched, int64_t P, const int32_t *indptr,
                   const int32_t *idx, const float *val, const float *grad, int64_t plane,
                   const uint8_t *sel, const int32_t *csc_pos, int V, float *Pbuf, hipStream_t st)
    {
        if constexpr (K != 8 && K != 16 && K != 32) {
            return MAXK_E_DIM;
        } else {
            const int2 *sc = reinterpret_cast<const int2 *>(sched);
            const unsigned blocks = (unsigned)ceil_div(P, kWavesPerBlock);
            if (edge_order)
                hipLaunchKernelGGL((bwd_rel8_gather_stage_kernel<K, kPmEdge>), dim3(blocks),
                                   dim3(kBlock), 0, st, sc, P, indptr, idx, val, grad, plane, sel,
                                   csc_pos, V, Pbuf);
            else
                hipLaunchKernelGGL((bwd_rel8_gather_stage_kernel<K, kPmCsc>), dim3(blocks),
                                   dim3(kBlock), 0, st, sc, P, indptr, idx, val, grad, plane, sel,
                                   csc_pos, V, Pbuf);
            return launch_status();
        }
    }
};

// BINNED phase 1: the shared staging kernel with bin positions as write slots
template <int K>
struct BinPhase1 {
    static int run(bool esel, const int32_t *sched, int64_t P, const int32_t *indptr,
                   const int32_t *idx, const float *val, const float *grad, const uint8_t *sel,
                   const int32_t *bin_pos, int V, int dim, int k, float *dxs, float *Pbuf,
                   hipStream_t st)
    {
        if constexpr (K != 8 && K != 16 && K != 32) {
            return MAXK_E_DIM;
        } else {
            const int64_t blocks = ceil_div(P, kWavesPerBlock);
            if (esel)
                hipLaunchKernelGGL((bwd_panel_kernel<K, true, true, kPmBin>), dim3((unsigned)blocks),
                                   dim3(kBlock), row_lds_bytes(), st,
                                   reinterpret_cast<const int2 *>(sched), P, indptr, idx, val,
                                   grad, sel, bin_pos, V, dim, k, dxs, Pbuf);
            else
                hipLaunchKernelGGL((bwd_panel_kernel<K, true, false, kPmBin>),
                                   dim3((unsigned)blocks), dim3(kBlock), row_lds_bytes(), st,
                                   reinterpret_cast<const int2 *>(sched), P, indptr, idx, val,
                                   grad, sel, bin_pos, V, dim, k, dxs, Pbuf);
            return launch_status();
        }
    }
};

}  // namespace

extern "C" {

int maxk_cbsr_bank_order_ex(const float *cbsr_data, const uint8_t *cbsr_sel, int num_rows,
                            int dim_k, int num_rel, float *out_data, uint8_t *out_sel,
                            uint16_t *out_packed, void *stream)
{
    return cbsr_bank_order_impl(cbsr_data, cbsr_sel, num_rows, dim_k, num_rel, out_data, out_sel,
                                out_packed, stream);
}

int maxk_cbsr_colmask(const float *cbsr_data, const uint8_t *cbsr_sel, int num_rows, int dim_k,
                      float *sorted_data, uint32_t *mask_rec, void *stream)
{
    if (dim_k < 4 || dim_k > 32 || (dim_k & (dim_k - 1))) return MAXK_E_DIM;
    if (num_rows < 0 || (num_rows > 0 && (!cbsr_data || !cbsr_sel || !sorted_data || !mask_rec)))
        return MAXK_E_ARG;
    if (reinterpret_cast<uintptr_t>(mask_rec) & 7) return MAXK_E_ARG;
    if (num_rows == 0) return MAXK_OK;
    return dispatch_k<CbsrColmask>(dim_k, cbsr_data, cbsr_sel, num_rows, sorted_data,
                                   reinterpret_cast<uint2 *>(mask_rec), as_stream(stream));
}

int maxk_spgemm_forward_multi_gather(const int32_t *sched, int64_t num_panels,
                                     const int32_t *indptr, const int32_t *indices,
                                     const float *values, int num_rel, const float *sorted_data,
                                     const uint32_t *mask_rec, int num_rows, int dim_origin,
                                     int dim_k, float *out, void *workspace,
                                     size_t workspace_bytes, void *stream)
{
    if (!sched || !indptr || !out || num_panels < 1 || num_rows < 0) return MAXK_E_ARG;
    if (num_rel != 8 || dim_origin != kMaxDim) return MAXK_E_DIM;
    if (dim_k < 4 || dim_k > 32 || (dim_k & (dim_k - 1))) return MAXK_E_DIM;
    if (num_rows == 0) return MAXK_OK;
    if (!indices || !values || !sorted_data || !mask_rec) return MAXK_E_ARG;
    if ((reinterpret_cast<uintptr_t>(mask_rec) & 7) || (reinterpret_cast<uintptr_t>(out) & 15))
        return MAXK_E_ARG;
    if (!workspace ||
        workspace_bytes < maxk_forward_multi_workspace_bytes(num_panels, dim_origin, num_rel))
        return MAXK_E_WORKSPACE;
    float *carry = static_cast<float *>(workspace);
    int32_t *carry_row = reinterpret_cast<int32_t *>(
        static_cast<char *>(workspace) +
        align_up((size_t)num_panels * num_rel * kMaxDim * sizeof(float), 256));
    return dispatch_k<FwdRel8Gather>(dim_k, sched, num_panels, indptr, indices, values, sorted_data,
                                     reinterpret_cast<const uint2 *>(mask_rec), num_rows, out, carry,
                                     carry_row, as_stream(stream));
}

int maxk_sspmm_backward_multi_banked(int algo, const int32_t *sched, int64_t num_panels,
                                     const int32_t *indptr, const int32_t *indices,
                                     const float *values, int num_rel, const float *grad,
                                     const uint16_t *sel_banked, int num_rows, int num_cols,
                                     int64_t num_edges, int dim_origin, int dim_k, float *dxs,
                                     const int32_t *csc_pos, const int32_t *csc_sched,
                                     int64_t csc_num_panels, const int32_t *csc_indptr,
                                     void *workspace, size_t workspace_bytes, void *stream)
{
    if (num_rel != 8 || dim_k != 32) return MAXK_E_DIM;
    if (!sel_banked && num_cols > 0) return MAXK_E_ARG;
    return sspmm_backward_multi_impl(
        algo, num_panels, sched, indptr, indices, values, num_rel, grad, sel_banked, num_rows,
        num_cols, num_edges, dim_origin, dim_k, dxs, csc_pos, csc_sched, csc_num_panels,
        csc_indptr, workspace, workspace_bytes, stream,
        [&](bool edge_order, float *Pbuf, hipStream_t st) {
            const unsigned blocks = (unsigned)ceil_div(num_panels, kWavesPerBlock);
            const size_t lds = (size_t)kWavesPerBlock * kMaxDim * 8 * sizeof(float);
            const int2 *sc = reinterpret_cast<const int2 *>(sched);
            const int64_t plane = (int64_t)num_rows * dim_origin;
            if (edge_order)
                hipLaunchKernelGGL(bwd_multi_stage_banked_kernel<kPmEdge>, dim3(blocks),
                                   dim3(kBlock), lds, st, sc, num_panels, indptr, indices, values,
                                   grad, plane, csc_pos, num_rows, dim_origin, Pbuf, sel_banked);
            else
                hipLaunchKernelGGL(bwd_multi_stage_banked_kernel<kPmCsc>, dim3(blocks),
                                   dim3(kBlock), lds, st, sc, num_panels, indptr, indices, values,
                                   grad, plane, csc_pos, num_rows, dim_origin, Pbuf, sel_banked);
            return launch_status();
        });
}

int maxk_sspmm_backward_multi_gather(int algo, const int32_t *sched, int64_t num_panels,
                                     const int32_t *indptr, const int32_t *indices,
                                     const float *values, int num_rel, const float *grad,
                                     const uint8_t *cbsr_sel, int num_rows, int num_cols,
                                     int64_t num_edges, int dim_origin, int dim_k, float *dxs,
                                     const int32_t *csc_pos, const int32_t *csc_sched,
                                     int64_t csc_num_panels, const int32_t *csc_indptr,
                                     void *workspace, size_t workspace_bytes, void *stream)
{
    if (num_rel != 8 || dim_origin != kMaxDim || dim_k > 32) return MAXK_E_DIM;
    return sspmm_backward_multi_impl(
        algo, num_panels, sched, indptr, indices, values, num_rel, grad, cbsr_sel, num_rows,
        num_cols, num_edges, dim_origin, dim_k, dxs, csc_pos, csc_sched, csc_num_panels,
        csc_indptr, workspace, workspace_bytes, stream,
        [&](bool edge_order, float *Pbuf, hipStream_t st) {
            return dispatch_k<BwdRel8Gather>(dim_k, edge_order, sched, num_panels, indptr, indices,
                                             values, grad, (int64_t)num_rows * dim_origin, cbsr_sel,
                                             csc_pos, num_rows, Pbuf, st);
        });
}

size_t maxk_backward_binned_workspace_bytes(int64_t num_slots, int dim_k)
{
    if (num_slots < 0 || (dim_k != 8 && dim_k != 16 && dim_k != 32)) return 0;
    return align_up((size_t)num_slots * dim_k * sizeof(float), 256);
}

int maxk_sspmm_backward_binned(const int32_t *sched, int64_t num_panels, const int32_t *indptr,
                               const int32_t *indices, const float *values, const float *grad,
                               const uint8_t *sel, int edge_selectors, int num_rows, int num_cols,
                               int64_t num_edges, int dim_origin, int dim_k, float *dxs,
                               const int32_t *bin_pos, const int32_t *bin_ptr,
                               const uint8_t *bin_dst, int num_bins, int64_t num_slots,
                               void *workspace, size_t workspace_bytes, void *stream)
{
    if (!sched || !indptr || !dxs || num_panels < 1 || num_rows < 0 || num_cols < 0 ||
        num_edges < 0 || num_slots < 0)
        return MAXK_E_ARG;
    if (!dims_ok(dim_origin, dim_k)) return MAXK_E_DIM;
    if (dim_k != 8 && dim_k != 16 && dim_k != 32) return MAXK_E_DIM;
    hipStream_t st = as_stream(stream);
    if (num_cols == 0) return MAXK_OK;
    if (num_rows == 0 || num_edges == 0) return zero_floats(dxs, (size_t)num_cols * dim_k, st);
    if (!indices || !values || !grad || !sel || !bin_pos || !bin_ptr || !bin_dst) return MAXK_E_ARG;
    if (num_bins != (int)((num_cols + kBinDests - 1) / kBinDests) || num_slots < num_edges ||
        num_slots > INT32_MAX)
        return MAXK_E_ARG;
    if (!workspace || workspace_bytes < maxk_backward_binned_workspace_bytes(num_slots, dim_k))
        return MAXK_E_WORKSPACE;
    float *Pbuf = static_cast<float *>(workspace);
    int rc = dispatch_k<BinPhase1>(dim_k, edge_selectors != 0, sched, num_panels, indptr, indices,
                                   values, grad, sel, bin_pos, num_rows, dim_origin, dim_k, dxs,
                                   Pbuf, st);
    if (rc) return rc;
    const unsigned blocks = (unsigned)num_bins;      // one wave (block) per bin
    const size_t lds = (size_t)kBinDests * (dim_k + 4) * sizeof(float);
    switch (dim_k) {
    case 8:
        hipLaunchKernelGGL(bwd_bin_sum_kernel<8>, dim3(blocks), dim3(kWave), lds, st, bin_ptr,
                           num_bins, bin_dst, Pbuf, num_cols, dxs);
        break;
    case 16:
        hipLaunchKernelGGL(bwd_bin_sum_kernel<16>, dim3(blocks), dim3(kWave), lds, st, bin_ptr,
                           num_bins, bin_dst, Pbuf, num_cols, dxs);
        break;
    default:
        hipLaunchKernelGGL(bwd_bin_sum_kernel<32>, dim3(blocks), dim3(kWave), lds, st, bin_ptr,
                           num_bins, bin_dst, Pbuf, num_cols, dxs);
        break;
    }
    return launch_status();
}

}  // extern "C"
