// maxk_spgemm.hip -- MI355X (gfx950) kernels for MaxK-GNN aggregation.
//
// Forward  SpGEMM  Y[r,:]   = sum_e val[e] * scatter_h(data[c], sel[c])   (K1, spmm_maxk.cu:17-106)
// Backward SSpMM   dXs[c,l] = sum_{e:idx[e]=c} val[e] * G[row(e), sel[c,l]] (K2, spmm_maxk_backward.cu:15-115)
//
// Design (DESIGN.md has the full rationale, the measurements and the rooflines):
//  * Work decomposition: merge-path panels over "edges of row r, end of row r"
//    (one wavefront = one panel, equal edge+row cost), built on the device
//    from indptr.  Rows are never assumed short; a row split across panels is
//    finished by a carry fixup, so no output is pre-zeroed and no global
//    atomic touches a row that one wave owns.
//  * Forward: EPS edges per wave-instruction, each with a private LDS row copy
//    (plain ds_read/add/ds_write is race-free; LDS float atomics measured ~7x
//    slower).  CBSR data gathered non-temporally, selector words plain; for
//    k <= 16 a packed record (data + selectors in one line).  Fused
//    multi-relation variants share one CBSR gather across R relations.
//  * Backward, three algorithms behind one entry point:
//      ATOMIC  push: G[r,:] staged in LDS once per (row, panel); per edge the
//              k sampled gradients are added into dXs[c,:] with no-return
//              global float atomics (the reference's scheme, fixed).
//      STAGED  push to staging rows P[csc_pos[e]] (non-temporal 16 B stores),
//              then a merge-path segmented sum over the CSC ranges.
//      LOCAL   destination-owned: dXs and selectors of <= dmax destinations in
//              a wave's LDS, in-edges sorted by source row, one launch per
//              source band so the G window stays cache-resident; edge records
//              read into SGPRs (k = 32, 64).
//  * wave64 everywhere; no CUDA-isms, no warp32 tiling.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/maxk_spgemm.h"
#include "tile_format.h"

#define MAXK_VERSION_STRING "maxk-mi355x 0.1 (gfx950, wave64)"

namespace {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;
constexpr int kMaxDim = 256;

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

__device__ __forceinline__ void wave_sync_lds()
{
    // LDS operations of one wave complete in issue order; this keeps the
    // compiler from moving LDS accesses across the point and makes every
    // lane's ds_add visible to the following ds_read of another lane.
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void gbl_add(float *p, float v)
{
    // no-return global_atomic_add_f32 (agent scope: adders may sit on any XCD)
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------
// Merge-path schedule
// ---------------------------------------------------------------------------
// Cost of the point where row i starts: f(i) = (indptr[i]-indptr[0]) + i*row_cost.
// For cost d, row i(d) = max{i : f(i) <= d}; edge j(d) = min(indptr[i] + d - f(i), indptr[i+1]).
__global__ void schedule_kernel(const int32_t *__restrict__ indptr, int num_rows, int panel_cost,
                                int row_cost, int2 *__restrict__ sched, int64_t num_panels)
{
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p > num_panels) return;
    const int32_t base = indptr[0];
    const int64_t total = (int64_t)(indptr[num_rows] - base) + (int64_t)num_rows * row_cost;
    int64_t d = p * (int64_t)panel_cost;
    if (d > total || p == num_panels) d = total;
    int lo = 0, hi = num_rows;  // invariant: f(lo) <= d; answer in [lo, hi]
    while (lo < hi) {
        const int mid = (int)(((int64_t)lo + hi + 1) >> 1);
        const int64_t f = (int64_t)(indptr[mid] - base) + (int64_t)mid * row_cost;
        if (f <= d) lo = mid; else hi = mid - 1;
    }
    int j;
    if (lo >= num_rows) {
        j = indptr[num_rows];
    } else {
        const int64_t f = (int64_t)(indptr[lo] - base) + (int64_t)lo * row_cost;
        const int64_t jj = (int64_t)indptr[lo] + (d - f);
        j = (int)(jj < (int64_t)indptr[lo + 1] ? jj : (int64_t)indptr[lo + 1]);
    }
    sched[p] = make_int2(lo, j);
}

// warp4 (generate_meta.py:26-48) on the device: per-row chunk counts, then fill.
__global__ void warp4_count_kernel(const int32_t *__restrict__ indptr, int num_rows, int nz,
                                   int32_t *__restrict__ counts)
{
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= num_rows) return;
    const int deg = indptr[r + 1] - indptr[r];
    counts[r] = (deg + nz - 1) / nz;
}

__global__ void warp4_fill_kernel(const int32_t *__restrict__ indptr, int num_rows, int nz,
                                  const int32_t *__restrict__ offsets, int4 *__restrict__ warp4)
{
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= num_rows) return;
    const int b = indptr[r], deg = indptr[r + 1] - b;
    int w = offsets[r];
    for (int t = 0; t < deg; t += nz, ++w)
        warp4[w] = make_int4(r, b + t, deg - t < nz ? deg - t : nz, 0);
}

// Exclusive scan of c[0:n) in place by one workgroup (once-per-graph builder),
// total written to *total.
__global__ __launch_bounds__(256) void exclusive_scan_1block(int32_t *c, int n, int32_t *total)
{
    __shared__ int32_t part[256];
    __shared__ int32_t carry_in;
    if (threadIdx.x == 0) carry_in = 0;
    __syncthreads();
    for (int base = 0; base < n; base += 256 * 16) {
        int loc[16];
        int s = 0;
        for (int t = 0; t < 16; ++t) {
            const int i = base + threadIdx.x * 16 + t;
            loc[t] = i < n ? c[i] : 0;
            s += loc[t];
        }
        part[threadIdx.x] = s;
        __syncthreads();
        for (int off = 1; off < 256; off <<= 1) {
            const int v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
            __syncthreads();
            part[threadIdx.x] += v;
            __syncthreads();
        }
        int run = carry_in + part[threadIdx.x] - s;
        for (int t = 0; t < 16; ++t) {
            const int i = base + threadIdx.x * 16 + t;
            if (i < n) c[i] = run;
            run += loc[t];
        }
        __syncthreads();
        if (threadIdx.x == 255) carry_in += part[255];
        __syncthreads();
    }
    if (threadIdx.x == 0) *total = carry_in;
}

// ---------------------------------------------------------------------------
// Forward: gather-scatter of one edge range into the wave's LDS rows.
//
// LDS float atomics (ds_add_f32) are ~7x slower than the gathers on gfx950
// (tools/ablate/fwd_ablate.hip), so the accumulation is a plain
// ds_read + v_add + ds_write.  That is race-free because every lane of one
// wave-instruction writes a distinct LDS word: the LPE lanes of one edge own
// distinct selected columns (a CBSR row has k distinct columns), and the EPS
// edges of one step each own a private copy of the row accumulator.  Copies
// are summed when the row is flushed.  Later steps are ordered after earlier
// ones by the in-order LDS queue of the wave (the compiler cannot reorder the
// may-alias accesses of one lane).
//
// Layout per compile-time K: VEC consecutive CBSR entries per lane (dwordx4 /
// dwordx2 / dword data + the matching selector bytes), LPE lanes per edge,
// EPS = 64 / LPE edges per step = LDS row copies.  LPE >= 8 keeps the copies
// at <= 8 KB per wave for every k >= 8.
// ---------------------------------------------------------------------------
#ifndef FWD_VEC16
// CBSR entries per lane at k = 16: 1 (16 lanes per edge, 4 row copies) measured
// 3.16 ms against 4.14 ms for 2 on products (round 5, tools/exp_fwd_small_k.py)
#define FWD_VEC16 1
#endif
#ifndef FWD_VEC8
#define FWD_VEC8 1    // ... at k = 8
#endif
#ifndef FWD_VEC32
#define FWD_VEC32 4   // ... at k = 32 (development knob)
#endif
#ifndef FWD_VEC64
#define FWD_VEC64 4   // ... at k = 64 (development knob)
#endif
template <int K>
struct FwdLayout {
    static constexpr int VEC = K > 64 ? 4 : K == 64 ? FWD_VEC64
                             : K >= 32 ? FWD_VEC32
                             : (K >= 16 ? FWD_VEC16 : (K >= 8 ? FWD_VEC8 : 1));
    static constexpr int LPE = K / VEC;
    static constexpr int EPS = kWave / LPE;
};

// Generic k: 64/k edges per step, capped at 8 (each slot owns a 1 KB row copy;
// uncapped, k = 1 would need 64 KB per wave and the launch would fail).
__host__ __device__ constexpr int fwd_copies_generic(int k)
{
    return k >= kWave ? 1 : (kWave / k < 8 ? kWave / k : 8);
}

template <int K>
__host__ __device__ constexpr int fwd_copies(int k)
{
    if constexpr (K > 0) return FwdLayout<K>::EPS;
    else return fwd_copies_generic(k);
}

template <int VEC>
struct VecT;
template <> struct VecT<4> { typedef f4 D; typedef uint32_t S; };
template <> struct VecT<2> { typedef float D __attribute__((ext_vector_type(2))); typedef uint16_t S; };
template <> struct VecT<1> { typedef float D; typedef uint8_t S; };

template <int VEC>
__device__ __forceinline__ void rmw_acc(float *acc, typename VecT<VEC>::S sb, float v,
                                        typename VecT<VEC>::D d)
{
    if constexpr (VEC == 4) {
        float *p0 = acc + (sb & 0xff), *p1 = acc + ((sb >> 8) & 0xff);
        float *p2 = acc + ((sb >> 16) & 0xff), *p3 = acc + (sb >> 24);
        *p0 += v * d.x; *p1 += v * d.y; *p2 += v * d.z; *p3 += v * d.w;
    } else if constexpr (VEC == 2) {
        float *p0 = acc + (sb & 0xff), *p1 = acc + (sb >> 8);
        *p0 += v * d.x; *p1 += v * d.y;
    } else {
        acc[sb] += v * d;
    }
}

// Packed CBSR (k <= 16): one record per node = k fp32 values, then k selector
// bytes, padded to RS = 32 / 64 / 128 bytes (k = 4 / 8 / 16), so a gathered
// neighbour costs one cache line instead of two (data line + selector line).
template <int K>
struct Packed {
    static constexpr int RS = K == 4 ? 32 : (K == 8 ? 64 : (K == 16 ? 128 : 0));
};

// ESEL: also write the gathered selector bytes in edge order, esel[e * K + l]
// (the backward's STAGED_EDGE pass then reads them sequentially instead of
// gathering one selector line per edge a second time).
#ifndef FWD_ESEL_DPP
#define FWD_ESEL_DPP 0
#endif
#ifndef FWD_ESEL_NT
#define FWD_ESEL_NT 0  // plain stores: products k=8 +0.26 ms vs +0.34 nt, k=32 +0.89 vs +1.04
#endif
// lane i <- lane i ^ 1 / i ^ 2 (DPP quad_perm [1,0,3,2] / [2,3,0,1])
__device__ __forceinline__ uint32_t dpp_xor1(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t dpp_xor2(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
}

// The edge stream one batch ahead (FWD_PF): pf holds the lane's (column, value)
// of the batch that starts at e0 on entry and of the batch that starts at e1 --
// the next row's first -- on return, loaded while this batch's gathers run, so
// a row's first gathers do not wait for its edge loads.  pend bounds the loads
// (the panel's last edge).  Used by the cacheable-gather (column-blocked) form
// only: Reddit k=32 forward 2.38 -> 2.34 ms, while the products forms (short
// rows, non-temporal or packed gathers) lost 1-4 % with it.
#ifndef FWD_PF
#define FWD_PF 1
#endif
template <int K, bool NTD>
constexpr bool fwd_pf_on()
{
    return K > 0 && FWD_PF && !NTD;
}
struct FwdPf {
    int c = 0;
    float v = 0.f;
};
__device__ __forceinline__ void fwd_pf_load(FwdPf &pf, int b, int pend,
                                            const int32_t *__restrict__ idx,
                                            const float *__restrict__ val)
{
    const int e = b + lane_id();
    pf.c = 0;
    pf.v = 0.f;
    if (e < pend) {
        pf.c = __builtin_nontemporal_load(idx + e);
        pf.v = __builtin_nontemporal_load(val + e);
    }
}

template <int K, int RS = 0, bool ESEL = false, bool NTD = true, bool PF = false>
__device__ __forceinline__ void fwd_edges_vec(int e0, int e1, const int32_t *__restrict__ idx,
                                              const float *__restrict__ val,
                                              const float *__restrict__ data,
                                              const uint8_t *__restrict__ sel, float *acc,
                                              uint8_t *__restrict__ esel, FwdPf *pf = nullptr,
                                              int pend = 0)
{
    using Lay = FwdLayout<K>;
    constexpr int VEC = Lay::VEC, LPE = Lay::LPE, EPS = Lay::EPS;
    constexpr int STEPS = kWave / EPS;  // steps per 64-edge batch
#ifndef FWD_U
#define FWD_U 8
#endif
    constexpr int U = STEPS < FWD_U ? STEPS : FWD_U;  // gathers in flight per lane
    using D = typename VecT<VEC>::D;
    using SB = typename VecT<VEC>::S;
    const int lane = lane_id();
    const int sub = lane % LPE;
    const int slot = lane / LPE;
    float *my_acc = acc + slot * kMaxDim;
    for (int base = e0; base < e1; base += kWave) {
        const int n = (e1 - base) < kWave ? (e1 - base) : kWave;
        int my_c = 0;
        float my_v = 0.f;
        if constexpr (PF) {
            my_c = pf->c;
            my_v = pf->v;
            fwd_pf_load(*pf, base + kWave < e1 ? base + kWave : e1, pend, idx, val);
        } else if (lane < n) {
            my_c = __builtin_nontemporal_load(idx + base + lane);
            my_v = __builtin_nontemporal_load(val + base + lane);
        }
#pragma unroll
        for (int s0 = 0; s0 < STEPS; s0 += U) {
            if (s0 * EPS >= n) break;
            D d[U];
            SB sb[U];
            float v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int t = (s0 + u) * EPS + slot;
                const int c = __shfl(my_c, t < kWave ? t : 0);
                v[u] = __shfl(my_v, t < kWave ? t : 0);
                if (t < n) {
                    if constexpr (RS == 0) {
                        const size_t off = (size_t)c * K + sub * VEC;
                        // data rows non-temporal (measured 3.45 -> 3.18 ms on Reddit k=32);
                        // selector words plain (nt 4-B loads measured slower)
                        // (NTD false: cacheable, for the column-blocked forward whose
                        // block-major sweep re-reads a block's rows from L2)
                        if constexpr (NTD)
                            d[u] = __builtin_nontemporal_load(reinterpret_cast<const D *>(data + off));
                        else
                            d[u] = *reinterpret_cast<const D *>(data + off);
                        sb[u] = *reinterpret_cast<const SB *>(sel + off);
                    } else {  // data = record base, sel = record base + 4K bytes
                        const size_t rec = (size_t)c * RS;
#if FWD_PACKED_NT
                        d[u] = __builtin_nontemporal_load(reinterpret_cast<const D *>(reinterpret_cast<const uint8_t *>(data) + rec + 4 * sub * VEC));
                        sb[u] = __builtin_nontemporal_load(reinterpret_cast<const SB *>(sel + rec + sub * VEC));
#else
                        d[u] = *reinterpret_cast<const D *>(reinterpret_cast<const uint8_t *>(data) + rec + 4 * sub * VEC);
                        sb[u] = *reinterpret_cast<const SB *>(sel + rec + sub * VEC);
#endif
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int t = (s0 + u) * EPS + slot;
                if (t < n) rmw_acc<VEC>(my_acc, sb[u], v[u], d[u]);
                if constexpr (ESEL) {
                    // one dword store per 4 selector bytes: neighbouring lanes of the
                    // edge hand theirs over (byte / short stores ran at ~1 TB/s)
                    uint32_t w = (uint32_t)sb[u];
#if FWD_ESEL_DPP  // DPP quad permutes (no LDS op)
                    if constexpr (VEC == 2) w |= dpp_xor1(w) << 16;
                    if constexpr (VEC == 1) {
                        w |= dpp_xor1(w) << 8;
                        w |= dpp_xor2(w) << 16;
                    }
#else
                    if constexpr (VEC == 2) w |= (uint32_t)__shfl_xor((int)w, 1) << 16;
                    if constexpr (VEC == 1) {
                        w |= (uint32_t)__shfl_xor((int)w, 1) << 8;
                        w |= (uint32_t)__shfl_xor((int)w, 2) << 16;
                    }
#endif
                    constexpr int SPL = 4 / VEC;  // lanes per stored dword
                    if (t < n && sub % SPL == 0) {
                        uint32_t *dst = reinterpret_cast<uint32_t *>(esel + (size_t)(base + t) * K + sub * VEC);
#if FWD_ESEL_NT
                        __builtin_nontemporal_store(w, dst);
#else
                        *dst = w;
#endif
                    }
                }
            }
        }
    }
}


// Any k: one CBSR entry per lane, EPS = 64 / min(k, 64) row copies.
__device__ __forceinline__ void fwd_edges_scalar(int e0, int e1, int k,
                                                 const int32_t *__restrict__ idx,
                                                 const float *__restrict__ val,
                                                 const float *__restrict__ data,
                                                 const uint8_t *__restrict__ sel, float *acc,
                                                 uint8_t *__restrict__ esel)
{
    const int lane = lane_id();
    if (k <= kWave) {
        const int eps = fwd_copies_generic(k);
        const int slot = lane / k, l = lane % k;
        float *my_acc = acc + slot * kMaxDim;
        for (int e = e0; e < e1; e += eps) {
            const int my = e + slot;
            if (slot < eps && my < e1) {
                const int c = idx[my];
                const float v = val[my];
                const size_t off = (size_t)c * k + l;
                my_acc[sel[off]] += v * data[off];
                if (esel) esel[(size_t)my * k + l] = sel[off];
            }
        }
    } else {
        for (int e = e0; e < e1; ++e) {
            const int c = idx[e];
            const float v = val[e];
            for (int l = lane; l < k; l += kWave) {
                const size_t off = (size_t)c * k + l;
                acc[sel[off]] += v * data[off];
                if (esel) esel[(size_t)e * k + l] = sel[off];
            }
        }
    }
}

template <int K, int RS = 0, bool ESEL = false, bool NTD = true>
__device__ __forceinline__ void fwd_edges(int e0, int e1, int k, const int32_t *__restrict__ idx,
                                          const float *__restrict__ val,
                                          const float *__restrict__ data,
                                          const uint8_t *__restrict__ sel, float *acc,
                                          uint8_t *__restrict__ esel = nullptr)
{
    if constexpr (K > 0)
        fwd_edges_vec<K, RS, ESEL, NTD>(e0, e1, idx, val, data, sel, acc, esel);
    else
        fwd_edges_scalar(e0, e1, k, idx, val, data, sel, acc, ESEL ? esel : nullptr);
}

// Row flushes: sum the `copies` LDS row copies, zero them, and store / add.
enum FlushOp { kStore = 0, kAtomic = 1, kAdd = 2 };

#ifndef FWD_NT_OUT
#define FWD_NT_OUT 1  // nt row stores: -1 % fwd on Reddit and products (tools/nt_sweep.sh)
#endif
#ifndef FWD_PACKED_NT
#define FWD_PACKED_NT 0
#endif

// SUMP (sp != nullptr, kStore only): the row is stored as
// ((sp[0] + sp[ss]) + ... + sp[(nsp-1)*ss]) + row -- the column-blocked
// forward's last block adding the earlier blocks' partial rows, in block
// order: bitwise what maxk_rows_sum gives over all nb parts.
template <int OP>
__device__ __forceinline__ void flush_row(float *acc, int copies, float *__restrict__ dst, int dim,
                                          const float *__restrict__ sp = nullptr, int nsp = 0,
                                          size_t ss = 0)
{
    const int lane = lane_id();
    wave_sync_lds();
    if (OP != kAtomic && (dim & 3) == 0) {
        for (int c4 = lane; c4 < (dim >> 2); c4 += kWave) {
            f4 a = reinterpret_cast<f4 *>(acc)[c4];
            reinterpret_cast<f4 *>(acc)[c4] = f4{0.f, 0.f, 0.f, 0.f};
            for (int cp = 1; cp < copies; ++cp) {
                f4 *q = reinterpret_cast<f4 *>(acc + cp * kMaxDim) + c4;
                a += *q;
                *q = f4{0.f, 0.f, 0.f, 0.f};
            }
            if (OP == kAdd) a += reinterpret_cast<const f4 *>(dst)[c4];  // row owned by this wave
            if (OP == kStore && sp) {
                f4 s = __builtin_nontemporal_load(reinterpret_cast<const f4 *>(sp) + c4);
                for (int q = 1; q < nsp; ++q)
                    s += __builtin_nontemporal_load(reinterpret_cast<const f4 *>(sp + q * ss) + c4);
                a = s + a;
            }
#if FWD_NT_OUT
            __builtin_nontemporal_store(a, reinterpret_cast<f4 *>(dst) + c4);
#else
            reinterpret_cast<f4 *>(dst)[c4] = a;
#endif
        }
    } else {
        for (int c = lane; c < dim; c += kWave) {  // 256 contiguous bytes per instruction
            float a = acc[c];
            acc[c] = 0.f;
            for (int cp = 1; cp < copies; ++cp) {
                a += acc[cp * kMaxDim + c];
                acc[cp * kMaxDim + c] = 0.f;
            }
            if (OP == kStore && sp) {
                float t = sp[c];
                for (int q = 1; q < nsp; ++q) t += sp[q * ss + c];
                a = t + a;
            }
            if (OP == kStore) dst[c] = a;
            else if (OP == kAtomic) gbl_add(dst + c, a);
            else dst[c] += a;
        }
    }
    wave_sync_lds();
}

__device__ __forceinline__ void zero_lds(float *acc, int n)
{
    for (int c = lane_id(); c < n; c += kWave) acc[c] = 0.f;
    wave_sync_lds();
}

// Panel-scheduled forward.  Rows [i0, i1) are finished and owned by this
// wave (plain store); row i1 is in progress at the panel end -> carry.
// Occupancy target of the forward's register allocation: 5 waves per SIMD (the
// LDS row copies allow 5 at k = 8 / 32 and 10 at k = 16) fits the packed k = 16
// form without scratch (products k=16 forward 3.17 -> 3.11 ms); the other forms
// keep the compiler's 4 (at k = 32 / 64, 5 spills: Reddit 2.34 -> 2.62 ms).
template <int K, int RS, bool ESEL>
constexpr int fwd_waves_per_eu()
{
    return K == 16 && RS > 0 && !ESEL ? 5 : 1;
}
template <int K, int RS = 0, bool ACC = false, bool ESEL = false, bool NTD = true>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(fwd_waves_per_eu<K, RS, ESEL>())))
void fwd_panel_kernel(
    const int2 *__restrict__ sched, int64_t num_panels, const int32_t *__restrict__ indptr,
    const int32_t *__restrict__ idx, const float *__restrict__ val,
    const float *__restrict__ data, const uint8_t *__restrict__ sel, int num_rows, int dim,
    int k, float *__restrict__ out, float *__restrict__ carry, int32_t *__restrict__ carry_row,
    float *__restrict__ owner, uint8_t *__restrict__ esel, const float *__restrict__ sump,
    int nsump)
{
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int dimp = (dim + 3) & ~3;
    const int copies = fwd_copies<K>(k);
    // selectors are uint8, so a full 256-float row per copy is never overrun
    float *acc = lds + (threadIdx.x / kWave) * copies * kMaxDim;
    const int64_t w = (int64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave;
    if (w >= num_panels) return;
    zero_lds(acc, copies * kMaxDim);
    const int2 a = sched[w], b = sched[w + 1];
    const int i0 = a.x, j0 = a.y, i1 = b.x, j1 = b.y;
    int e = j0;
    // a first row that began in an earlier panel is split: its part goes to
    // this panel's owner slot, and carry_fixup_owner_kernel adds the parts up
    // in panel order (one writer per row, no atomics, bitwise deterministic)
    const bool split_first = i0 < i1 && j0 > indptr[i0];
    int has_carry = 0;
    if constexpr (fwd_pf_on<K, NTD>()) {
        // the edge stream one batch ahead across rows (FwdPf); e == eb at the carry
        FwdPf pf;
        fwd_pf_load(pf, j0, j1, idx, val);
        for (int r = i0; r < i1; ++r) {
            const int re = indptr[r + 1];
            if (e < re)
                fwd_edges_vec<K, RS, ESEL, NTD, true>(e, re, idx, val, data, sel, acc, esel, &pf, j1);
            if (r == i0 && split_first)
                flush_row<kStore>(acc, copies, owner + (size_t)w * dimp, dim);
            else if (!ACC && sump)
                flush_row<kStore>(acc, copies, out + (size_t)r * dim, dim, sump + (size_t)r * dim,
                                  nsump, (size_t)num_rows * dim);
            else
                flush_row<ACC ? kAdd : kStore>(acc, copies, out + (size_t)r * dim, dim);
            e = re;
        }
        if (i1 < num_rows) {
            const int eb = e > indptr[i1] ? e : indptr[i1];
            if (eb < j1) {
                if (eb != e) fwd_pf_load(pf, eb, j1, idx, val);
                fwd_edges_vec<K, RS, ESEL, NTD, true>(eb, j1, idx, val, data, sel, acc, esel, &pf, j1);
                has_carry = 1;
            }
        }
    } else {
        for (int r = i0; r < i1; ++r) {
            const int re = indptr[r + 1];
            if (e < re) fwd_edges<K, RS, ESEL, NTD>(e, re, k, idx, val, data, sel, acc, esel);
            if (r == i0 && split_first)
                flush_row<kStore>(acc, copies, owner + (size_t)w * dimp, dim);
            else if (!ACC && sump)
                flush_row<kStore>(acc, copies, out + (size_t)r * dim, dim, sump + (size_t)r * dim,
                                  nsump, (size_t)num_rows * dim);
            else
                flush_row<ACC ? kAdd : kStore>(acc, copies, out + (size_t)r * dim, dim);
            e = re;
        }
        if (i1 < num_rows) {
            const int eb = e > indptr[i1] ? e : indptr[i1];
            if (eb < j1) {
                fwd_edges<K, RS, ESEL, NTD>(eb, j1, k, idx, val, data, sel, acc, esel);
                has_carry = 1;
            }
        }
    }
    if (has_carry) {
        flush_row<kStore>(acc, copies, carry + (size_t)w * dimp, dimp);
        if (lane_id() == 0) carry_row[w] = i1;
    } else if (lane_id() == 0) {
        carry_row[w] = -1;
    }
}

// Adds the panels' carry rows into the output (after the owners stored their
// rows): nrel relations, carry rows carry_stride apart, output relations
// rel_stride apart.  The carries of one row come from consecutive panels (a
// row split by merge-path spans panels w1..w2, w2 its owner), so the wave of
// the first such panel sums them all and updates the row with a plain
// read-add-store -- every row has one writer, no atomics (the atomic form
// cost ~2x: 64-B memory-side atomic requests).
__global__ __launch_bounds__(kBlock) void carry_fixup_kernel(
    int64_t num_panels, const float *__restrict__ carry, const int32_t *__restrict__ carry_row,
    float *__restrict__ out, int dim, int carry_stride, int nrel = 1, size_t rel_stride = 0)
{
    const int64_t w = (int64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave;
    if (w >= num_panels) return;
    const int r = carry_row[w];
    if (r < 0 || (w > 0 && carry_row[w - 1] == r)) return;
    int64_t w_end = w + 1;
    while (w_end < num_panels && carry_row[w_end] == r) ++w_end;
    if ((dim & 3) == 0 && (carry_stride & 3) == 0 && (rel_stride & 3) == 0 &&
        ((reinterpret_cast<uintptr_t>(out) | reinterpret_cast<uintptr_t>(carry)) & 15) == 0) {
        // 16 B per lane (a 256-wide row is one wave-instruction), the relations'
        // loads issued together: the multi-relation forward's fixup (8 relations
        // x 1 KB per split row) took 0.35 ms of proteins' 5.2 ms with 4-B lanes.
        // Same additions in the same order as the scalar loop below.
        const int d4 = dim >> 2;
        for (int c4 = lane_id(); c4 < d4; c4 += kWave) {
            for (int q0 = 0; q0 < nrel; q0 += 4) {
                const int nq = nrel - q0 < 4 ? nrel - q0 : 4;
                f4 a[4];
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (j < nq)
                        a[j] = reinterpret_cast<const f4 *>(out + (q0 + j) * rel_stride +
                                                            (size_t)r * dim)[c4];
                for (int64_t v = w; v < w_end; ++v) {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (j < nq)
                            a[j] += reinterpret_cast<const f4 *>(
                                carry + ((size_t)v * nrel + q0 + j) * carry_stride)[c4];
                }
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (j < nq)
                        reinterpret_cast<f4 *>(out + (q0 + j) * rel_stride + (size_t)r * dim)[c4] = a[j];
            }
        }
        return;
    }
    for (int q = 0; q < nrel; ++q) {
        float *dst = out + q * rel_stride + (size_t)r * dim;
        for (int c = lane_id(); c < dim; c += kWave) {
            float a = dst[c];
            for (int64_t v = w; v < w_end; ++v) a += carry[((size_t)v * nrel + q) * carry_stride + c];
            dst[c] = a;
        }
    }
}

// Forward fixup: row r split over panels w .. w_end (carries of w .. w_end-1,
// the owner's part in owner slot w_end) is summed in panel order by the wave
// of its first panel and stored (ACC: added) -- the output row is not read
// unless accumulating.
// The carrying panels are consecutive; between the last of them and the
// owner (the first panel whose end lies past row r) there can be empty panels
// (panel_cost < row_cost: boundaries inside a row's end cost), which carry
// nothing and have no owner slot.
template <bool ACC>
__global__ __launch_bounds__(kBlock) void carry_fixup_owner_kernel(
    const int2 *__restrict__ sched, int64_t num_panels, const float *__restrict__ carry,
    const float *__restrict__ owner, const int32_t *__restrict__ carry_row,
    float *__restrict__ out, int dim, int dimp, int num_rows, const float *__restrict__ sump,
    int nsump)
{
    const int64_t w = (int64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave;
    if (w >= num_panels) return;
    const int r = carry_row[w];
    if (r < 0 || (w > 0 && carry_row[w - 1] == r)) return;
    int64_t w_end = w + 1;
    while (w_end < num_panels && carry_row[w_end] == r) ++w_end;
    int64_t own = w_end;
    while (sched[own + 1].x <= r) ++own;   // the panel that owns row r (exists: r < num_rows)
    float *dst = out + (size_t)r * dim;
    if ((dim & 3) == 0) {
        for (int c4 = lane_id(); c4 < (dim >> 2); c4 += kWave) {
            f4 a = reinterpret_cast<const f4 *>(owner + (size_t)own * dimp)[c4];
            for (int64_t v = w; v < w_end; ++v) a += reinterpret_cast<const f4 *>(carry + (size_t)v * dimp)[c4];
            if (ACC) a += reinterpret_cast<const f4 *>(dst)[c4];
            if (!ACC && sump) {  // earlier blocks' partial rows first (flush_row's SUMP order)
                const f4 *sp = reinterpret_cast<const f4 *>(sump + (size_t)r * dim) + c4;
                f4 t = sp[0];
                for (int q = 1; q < nsump; ++q) t += sp[(size_t)q * num_rows * (dim >> 2)];
                a = t + a;
            }
            __builtin_nontemporal_store(a, reinterpret_cast<f4 *>(dst) + c4);
        }
    } else {
        for (int c = lane_id(); c < dim; c += kWave) {
            float a = owner[(size_t)own * dimp + c];
            for (int64_t v = w; v < w_end; ++v) a += carry[(size_t)v * dimp + c];
            if (!ACC && sump) {
                float t = sump[(size_t)r * dim + c];
                for (int q = 1; q < nsump; ++q) t += sump[((size_t)q * num_rows + r) * dim + c];
                a = t + a;
            }
            dst[c] = ACC ? dst[c] + a : a;
        }
    }
}

// ---------------------------------------------------------------------------
// Dense SpMM baseline Y = A . X, X fp32[V, dim] dense (the
// kernels the reference compares MaxK against, GNNAdvisor's SAG
// spmm_gnna.cu:60-140 and cuSPARSE spmm_cusparse.cu:6-62).  Same merge-path
// panels as the MaxK forward.  A gathered X row is contiguous, so there is no
// scatter: LPE lanes own 4 consecutive columns each and accumulate in
// registers; EPS = 64 / LPE edges per step, their partial sums reduced with
// cross-lane shuffles at each row flush.  No LDS.
// ---------------------------------------------------------------------------
template <int LPE>
__device__ __forceinline__ void dense_edges(int e0, int e1, int dim, const int32_t *__restrict__ idx,
                                            const float *__restrict__ val,
                                            const float *__restrict__ x, f4 &acc)
{
    constexpr int EPS = kWave / LPE;
    constexpr int STEPS = LPE;  // steps per 64-edge batch
    constexpr int U = STEPS < 8 ? STEPS : 8;
    const int lane = lane_id();
    const int sub = lane % LPE, slot = lane / LPE;
    const bool col_ok = sub * 4 < dim;
    for (int base = e0; base < e1; base += kWave) {
        const int n = (e1 - base) < kWave ? (e1 - base) : kWave;
        int my_c = 0;
        float my_v = 0.f;
        if (lane < n) {
            my_c = __builtin_nontemporal_load(idx + base + lane);
            my_v = __builtin_nontemporal_load(val + base + lane);
        }
#pragma unroll
        for (int s0 = 0; s0 < STEPS; s0 += U) {
            if (s0 * EPS >= n) break;
            f4 d[U];
            float v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int t = (s0 + u) * EPS + slot;
                const int c = __shfl(my_c, t);
                v[u] = __shfl(my_v, t);
                d[u] = f4{0.f, 0.f, 0.f, 0.f};
                if (t < n && col_ok) d[u] = *reinterpret_cast<const f4 *>(x + (size_t)c * dim + sub * 4);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) acc += v[u] * d[u];
        }
    }
}

template <int LPE>
__device__ __forceinline__ void dense_flush(f4 &acc, float *__restrict__ dst, int dim)
{
#pragma unroll
    for (int m = LPE; m < kWave; m <<= 1) {
        acc.x += __shfl_xor(acc.x, m);
        acc.y += __shfl_xor(acc.y, m);
        acc.z += __shfl_xor(acc.z, m);
        acc.w += __shfl_xor(acc.w, m);
    }
    const int lane = lane_id();
    if (lane < LPE && lane * 4 < dim) reinterpret_cast<f4 *>(dst)[lane] = acc;
    acc = f4{0.f, 0.f, 0.f, 0.f};
}

template <int LPE>
__global__ __launch_bounds__(kBlock) void dense_panel_kernel(
    const int2 *__restrict__ sched, int64_t num_panels, const int32_t *__restrict__ indptr,
    const int32_t *__restrict__ idx, const float *__restrict__ val, const float *__restrict__ x,
    int num_rows, int dim, float *__restrict__ out, float *__restrict__ carry,
    int32_t *__restrict__ carry_row)
{
    const int64_t w = (int64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave;
    if (w >= num_panels) return;
    const int2 a = sched[w], b = sched[w + 1];
    const int i0 = a.x, j0 = a.y, i1 = b.x, j1 = b.y;
    f4 acc = f4{0.f, 0.f, 0.f, 0.f};
    int e = j0;
    for (int r = i0; r < i1; ++r) {
        const int re = indptr[r + 1];
        if (e < re) dense_edges<LPE>(e, re, dim, idx, val, x, acc);
        dense_flush<LPE>(acc, out + (size_t)r * dim, dim);
        e = re;
    }
    int has_carry = 0;
    if (i1 < num_rows) {
        const int eb = e > indptr[i1] ? e : indptr[i1];
        if (eb < j1) {
            dense_edges<LPE>(eb, j1, dim, idx, val, x, acc);
            has_carry = 1;
        }
    }
    if (has_carry) {
        dense_flush<LPE>(acc, carry + (size_t)w * dim, dim);
        if (lane_id() == 0) carry_row[w] = i1;
    } else if (lane_id() == 0) {
        carry_row[w] = -1;
    }
}

// ---------------------------------------------------------------------------
// Fused multi-relation forward (ogbn-proteins, config 5):
// Y_q = A_q . X^ for q < R relations sharing one CSR and one CBSR, edge values
// val[e * R + q].  Parity: R independent calls of the single-relation forward.
// One edge per wave-step: the CBSR row is gathered once (LPE lanes x VEC
// entries, as FwdLayout) and reused by RP = 64 / LPE relations at once (lane
// group q), ceil(R / RP) passes.  Each relation owns one LDS row of MROW
// floats; the 4-float skew between relation rows puts the same selected
// column of different relations in different banks.  No row copies are
// needed: the lanes of one relation in one step touch distinct columns.
// ---------------------------------------------------------------------------
constexpr int kMultiRow = kMaxDim + 4;
constexpr int kMaxRel = 16;

template <int K>
__device__ __forceinline__ void fwd_multi_edges(int e0, int e1, int R,
                                                const int32_t *__restrict__ idx,
                                                const float *__restrict__ val,
                                                const float *__restrict__ data,
                                                const uint8_t *__restrict__ sel, float *acc)
{
    using Lay = FwdLayout<K>;
    constexpr int VEC = Lay::VEC, LPE = Lay::LPE, RP = kWave / LPE;
    constexpr int U = 8;
    using D = typename VecT<VEC>::D;
    using SB = typename VecT<VEC>::S;
    const int lane = lane_id();
    const int sub = lane % LPE, grp = lane / LPE;
    const int passes = (R + RP - 1) / RP;
    for (int base = e0; base < e1; base += kWave) {
        const int n = (e1 - base) < kWave ? (e1 - base) : kWave;
        const int my_c = lane < n ? __builtin_nontemporal_load(idx + base + lane) : 0;
        for (int s0 = 0; s0 < n; s0 += U) {
            D d[U];
            SB sb[U];
            float v[U];
            // CBSR gathers and the first pass's edge values in flight together
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (s0 + u >= n) break;
                const int c = __builtin_amdgcn_readlane(my_c, s0 + u);
                const size_t off = (size_t)c * K + sub * VEC;
                d[u] = __builtin_nontemporal_load(reinterpret_cast<const D *>(data + off));
                sb[u] = *reinterpret_cast<const SB *>(sel + off);
                v[u] = grp < R ? val[(size_t)(base + s0 + u) * R + grp] : 0.f;
            }
            for (int p = 0; p < passes; ++p) {
                const int q = p * RP + grp;
                if (p > 0) {
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        if (s0 + u >= n) break;
                        v[u] = q < R ? val[(size_t)(base + s0 + u) * R + q] : 0.f;
                    }
                }
                if (q < R) {
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        if (s0 + u >= n) break;
                        rmw_acc<VEC>(acc + q * kMultiRow, sb[u], v[u], d[u]);
                    }
                }
            }
        }
    }
}

// Store the R accumulator rows to dst + q * rel_stride and zero them.
__device__ __forceinline__ void flush_multi(float *acc, int R, float *__restrict__ dst,
                                            size_t rel_stride, int dim)
{
    const int lane = lane_id();
    wave_sync_lds();
    if ((dim & 3) == 0) {
        const int d4 = dim >> 2;
        for (int i = lane; i < R * d4; i += kWave) {
            const int q = i / d4, c4 = i - q * d4;
            f4 *src = reinterpret_cast<f4 *>(acc + q * kMultiRow) + c4;
            reinterpret_cast<f4 *>(dst + q * rel_stride)[c4] = *src;
            *src = f4{0.f, 0.f, 0.f, 0.f};
        }
    } else {
        for (int i = lane; i < R * dim; i += kWave) {
            const int q = i / dim, c = i - q * dim;
            dst[q * rel_stride + c] = acc[q * kMultiRow + c];
            acc[q * kMultiRow + c] = 0.f;
        }
    }
    wave_sync_lds();
}

// Relation-vector form for R = 4*R4 relations (R4 in {1, 2, 4}, so that
// L = K*R4 divides or is a multiple of 64): the accumulator is laid out
// [col][R] so one lane owns (selected entry j, relation quad rq) and updates
// four relations with one ds_read_b128 + ds_write_b128 per edge; the edge's
// four values arrive as one float4.  L = K*R4 lanes per edge: EPS = 64/L
// edges per step with private row copies when L < 64, else L/64 passes.
// Lanes of one step write distinct words (an edge's selected columns are
// distinct; different edges use different copies).
#ifndef FWD_REL8_SWZ
#define FWD_REL8_SWZ 1   // R = 8: 8-float column records, quads XOR-swizzled (0: 12-float records)
#endif
// R = 8, k = 32: lane 2j + q works on (entry j, relation quad q) instead of lane
// j + 32q.  A ds_read_b128 lane group (16 lanes) then covers 8 entries x both
// quads, whose 16-B units 2c + (q ^ c>>3&1) are distinct mod 16 iff the 8
// columns differ mod 8; a ds_write_b128 group (8 contiguous lanes) covers 4
// entries, distinct mod 8 iff their columns differ mod 4 -- and the bank order
// (cbsr_bank_order_kernel, mode 2) makes both hold wherever the row allows.
// A bank-conflict model of the two layouts (32 random columns of 256) gives
// 27 -> 22 LDS cycles per edge.  Same elements, same order: same bits.
#ifndef FWD_REL8_ILV
#define FWD_REL8_ILV 1
#endif
template <int K, int R4>
struct Rel4 {
    static_assert((R4 & (R4 - 1)) == 0, "R4 must be a power of two");
    static constexpr int R = 4 * R4;
    static constexpr int L = K * R4;
    static constexpr int EPS = L >= kWave ? 1 : kWave / L;
    static constexpr int PASSES = L >= kWave ? L / kWave : 1;
    static constexpr int U = PASSES >= 8 ? 1 : 8 / PASSES;
    // floats per column record: an odd number of float4 quads, so the 4-bank
    // group of a b128 access (= col * S/4 mod 16) takes all 16 values; with
    // plain S = 8 (R = 8) only 8 groups were used: 19 conflict cycles per
    // ds_*_b128 measured on proteins (SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS).
    // R = 8 now keeps S = 8 with the two quads of column col swapped when bit 3
    // of col is set (SWZ): quad 0's 16-B unit 2*col + (col >> 3 & 1) again
    // takes all 16 values mod 16, and the record is 8 KB per copy instead of
    // 12 (proteins forward 5.32 -> 5.12 ms, same sums bit for bit)
    static constexpr bool SWZ = FWD_REL8_SWZ && R4 == 2;
    static constexpr bool ILV = FWD_REL8_ILV && SWZ && K == 32;   // lane = 2 * entry + quad
    static __device__ __forceinline__ int entry(int item) { return ILV ? item >> 1 : item % K; }
    static __device__ __forceinline__ int quad(int item) { return ILV ? item & 1 : item / K; }
    static constexpr int S = (R4 & 1) || SWZ ? R : R + 4;
    static constexpr int ROW = kMaxDim * S;  // floats per accumulator copy
    // word offset of relation quad rq of column col
    static __device__ __forceinline__ uint32_t off(uint32_t col, int rq)
    {
        return col * S + 4 * (SWZ ? ((uint32_t)rq ^ ((col >> 3) & 1u)) : (uint32_t)rq);
    }
};

// One round of U edges (EPS == 1: every lane works on the same edge): the
// edge's column index is wave-uniform, so the CBSR row and edge-value row
// pointers are scalar and every load is saddr + a constant lane offset.
template <int K, int R4, bool FULL>
__device__ __forceinline__ void rel4_round_uniform(int my_c, int base, int s0, int n,
                                                   const float *__restrict__ val,
                                                   const float *__restrict__ data,
                                                   const uint8_t *__restrict__ sel, float *my)
{
    using C = Rel4<K, R4>;
    constexpr int R = C::R, PASSES = C::PASSES, U = C::U;
    const int lane = lane_id();
    float d[U][PASSES];
    uint32_t col[U][PASSES];
    f4 v[U][PASSES];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if (!FULL && s0 + u >= n) break;
        const int c = __builtin_amdgcn_readlane(my_c, s0 + u);
        const float *drow = data + (size_t)c * K;
        const uint8_t *srow = sel + (size_t)c * K;
        // per-lane float4 of the edge's values (scalar loads + per-lane
        // select measured slower: 8.37 vs 7.33 ms on proteins R=8)
        const f4 *vrow = reinterpret_cast<const f4 *>(val + (size_t)(base + s0 + u) * R);
#pragma unroll
        for (int p = 0; p < PASSES; ++p) {
            const int item = lane + p * kWave;
            const int j = C::entry(item), rq = C::quad(item);
            d[u][p] = drow[j];
            col[u][p] = srow[j];
            v[u][p] = vrow[rq];
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if (!FULL && s0 + u >= n) break;
#pragma unroll
        for (int p = 0; p < PASSES; ++p) {
            const int rq = C::quad(lane + p * kWave);
            f4 *a = reinterpret_cast<f4 *>(my + C::off(col[u][p], rq));
            *a += d[u][p] * v[u][p];
        }
    }
}

template <int K, int R4>
__device__ __forceinline__ void fwd_rel4_edges(int e0, int e1, const int32_t *__restrict__ idx,
                                               const float *__restrict__ val,
                                               const float *__restrict__ data,
                                               const uint8_t *__restrict__ sel, float *acc)
{
    using C = Rel4<K, R4>;
    constexpr int R = C::R, L = C::L, EPS = C::EPS, PASSES = C::PASSES, U = C::U;
    const int lane = lane_id();
    const int slot = EPS > 1 ? lane / L : 0;
    float *my = acc + slot * C::ROW;
    for (int base = e0; base < e1; base += kWave) {
        const int n = __builtin_amdgcn_readfirstlane((e1 - base) < kWave ? (e1 - base) : kWave);
        const int my_c = lane < n ? __builtin_nontemporal_load(idx + base + lane) : 0;
        if constexpr (EPS == 1) {
            int s0 = 0;
            for (; s0 + U <= n; s0 += U)
                rel4_round_uniform<K, R4, true>(my_c, base, s0, n, val, data, sel, my);
            if (s0 < n) rel4_round_uniform<K, R4, false>(my_c, base, s0, n, val, data, sel, my);
        } else {
            for (int s0 = 0; s0 < n; s0 += U * EPS) {
                float d[U][PASSES];
                uint32_t col[U][PASSES];
                f4 v[U][PASSES];
                bool ok[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int t = s0 + u * EPS + slot;
                    ok[u] = t < n;
                    const int c = __shfl(my_c, t < kWave ? t : 0);
#pragma unroll
                    for (int p = 0; p < PASSES; ++p) {
                        const int item = lane % L;
                        const int j = item % K, rq = item / K;
                        if (ok[u]) {
                            const size_t off = (size_t)c * K + j;
                            d[u][p] = data[off];
                            col[u][p] = sel[off];
                            v[u][p] = *reinterpret_cast<const f4 *>(val + (size_t)(base + t) * R + 4 * rq);
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    if (!ok[u]) continue;
#pragma unroll
                    for (int p = 0; p < PASSES; ++p) {
                        const int rq = (lane % L) / K;
                        f4 *a = reinterpret_cast<f4 *>(my + C::off(col[u][p], rq));
                        *a += d[u][p] * v[u][p];
                    }
                }
            }
        }
    }
}

// Sum the row copies of the [col][R] accumulator, store relation q's row to
// dst + q * rel_stride, zero the copies.
template <int K, int R4>
__device__ __forceinline__ void flush_rel4(float *acc, float *__restrict__ dst, size_t rel_stride,
                                           int dim)
{
    using C = Rel4<K, R4>;
    constexpr int R = C::R;
    const int lane = lane_id();
    wave_sync_lds();
    const int d4 = (dim + 3) >> 2;
    for (int i = lane; i < R * d4; i += kWave) {
        const int q = i / d4, c4 = i - q * d4;
        f4 s = f4{0.f, 0.f, 0.f, 0.f};
        for (int cp = 0; cp < C::EPS; ++cp) {
            float *b = acc + cp * C::ROW + (q & 3);
            const int c0 = 4 * c4;
            float *b0 = b + C::off(c0, q >> 2), *b1 = b + C::off(c0 + 1, q >> 2);
            float *b2 = b + C::off(c0 + 2, q >> 2), *b3 = b + C::off(c0 + 3, q >> 2);
            s.x += *b0; s.y += *b1; s.z += *b2; s.w += *b3;
            *b0 = 0.f; *b1 = 0.f; *b2 = 0.f; *b3 = 0.f;
        }
        float *o = dst + q * rel_stride + 4 * c4;
        if ((dim & 3) == 0) {
            *reinterpret_cast<f4 *>(o) = s;
        } else {
            const float sv[4] = {s.x, s.y, s.z, s.w};
            for (int t = 0; t < 4 && 4 * c4 + t < dim; ++t) o[t] = sv[t];
        }
    }
    wave_sync_lds();
}

template <int K, int R4>
__global__ __launch_bounds__(kBlock) void fwd_rel4_panel_kernel(
    const int2 *__restrict__ sched, int64_t num_panels, const int32_t *__restrict__ indptr,
    const int32_t *__restrict__ idx, const float *__restrict__ val,
    const float *__restrict__ data, const uint8_t *__restrict__ sel, int num_rows, int dim,
    float *__restrict__ out, float *__restrict__ carry, int32_t *__restrict__ carry_row)
{
    using C = Rel4<K, R4>;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int dimp = (dim + 3) & ~3;
    float *acc = lds + (threadIdx.x / kWave) * C::EPS * C::ROW;
    const int64_t w = (int64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave;
    if (w >= num_panels) return;
    zero_lds(acc, C::EPS * C::ROW);
    const size_t rs = (size_t)num_rows * dim;
    const int2 a = sched[w], b = sched[w + 1];
    const int i0 = a.x, j0 = a.y, i1 = b.x, j1 = b.y;
    int e = j0;
    for (int r = i0; r < i1; ++r) {
        const int re = indptr[r + 1];
        if (e < re) fwd_rel4_edges<K, R4>(e, re, idx, val, data, sel, acc);
        flush_rel4<K, R4>(acc, out + (size_t)r * dim, rs, dim);
        e = re;
    }
    int has_carry = 0;
    if (i1 < num_rows) {
        const int eb = e > indptr[i1] ? e : indptr[i1];
        if (eb < j1) {
            fwd_rel4_edges<K, R4>(eb, j1, idx, val, data, sel, acc);
            has_carry = 1;
        }
    }
    if (has_carry) {
        flush_rel4<K, R4>(acc, carry + (size_t)w * C::R * dimp, dimp, dimp);
        if (lane_id() == 0) carry_row[w] = i1;
    } else if (lane_id() == 0) {
        carry_row[w] = -1;
    }
}

template <int K>
__global__ __launch_bounds__(kBlock) void fwd_multi_panel_kernel(
    const int2 *__restrict__ sched, int64_t num_panels, const int32_t *__restrict__ indptr,
    const int32_t *__restrict__ idx, const float *__restrict__ val, int R,
    const float *__restrict__ data, const uint8_t *__restrict__ sel, int num_rows, int dim,
    float *__restrict__ out, float *__restrict__ carry, int32_t *__restrict__ carry_row)
{
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int dimp = (dim + 3) & ~3;
    float *acc = lds + (threadIdx.x / kWave) * R * kMultiRow;
    const int64_t w = (int64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave;
    if (w >= num_panels) return;
    zero_lds(acc, R * kMultiRow);
    const size_t rs = (size_t)num_rows * dim;  // relation stride of the output
    const int2 a = sched[w], b = sched[w + 1];
    const int i0 = a.x, j0 = a.y, i1 = b.x, j1 = b.y;
    int e = j0;
    for (int r = i0; r < i1; ++r) {
        const int re = indptr[r + 1];
        if (e < re) fwd_multi_edges<K>(e, re, R, idx, val, data, sel, acc);
        flush_multi(acc, R, out + (size_t)r * dim, rs, dim);
        e = re;
    }
    int has_carry = 0;
    if (i1 < num_rows) {
        const int eb = e > indptr[i1] ? e : indptr[i1];
        if (eb < j1) {
            fwd_multi_edges<K>(eb, j1, R, idx, val, data, sel, acc);
            has_carry = 1;
        }
    }
    if (has_carry) {
        flush_multi(acc, R, carry + (size_t)w * R * dimp, dimp, dimp);
        if (lane_id() == 0) carry_row[w] = i1;
    } else if (lane_id() == 0) {
        carry_row[w] = -1;
    }
}

// warp4-driven forward (drop-in for the reference launcher).  A wave takes a
// run of `run` consecutive chunks; rows entirely inside the run are added
// with plain read-modify-write, rows crossing a run edge with global atomics.
// Requires the chunks of a row to be consecutive (generate_meta.py order).
template <int K>
__global__ __launch_bounds__(kBlock) void fwd_warp4_kernel(
    const int4 *__restrict__ warp4, int num_warps, int run, const int32_t *__restrict__ idx,
    const float *__restrict__ val, const float *__restrict__ data,
    const uint8_t *__restrict__ sel, int dim, int k, float *__restrict__ out)
{
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int copies = fwd_copies<K>(k);
    float *acc = lds + (threadIdx.x / kWave) * copies * kMaxDim;
    const int64_t w = (int64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave;
    const int64_t q0 = w * run;
    if (q0 >= num_warps) return;
    const int q1 = (int)((q0 + run) < num_warps ? (q0 + run) : num_warps);
    zero_lds(acc, copies * kMaxDim);
    const int head_row = q0 > 0 ? warp4[q0 - 1].x : -1;
    const int tail_row = q1 < num_warps ? warp4[q1].x : -1;
    int cur = -1;
    for (int q = (int)q0; q < q1; ++q) {
        const int4 ch = warp4[q];
        if (ch.x != cur) {
            if (cur >= 0) {
                float *dst = out + (size_t)cur * dim;
                if (cur == head_row) flush_row<kAtomic>(acc, copies, dst, dim);
                else flush_row<kAdd>(acc, copies, dst, dim);
            }
            cur = ch.x;
        }
        fwd_edges<K>(ch.y, ch.y + ch.z, k, idx, val, data, sel, acc);
    }
    if (cur >= 0) {
        float *dst = out + (size_t)cur * dim;
        if (cur == head_row || cur == tail_row) flush_row<kAtomic>(acc, copies, dst, dim);
        else flush_row<kAdd>(acc, copies, dst, dim);
    }
}

// ---------------------------------------------------------------------------
// Backward
// ---------------------------------------------------------------------------
// Stage G[r, 0:dim] into the wave's LDS row.
__device__ __forceinline__ void stage_row(float *gs, const float *__restrict__ g, int dim)
{
    wave_sync_lds();
    const int lane = lane_id();
    if ((dim & 3) == 0) {
        for (int c4 = lane; c4 < (dim >> 2); c4 += kWave)
            reinterpret_cast<f4 *>(gs)[c4] = reinterpret_cast<const f4 *>(g)[c4];
    } else {
        for (int c = lane; c < dim; c += kWave) gs[c] = g[c];
    }
    // selector bytes >= dim (invalid input) read 0: every algorithm then gives
    // such an entry no contribution, as LOCAL and the forward do
    for (int c = dim + lane; c < kMaxDim; c += kWave) gs[c] = 0.f;
    wave_sync_lds();
}

#ifndef BWD_ATOMIC_U
#define BWD_ATOMIC_U 8  // selector loads in flight (4 / 8 / 16 measured equal)
#endif

// ATOMIC push over one edge range of row r (G[r] already staged in gs).
__device__ __forceinline__ void bwd_edges_atomic(int e0, int e1, int k,
                                                 const int32_t *__restrict__ idx,
                                                 const float *__restrict__ val,
                                                 const uint8_t *__restrict__ sel,
                                                 const float *gs, float *__restrict__ dxs)
{
    const int lane = lane_id();
    if (k <= kWave) {
        const int eps = kWave / k;
        const int slot = lane / k, l = lane % k;
        for (int base = e0; base < e1; base += kWave) {
            const int n = (e1 - base) < kWave ? (e1 - base) : kWave;
            int my_c = 0;
            float my_v = 0.f;
            if (lane < n) {
                my_c = __builtin_nontemporal_load(idx + base + lane);
                my_v = __builtin_nontemporal_load(val + base + lane);
            }
            for (int s = 0; s < n; s += eps) {
                const int t = s + slot;
                const int c = __shfl(my_c, t < kWave ? t : 0);
                const float v = __shfl(my_v, t < kWave ? t : 0);
                if (slot < eps && t < n) {
                    const size_t off = (size_t)c * k + l;
                    gbl_add(dxs + off, v * gs[sel[off]]);
                }
            }
        }
    } else {
        for (int e = e0; e < e1; ++e) {
            const int c = idx[e];
            const float v = val[e];
            for (int l = lane; l < k; l += kWave) {
                const size_t off = (size_t)c * k + l;
                gbl_add(dxs + off, v * gs[sel[off]]);
            }
        }
    }
}

// ATOMIC push with the coalesced lane mapping of bwd_edges_atomic (lane l ->
// column l of an edge, so one atomic instruction covers contiguous floats) and
// U selector loads in flight (products k=16: 7.38 -> 6.08 ms, k=32: 13.2 ->
// 12.6; at k >= 16 the chip's float-atomic rate, ~320 G/s, is the bound).
template <int K>
__device__ __forceinline__ void bwd_edges_atomic_u(int e0, int e1, const int32_t *__restrict__ idx,
                                                   const float *__restrict__ val,
                                                   const uint8_t *__restrict__ sel,
                                                   const float *gs, float *__restrict__ dxs)
{
    constexpr int EPS = kWave / K;
    constexpr int STEPS = kWave / EPS;
    constexpr int U = STEPS < BWD_ATOMIC_U ? STEPS : BWD_ATOMIC_U;
    const int lane = lane_id();
    const int slot = lane / K, l = lane % K;
    for (int base = e0; base < e1; base += kWave) {
        const int n = (e1 - base) < kWave ? (e1 - base) : kWave;
        int my_c = 0;
        float my_v = 0.f;
        if (lane < n) {
            my_c = __builtin_nontemporal_load(idx + base + lane);
            my_v = __builtin_nontemporal_load(val + base + lane);
        }
#pragma unroll
        for (int s0 = 0; s0 < STEPS; s0 += U) {
            if (s0 * EPS >= n) break;
            uint32_t sb[U];
            int cs[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int t = (s0 + u) * EPS + slot;
                cs[u] = __shfl(my_c, t);
                sb[u] = t < n ? sel[(size_t)cs[u] * K + l] : 0u;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int t = (s0 + u) * EPS + slot;
                const float v = __shfl(my_v, t);
                if (t < n) gbl_add(dxs + (size_t)cs[u] * K + l, v * gs[sb[u]]);
            }
        }
    }
}

// STAGED push: P[csc_pos[e], 0:K] = val[e] * G[r, sel[c, 0:K]], K/4 lanes per
// edge, 4 selected columns per lane, U selector loads in flight.
// (The same lane mapping with 4 float atomics per lane for ATOMIC measured 4x
// slower: lane-strided atomics do not coalesce.)
// ESEL: sel holds the edge selectors (uint8[E, K], CSR edge order, written by
// the forward): read sequentially at the edge's own index instead of gathered
// at its destination's row.
// P rows are padded to KP floats: at K = 8 a 32-B row is half a 64-B DRAM
// sector, and scattered half-sector writes cost a read-modify-write (products
// k=8 STAGED 6.2 ms); a full 64-B row (zeros in the pad) is written whole.
template <int K>
struct PRow {
    static constexpr int KP = K == 8 ? 16 : K;
};

// Where the products go (PM): kPmCsc -- P[csc_pos[e]], rows padded (PRow);
// kPmEdge -- P rows in edge (CSR) order, P[e], written as one sequential stream
// (unpadded; the EDGE_GATHER segmented sum gathers them per destination);
// kPmBin -- P[bin_pos[e]], unpadded: the BINNED backward's destination bins,
// each bin's slots in (XCD, edge) order (maxk_bin_plan_build), so the rows a
// wave scatters land in lines its XCD's L2 fills before writing them back --
// plain stores, to be combined there (non-temporal ones would go out as
// partial lines).
constexpr int kPmCsc = 0, kPmEdge = 1, kPmBin = 2, kPmAppend = 3;

// kPmAppend -- the APPEND backward (MAXK_BWD_APPEND): the edge's products are
// appended, in arrival order, to its destination bin's region for this
// workgroup's XCD group (blockIdx % 8): one returning atomic per edge on the
// region's cursor (line-padded, initialised to the region's first entry by
// append_reset_kernel) gives the entry index, then the destination (4 B) and the
// K products go out as plain stores.  All appends of one XCD group to one bin
// land at that region's single write frontier, so its L2 gathers them into whole
// lines before they leave (the round-3 BINNED kept deterministic slots instead,
// and with ~25 partly written lines per bin segment they left L2 half-written:
// DESIGN §5).  The order in a region is the arrival order -- non-deterministic,
// as the reference's atomicAdd K2 (spmm_maxk_backward.cu:80,101).
struct AppendArgs {
    uint32_t magic;             // floor(2^32 / bin_size): bin = c / bin_size via umulhi + fixup
    int bin_size;
    int32_t *cursor;            // [num_bins * 8 * kCursorStride]
    int32_t *dst;               // [E] destination of each entry
};
constexpr int kCursorStride = 32;  // one 128-B line per cursor
constexpr size_t kAppendLds = 160 * 1024;   // phase 2: a bin's rows in one workgroup's LDS
constexpr int kAppendGroups = 8;   // XCD groups: blockIdx % 8

__device__ __forceinline__ int append_bin(int c, const AppendArgs &ap)
{
    int q = (int)__umulhi((uint32_t)c, ap.magic);
    if (c - q * ap.bin_size >= ap.bin_size) ++q;
    return q;
}

// The STAGED push's edge stream one batch ahead (BWD_PF, the forward's FwdPf
// with the staging position): on entry the lane's (column, value, position) of
// the batch that starts at e0, on return those of the batch that starts at e1;
// the panel kernel also loads the next row's gradient row during this row's
// gathers.  Used with node selectors at k <= 16 only (products k=16 STAGED
// 6.45 -> 6.28 ms, k=8 6.23 -> 6.02): the edge-selector forms (STAGED_EDGE,
// EDGE_GATHER phase 1) and k = 32 lost 2-4 % with it.
#ifndef BWD_PF
#define BWD_PF 1
#endif
template <int K, bool ESEL, int PM>
constexpr bool bwd_pf_on()
{
    return BWD_PF && K > 0 && K <= 16 && !ESEL && PM == kPmCsc;
}
struct BwdPf {
    int c = 0, p = 0;
    float v = 0.f;
};
template <bool CSRP>
__device__ __forceinline__ void bwd_pf_load(BwdPf &pf, int b, int pend,
                                            const int32_t *__restrict__ idx,
                                            const float *__restrict__ val,
                                            const int32_t *__restrict__ csc_pos)
{
    const int e = b + lane_id();
    pf.c = 0;
    pf.p = 0;
    pf.v = 0.f;
    if (e < pend) {
        pf.c = __builtin_nontemporal_load(idx + e);
        pf.v = __builtin_nontemporal_load(val + e);
        pf.p = CSRP ? e : __builtin_nontemporal_load(csc_pos + e);
    }
}

template <int K, bool ESEL = false, int PM = kPmCsc, bool PF = false>
__device__ __forceinline__ void bwd_edges_stage_vec(int e0, int e1,
                                                    const int32_t *__restrict__ idx,
                                                    const float *__restrict__ val,
                                                    const int32_t *__restrict__ csc_pos,
                                                    const uint8_t *__restrict__ sel,
                                                    const float *gs, float *__restrict__ P,
                                                    const AppendArgs &ap = AppendArgs{},
                                                    BwdPf *pf = nullptr, int pend = 0)
{
    constexpr bool CSRP = PM == kPmEdge || PM == kPmAppend;
    constexpr bool APP = PM == kPmAppend;
    constexpr int KP = PM == kPmCsc ? PRow<K>::KP : K;
    constexpr int LPE = KP / 4;
    constexpr int EPS = kWave / LPE;
    constexpr int STEPS = kWave / EPS;
    constexpr int U = STEPS < 8 ? STEPS : 8;
    const int lane = lane_id();
    const int sub = lane % LPE;
    const int slot = lane / LPE;
    for (int base = e0; base < e1; base += kWave) {
        const int n = (e1 - base) < kWave ? (e1 - base) : kWave;
        int my_c = 0, my_p = 0;
        float my_v = 0.f;
        if constexpr (PF) {
            my_c = pf->c;
            my_v = pf->v;
            my_p = pf->p;
            bwd_pf_load<CSRP>(*pf, base + kWave < e1 ? base + kWave : e1, pend, idx, val, csc_pos);
        } else if (lane < n) {
            my_c = __builtin_nontemporal_load(idx + base + lane);
            my_v = __builtin_nontemporal_load(val + base + lane);
            my_p = CSRP ? base + lane : __builtin_nontemporal_load(csc_pos + base + lane);
        }
#pragma unroll
        for (int s0 = 0; s0 < STEPS; s0 += U) {
            if (s0 * EPS >= n) break;
            uint32_t sb[U];
            int cu[U], slot_at[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int t = (s0 + u) * EPS + slot;
                const int c = __shfl(my_c, t < kWave ? t : 0);
                const size_t row = ESEL ? (size_t)(base + t) : (size_t)c;
                sb[u] = t < n && sub * 4 < K
                            ? *reinterpret_cast<const uint32_t *>(sel + row * K + sub * 4) : 0u;
                if constexpr (APP) {  // the entry's place: the U atomics in flight together
                    cu[u] = c;
                    slot_at[u] = 0;
                    if (t < n && sub == 0)
                        slot_at[u] = atomicAdd(ap.cursor + ((size_t)append_bin(c, ap) * kAppendGroups +
                                                            (blockIdx.x & (kAppendGroups - 1))) *
                                                               kCursorStride, 1);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int t = (s0 + u) * EPS + slot;
                const int p = APP ? __shfl(slot_at[u], slot * LPE) : __shfl(my_p, t < kWave ? t : 0);
                const float v = __shfl(my_v, t < kWave ? t : 0);
                if (t < n) {
                    f4 o = f4{0.f, 0.f, 0.f, 0.f};
                    if (sub * 4 < K) {
                        o.x = v * gs[sb[u] & 0xff];
                        o.y = v * gs[(sb[u] >> 8) & 0xff];
                        o.z = v * gs[(sb[u] >> 16) & 0xff];
                        o.w = v * gs[sb[u] >> 24];
                    }
                    // non-temporal: plain stores measured slower (Reddit 6.60 -> 6.97 ms,
                    // products 7.85 -> 8.20 ms): the staging lines would evict selector lines
                    f4 *dst = reinterpret_cast<f4 *>(P + (size_t)p * KP + sub * 4);
#ifndef MAXK_BIN_NT_STORE
                    if constexpr (PM == kPmBin || PM == kPmAppend) {
                        // plain stores: combined into lines in L2 (see kPmAppend)
                        *dst = o;
                        if (APP && sub == 0) ap.dst[p] = cu[u];
                    } else
#endif
                        __builtin_nontemporal_store(o, dst);
                }
            }
        }
    }
}

__device__ __forceinline__ void bwd_edges_stage_scalar(int e0, int e1, int k,
                                                       const int32_t *__restrict__ idx,
                                                       const float *__restrict__ val,
                                                       const int32_t *__restrict__ csc_pos,
                                                       const uint8_t *__restrict__ sel,
                                                       const float *gs, float *__restrict__ P,
                                                       bool esel)
{
    const int lane = lane_id();
    for (int e = e0; e < e1; ++e) {
        const size_t row = esel ? (size_t)e : (size_t)idx[e];
        const float v = val[e];
        const size_t p = (size_t)csc_pos[e];
        for (int l = lane; l < k; l += kWave) P[p * k + l] = v * gs[sel[row * k + l]];
    }
}

// Panel-scheduled backward push (ATOMIC when P == nullptr, STAGED otherwise).
template <int K, bool STAGED, bool ESEL = false, int PM = kPmCsc>
__global__ __launch_bounds__(kBlock) void bwd_panel_kernel(
    const int2 *__restrict__ sched, int64_t num_panels, const int32_t *__restrict__ indptr,
    const int32_t *__restrict__ idx, const float *__restrict__ val,
    const float *__restrict__ grad, const uint8_t *__restrict__ sel,
    const int32_t *__restrict__ csc_pos, int num_rows, int dim, int k,
    float *__restrict__ dxs, float *__restrict__ P)
{
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float *gs = lds + (threadIdx.x / kWave) * kMaxDim;
    zero_lds(gs, kMaxDim);  // columns >= dim read as 0
    const int64_t w = (int64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave;
    if (w >= num_panels) return;
    const int2 a = sched[w], b = sched[w + 1];
    const int i0 = a.x, j0 = a.y, i1 = b.x, j1 = b.y;
    const int rlast = i1 < num_rows ? i1 : num_rows - 1;
    if constexpr (STAGED && bwd_pf_on<K, ESEL, PM>()) {
        if (dim == kMaxDim) {
            // the next row's gradient row and edge batch loaded while this row's
            // selector gathers run: one f4 of G per lane, one BwdPf per lane
            constexpr bool CSRP = PM == kPmEdge || PM == kPmAppend;
            const int lane = lane_id();
            f4 gn = f4{0.f, 0.f, 0.f, 0.f};
            int gn_row = -1;
            BwdPf pf;
            bool first = true;
            for (int r = i0; r <= rlast; ++r) {
                const int rb = indptr[r], re = indptr[r + 1];
                const int eb = rb > j0 ? rb : j0;
                const int ee = re < j1 ? re : j1;
                if (eb >= ee) continue;
                if (gn_row != r)
                    gn = __builtin_nontemporal_load(reinterpret_cast<const f4 *>(grad + (size_t)r * dim) + lane);
                if (first) {
                    bwd_pf_load<CSRP>(pf, eb, j1, idx, val, csc_pos);
                    first = false;
                }
                wave_sync_lds();
                reinterpret_cast<f4 *>(gs)[lane] = gn;
                wave_sync_lds();
                if (r < rlast) {
                    gn = __builtin_nontemporal_load(reinterpret_cast<const f4 *>(grad + (size_t)(r + 1) * dim) + lane);
                    gn_row = r + 1;
                }
                bwd_edges_stage_vec<K, ESEL, PM, true>(eb, ee, idx, val, csc_pos, sel, gs, P,
                                                       AppendArgs{}, &pf, j1);
            }
            return;
        }
    }
    for (int r = i0; r <= rlast; ++r) {
        const int rb = indptr[r], re = indptr[r + 1];
        const int eb = rb > j0 ? rb : j0;
        const int ee = re < j1 ? re : j1;
        if (eb >= ee) continue;
        stage_row(gs, grad + (size_t)r * dim, dim);
        if constexpr (STAGED) {
            if constexpr (K > 0)
                bwd_edges_stage_vec<K, ESEL, PM>(eb, ee, idx, val, csc_pos, sel, gs, P);
            else
                bwd_edges_stage_scalar(eb, ee, k, idx, val, csc_pos, sel, gs, P, ESEL);
        } else {
            if constexpr (K >= 1 && K <= kWave)
                bwd_edges_atomic_u<K>(eb, ee, idx, val, sel, gs, dxs);
            else
                bwd_edges_atomic(eb, ee, k, idx, val, sel, gs, dxs);
        }
    }
}

// ---------------------------------------------------------------------------
// Multi-relation STAGED backward (config 5, ogbn-proteins R = 8; the backward
// of maxk_spgemm_forward_multi):
//   dXs[c,l] = sum_q sum_{e: idx[e]=c} val[e,q] * G_q[row(e), sel[c,l]].
// dXs has no relation axis, so the relation sum is taken per EDGE, in
// registers, before anything leaves the CU: phase 1 stages the R gradient rows
// of a source row in LDS relation-innermost and writes one product row per
// edge, P[e, l] = sum_q val[e,q] * G_q[r, sel[c,l]] -- the staging row of the
// single-relation STAGED (PM = kPmCsc) or EDGE_GATHER (kPmEdge) backward -- so
// phase 2 is that backward's segmented sum.  Per edge: R*4 B of values, 4 B
// index, a k-byte selector piece (the V*k table is cache-resident on
// proteins) and one staging row out and back; the R gradient rows of a source
// row are read once per panel.  (The composed backward makes R such passes;
// LOCAL rel8 gathers 32 B of interleaved gradient per selected entry.)
//
// LDS: per wave one 256-column row of R floats per column = R/4 16-B slots
// per column.  A 256-B bank row holds 64/R columns, so the ds_read_b128 of
// slot s at random columns would use only 16/(R/4) slot positions of the
// bank row; slot s of column j is stored at s ^ ((j / (64/R)) % (R/4)), so
// over j the reads of one logical slot cover all 16 positions.
// ---------------------------------------------------------------------------
template <int R>
struct RelLds {
    static constexpr int NS = R / 4;    // 16-B slots per column
    static constexpr int CPB = 64 / R;  // columns per 256-B bank row
    static __device__ __forceinline__ uint32_t off(uint32_t j, int s)
    {
        return j * (R * 4) + (((uint32_t)s ^ ((j / CPB) % NS)) << 4);
    }
};

// G_q[r, 0:dim] for q < R into the wave's LDS row (columns >= dim read as 0,
// the rule of stage_row).  dim % 4 == 0.
template <int R>
__device__ __forceinline__ void stage_rel_rows(char *gs, const float *__restrict__ grad,
                                               int64_t plane, int r, int dim)
{
    wave_sync_lds();
    const int j0 = lane_id() * 4;  // 64 lanes x 4 columns
    const float *g0 = grad + (size_t)r * dim + j0;
#pragma unroll
    for (int s = 0; s < R / 4; ++s) {
        f4 g[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
            g[i] = j0 < dim ? *reinterpret_cast<const f4 *>(g0 + (size_t)(4 * s + i) * plane)
                            : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < 4; ++c)
            *reinterpret_cast<f4 *>(gs + RelLds<R>::off(j0 + c, s)) =
                f4{g[0][c], g[1][c], g[2][c], g[3][c]};
    }
    wave_sync_lds();
}

// One source row's edge range [e0, e1): KP/4 lanes per edge, 4 selected
// columns per lane (as bwd_edges_stage_vec), the edge's R values loaded once
// by the lane that owns the edge and shuffled to the edge's lanes.
template <int K, int R, int PM>
__device__ __forceinline__ void bwd_multi_edges(int e0, int e1, const int32_t *__restrict__ idx,
                                                const float *__restrict__ val,
                                                const int32_t *__restrict__ csc_pos,
                                                const uint8_t *__restrict__ sel, const char *gs,
                                                float *__restrict__ P,
                                                const AppendArgs &ap = AppendArgs{})
{
    constexpr bool CSRP = PM == kPmEdge || PM == kPmAppend;
    constexpr bool APP = PM == kPmAppend;
    constexpr int KP = PM == kPmCsc ? PRow<K>::KP : K;
    constexpr int LPE = KP / 4;
    constexpr int EPS = kWave / LPE;
    constexpr int STEPS = kWave / EPS;
    constexpr int U = STEPS < 8 ? STEPS : 8;
    constexpr int NS = R / 4;
    const int lane = lane_id();
    const int sub = lane % LPE;
    const int slot = lane / LPE;
    for (int base = e0; base < e1; base += kWave) {
        const int n = (e1 - base) < kWave ? (e1 - base) : kWave;
        int my_c = 0, my_p = 0;
        f4 my_v[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) my_v[s] = f4{0.f, 0.f, 0.f, 0.f};
        if (lane < n) {
            my_c = __builtin_nontemporal_load(idx + base + lane);
            my_p = CSRP ? base + lane : __builtin_nontemporal_load(csc_pos + base + lane);
            const f4 *vp = reinterpret_cast<const f4 *>(val + (size_t)(base + lane) * R);
#pragma unroll
            for (int s = 0; s < NS; ++s) my_v[s] = __builtin_nontemporal_load(vp + s);
        }
#pragma unroll
        for (int s0 = 0; s0 < STEPS; s0 += U) {
            if (s0 * EPS >= n) break;
            uint32_t sb[U];
            int cu[U], slot_at[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int t = (s0 + u) * EPS + slot;
                const int c = __shfl(my_c, t);
                sb[u] = t < n && sub * 4 < K
                            ? *reinterpret_cast<const uint32_t *>(sel + (size_t)c * K + sub * 4)
                            : 0u;
                if constexpr (APP) {
                    cu[u] = c;
                    slot_at[u] = 0;
                    if (t < n && sub == 0)
                        slot_at[u] = atomicAdd(ap.cursor + ((size_t)append_bin(c, ap) * kAppendGroups +
                                                            (blockIdx.x & (kAppendGroups - 1))) *
                                                               kCursorStride, 1);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int t = (s0 + u) * EPS + slot;
                const int p = APP ? __shfl(slot_at[u], slot * LPE) : __shfl(my_p, t);
                f4 v[NS];
#pragma unroll
                for (int s = 0; s < NS; ++s)
                    v[s] = f4{__shfl(my_v[s].x, t), __shfl(my_v[s].y, t), __shfl(my_v[s].z, t),
                              __shfl(my_v[s].w, t)};
                if (t < n) {
                    f4 o = f4{0.f, 0.f, 0.f, 0.f};
                    if (sub * 4 < K) {
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const uint32_t j = (sb[u] >> (8 * i)) & 0xffu;
                            float acc = 0.f;
#pragma unroll
                            for (int s = 0; s < NS; ++s) {
                                const f4 g = *reinterpret_cast<const f4 *>(gs + RelLds<R>::off(j, s));
                                acc = fmaf(v[s].x, g.x, acc);
                                acc = fmaf(v[s].y, g.y, acc);
                                acc = fmaf(v[s].z, g.z, acc);
                                acc = fmaf(v[s].w, g.w, acc);
                            }
                            o[i] = acc;
                        }
                    }
                    if constexpr (APP) {   // plain stores: combined into lines in L2
                        *reinterpret_cast<f4 *>(P + (size_t)p * KP + sub * 4) = o;
                        if (sub == 0) ap.dst[p] = cu[u];
                    } else {
                        __builtin_nontemporal_store(
                            o, reinterpret_cast<f4 *>(P + (size_t)p * KP + sub * 4));
                    }
                }
            }
        }
    }
}

template <int K, int R, int PM>
__global__ __launch_bounds__(kBlock) void bwd_multi_stage_kernel(
    const int2 *__restrict__ sched, int64_t num_panels, const int32_t *__restrict__ indptr,
    const int32_t *__restrict__ idx, const float *__restrict__ val,
    const float *__restrict__ grad, int64_t plane, const uint8_t *__restrict__ sel,
    const int32_t *__restrict__ csc_pos, int num_rows, int dim, float *__restrict__ P)
{
    extern __shared__ __attribute__((aligned(16))) float lds[];
    char *gs = reinterpret_cast<char *>(lds + (threadIdx.x / kWave) * (kMaxDim * R));
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
        stage_rel_rows<R>(gs, grad, plane, r, dim);
        bwd_multi_edges<K, R, PM>(eb, ee, idx, val, csc_pos, sel, gs, P);
    }
}

// ---------------------------------------------------------------------------
// APPEND backward (MAXK_BWD_APPEND): write-combined
// propagation blocking.  Phase 1 is the STAGED push with the products appended
// to destination bins (kPmAppend above); phase 2 streams each bin's entries
// once and sums them into the bin's LDS rows with LDS float atomics, then
// writes the bin's dXs rows whole.  Bin b holds destinations [b*bin_size,
// (b+1)*bin_size), bin_size*K*4 <= 160 KB; its 8 regions (one per XCD group)
// are consecutive, so a bin is one contiguous range of entries
// [region_base[8b], region_base[8b+8]).  Per edge: 4 + 4K bytes out in phase 1
// and back in phase 2, against STAGED's random 64-B+ row stores and the CSC
// segmented sum.  Sum order: arrival order (non-deterministic).
// ---------------------------------------------------------------------------
template <int K, bool ESEL>
__global__ __launch_bounds__(kBlock) void bwd_append_kernel(
    const int2 *__restrict__ sched, int64_t num_panels, const int32_t *__restrict__ indptr,
    const int32_t *__restrict__ idx, const float *__restrict__ val,
    const float *__restrict__ grad, const uint8_t *__restrict__ sel, int num_rows, int dim,
    float *__restrict__ P, AppendArgs ap)
{
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float *gs = lds + (threadIdx.x / kWave) * kMaxDim;
    zero_lds(gs, kMaxDim);  // columns >= dim read as 0
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
        stage_row(gs, grad + (size_t)r * dim, dim);
        bwd_edges_stage_vec<K, ESEL, kPmAppend>(eb, ee, idx, val, nullptr, sel, gs, P, ap);
    }
}

template <int K, int R>
__global__ __launch_bounds__(kBlock) void bwd_multi_append_kernel(
    const int2 *__restrict__ sched, int64_t num_panels, const int32_t *__restrict__ indptr,
    const int32_t *__restrict__ idx, const float *__restrict__ val,
    const float *__restrict__ grad, int64_t plane, const uint8_t *__restrict__ sel,
    int num_rows, int dim, float *__restrict__ P, AppendArgs ap)
{
    extern __shared__ __attribute__((aligned(16))) float lds[];
    char *gs = reinterpret_cast<char *>(lds + (threadIdx.x / kWave) * (kMaxDim * R));
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
        stage_rel_rows<R>(gs, grad, plane, r, dim);
        bwd_multi_edges<K, R, kPmAppend>(eb, ee, idx, val, nullptr, sel, gs, P, ap);
    }
}

// cursor of region j := its first entry (phase 1's atomics then return entry indices)
__global__ __launch_bounds__(kBlock) void append_reset_kernel(const int32_t *__restrict__ region_base,
                                                              int n, int32_t *__restrict__ cursor)
{
    const int j = blockIdx.x * kBlock + threadIdx.x;
    if (j < n) cursor[(size_t)j * kCursorStride] = region_base[j];
}

constexpr int kReduceThreads = 1024;

// Phase 2: one workgroup per bin.  LPE = K/4 lanes per entry (16 B each), U
// entries per lane in flight; each lane adds its 4 products to the bin's LDS rows
// with ds_add_f32.  Entries of another bin (impossible for a consistent plan) are
// skipped rather than corrupting LDS.
template <int K>
__global__ __launch_bounds__(kReduceThreads) void bwd_bin_reduce_kernel(
    const int32_t *__restrict__ region_base, int bin_size, int num_cols,
    const int32_t *__restrict__ dst, const float *__restrict__ P, float *__restrict__ dxs)
{
    extern __shared__ __attribute__((aligned(16))) float lds[];
    constexpr int LPE = K / 4;
    constexpr int EPW = kWave / LPE;   // entries per wave-instruction
    constexpr int U = 8;
    const int b = blockIdx.x;
    const int c0 = b * bin_size;
    const int nd = min(bin_size, num_cols - c0);
    const int tid = threadIdx.x;
    for (int i = tid; i < nd * LPE; i += kReduceThreads)
        reinterpret_cast<f4 *>(lds)[i] = f4{0.f, 0.f, 0.f, 0.f};
    __syncthreads();
    const int64_t e0 = region_base[(size_t)b * kAppendGroups];
    const int64_t e1 = region_base[(size_t)(b + 1) * kAppendGroups];
    const int lane = lane_id();
    const int sub = lane % LPE, slot = lane / LPE;
    const int wv = tid / kWave;
    constexpr int NW = kReduceThreads / kWave;
    for (int64_t base = e0 + (int64_t)wv * EPW * U; base < e1; base += (int64_t)NW * EPW * U) {
        int d[U];
        f4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t e = base + u * EPW + slot;
            d[u] = -1;
            if (e < e1) {
                d[u] = __builtin_nontemporal_load(dst + e) - c0;
                v[u] = __builtin_nontemporal_load(reinterpret_cast<const f4 *>(P + e * K) + sub);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if ((uint32_t)d[u] < (uint32_t)nd) {
                float *a = lds + (size_t)d[u] * K + sub * 4;
                atomicAdd(a + 0, v[u].x);
                atomicAdd(a + 1, v[u].y);
                atomicAdd(a + 2, v[u].z);
                atomicAdd(a + 3, v[u].w);
            }
        }
    }
    __syncthreads();
    f4 *out = reinterpret_cast<f4 *>(dxs + (size_t)c0 * K);
    for (int i = tid; i < nd * LPE; i += kReduceThreads)
        __builtin_nontemporal_store(reinterpret_cast<const f4 *>(lds)[i], out + i);
}

// GNNAdvisor-style SAG baseline (kernels/spmm_gnna.cu:60-140, the reference's
// speedup-table comparison; not on the MaxK path): every row's neighbours are
// cut into parts of part_size (the warp4 chunks of maxk_warp4_build with
// warp_max_nz = part_size, exactly build_part's cut, spmm_gnna.cu:20-56), one
// wave per part sums its neighbours' dense rows in registers (lane: 4 columns)
// and adds the part's partial row into the output with no-return float atomics
// (the reference stages the partial in shared memory and adds with an atomic
// exchange loop).  values == NULL: unweighted, as the reference (it passes no
// degrees); else each neighbour row is scaled by its edge value.  out must be
// zeroed.  dim % 4 == 0, dim <= 256.
__global__ __launch_bounds__(kBlock) void gnna_sag_kernel(const int4 *__restrict__ parts,
                                                          int64_t num_parts,
                                                          const int32_t *__restrict__ idx,
                                                          const float *__restrict__ val,
                                                          const float *__restrict__ x, int dim,
                                                          float *__restrict__ out)
{
    const int64_t w = (int64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave;
    if (w >= num_parts) return;
    const int lane = lane_id();
    const int4 p = parts[w];   // (row, first edge, count, 0)
    const int c4 = lane * 4;
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    if (c4 < dim) {
        for (int e = p.y; e < p.y + p.z; ++e) {
            const int nid = idx[e];
            const f4 v = *reinterpret_cast<const f4 *>(x + (size_t)nid * dim + c4);
            const float a = val ? val[e] : 1.f;
            acc += a * v;
        }
        float *o = out + (size_t)p.x * dim + c4;
        gbl_add(o, acc.x);
        gbl_add(o + 1, acc.y);
        gbl_add(o + 2, acc.z);
        gbl_add(o + 3, acc.w);
    }
}

// STAGED phase 2: dxs[c, :] = sum of P rows [csc_indptr[c], csc_indptr[c+1]),
// merge-path panels over the CSC ranges, register accumulation + cross-slot
// reduction; split destinations go through the carry fixup.
// GATHER: CSC slot q's row is P[perm[q]] (P in edge order, unpadded) instead of P[q].
template <int K, bool GATHER = false>
__device__ __forceinline__ f4 seg_sum_vec(int q0, int q1, const float *__restrict__ P,
                                          const int32_t *__restrict__ perm = nullptr)
{
    constexpr int LPE = K / 4;
    constexpr int EPS = kWave / LPE;
    const int lane = lane_id();
    const int sub = lane % LPE;
    const int slot = lane / LPE;
    constexpr int KP = GATHER ? K : PRow<K>::KP;  // P row stride
    f4 s = f4{0.f, 0.f, 0.f, 0.f};
    constexpr int U = 4;
    int q = q0 + slot;
    for (; q + (U - 1) * EPS < q1; q += U * EPS) {
        f4 t[U];
        size_t row[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            row[u] = GATHER ? (size_t)__builtin_nontemporal_load(perm + q + u * EPS)
                            : (size_t)(q + u * EPS);
#pragma unroll
        for (int u = 0; u < U; ++u)
            t[u] = __builtin_nontemporal_load(
                reinterpret_cast<const f4 *>(P + row[u] * KP + sub * 4));
#pragma unroll
        for (int u = 0; u < U; ++u) {
            s.x += t[u].x; s.y += t[u].y; s.z += t[u].z; s.w += t[u].w;
        }
    }
    for (; q < q1; q += EPS) {
        const size_t row = GATHER ? (size_t)perm[q] : (size_t)q;
        const f4 t = __builtin_nontemporal_load(
            reinterpret_cast<const f4 *>(P + row * KP + sub * 4));
        s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
    }
#pragma unroll
    for (int m = LPE; m < kWave; m <<= 1) {
        s.x += __shfl_xor(s.x, m);
        s.y += __shfl_xor(s.y, m);
        s.z += __shfl_xor(s.z, m);
        s.w += __shfl_xor(s.w, m);
    }
    return s;  // every slot holds the total for its sub
}

template <int K, bool GATHER = false>
__global__ __launch_bounds__(kBlock) void bwd_segsum_kernel(
    const int2 *__restrict__ sched, int64_t num_panels, const int32_t *__restrict__ cptr,
    const float *__restrict__ P, int num_rows, int k, float *__restrict__ dxs,
    float *__restrict__ carry, int32_t *__restrict__ carry_row,
    const int32_t *__restrict__ perm = nullptr)
{
    const int64_t w = (int64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave;
    if (w >= num_panels) return;
    const int lane = lane_id();
    const int2 a = sched[w], b = sched[w + 1];
    const int i0 = a.x, j0 = a.y, i1 = b.x, j1 = b.y;
    int e = j0;
    if constexpr (K > 0) {
        constexpr int LPE = K / 4;
        const int sub = lane % LPE;
        const bool writer = lane < LPE;
        for (int c = i0; c < i1; ++c) {
            const int ce = cptr[c + 1];
            const f4 s = seg_sum_vec<K, GATHER>(e, ce, P, perm);
            if (writer) reinterpret_cast<f4 *>(dxs + (size_t)c * K)[sub] = s;
            e = ce;
        }
        int has = 0;
        f4 s = f4{0.f, 0.f, 0.f, 0.f};
        if (i1 < num_rows) {
            const int eb = e > cptr[i1] ? e : cptr[i1];
            if (eb < j1) {
                s = seg_sum_vec<K, GATHER>(eb, j1, P, perm);
                has = 1;
            }
        }
        if (has) {
            if (writer) reinterpret_cast<f4 *>(carry + (size_t)w * K)[sub] = s;
            if (lane == 0) carry_row[w] = i1;
        } else if (lane == 0) {
            carry_row[w] = -1;
        }
    } else {
        // generic k: lane l accumulates column l (and l+64, ...)
        for (int c = i0; c < i1; ++c) {
            const int ce = cptr[c + 1];
            for (int l = lane; l < k; l += kWave) {
                float s = 0.f;
                for (int q = e; q < ce; ++q) s += P[(size_t)q * k + l];
                dxs[(size_t)c * k + l] = s;
            }
            e = ce;
        }
        int has = 0;
        if (i1 < num_rows) {
            const int eb = e > cptr[i1] ? e : cptr[i1];
            if (eb < j1) {
                for (int l = lane; l < k; l += kWave) {
                    float s = 0.f;
                    for (int q = eb; q < j1; ++q) s += P[(size_t)q * k + l];
                    carry[(size_t)w * k + l] = s;
                }
                has = 1;
            }
        }
        if (lane == 0) carry_row[w] = has ? i1 : -1;
    }
}

// Backward, warp4-driven (drop-in): atomic push, G staged per row change.
__global__ __launch_bounds__(kBlock) void bwd_warp4_kernel(
    const int4 *__restrict__ warp4, int num_warps, int run, const int32_t *__restrict__ idx,
    const float *__restrict__ val, const float *__restrict__ grad,
    const uint8_t *__restrict__ sel, int dim, int k, float *__restrict__ dxs)
{
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float *gs = lds + (threadIdx.x / kWave) * kMaxDim;
    zero_lds(gs, kMaxDim);  // columns >= dim read as 0
    const int64_t w = (int64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave;
    const int64_t q0 = w * run;
    if (q0 >= num_warps) return;
    const int q1 = (int)((q0 + run) < num_warps ? (q0 + run) : num_warps);
    int cur = -1;
    for (int q = (int)q0; q < q1; ++q) {
        const int4 ch = warp4[q];
        if (ch.x != cur) {
            stage_row(gs, grad + (size_t)ch.x * dim, dim);
            cur = ch.x;
        }
        bwd_edges_atomic(ch.y, ch.y + ch.z, k, idx, val, sel, gs, dxs);
    }
}

// ---------------------------------------------------------------------------
// Backward LOCAL: destination-owned accumulation (no atomics, no staging rows)
//
// Wave w owns destinations [dstart[w], dstart[w+1]) (D <= 256): their dXs
// rows and selector rows live in the wave's LDS for the launch.  Its in-edges
// arrive as a list sorted by SOURCE row r, packed (r | c_local<<24, val) by
// the plan builder (ops.py).  The source rows are cut into bands, one launch
// per band (first band stores dXs, later ones reload and add), so the
// gradient rows G[r] the chip reads during a launch form a window of about
// 32 MB that the Infinity Cache serves: measured 4.8 ms with a resident
// window vs 10.8 ms when every wave sweeps all of G in one launch (Reddit
// shape, uniform sources; tools/exp_local_window.py).  Per edge the K lanes of a group gather
// G[r, sel[c, l]] (global, L2) and read-modify-write dXs[c, l] in LDS.
// EPS = 64/K edges share one wave-instruction; a group whose destinations
// collide is processed one edge at a time (plain LDS RMW stays race-free).
// ---------------------------------------------------------------------------
#ifndef LOCAL_U
#define LOCAL_U 8
#endif
#ifndef LOCAL_R
#define LOCAL_R 16  // edge records per SGPR round (k = 32, 64)
#endif

// Offset (in floats) of G[row, col] -> element pointer; 32-bit byte offsets
// (global_load saddr form) when the whole gradient array is below 4 GiB.
template <bool WIDE>
__device__ __forceinline__ const float *g_at(const float *grad, uint32_t row_off, uint32_t col)
{
    if constexpr (WIDE)
        return grad + ((uint64_t)row_off + col);
    else
        return reinterpret_cast<const float *>(reinterpret_cast<const char *>(grad) +
                                               ((row_off + col) << 2));
}

// A round's gathered values and destination slots, between issue and commit.
template <int K>
struct LocalRound {
    static constexpr int EPS = kWave / K;
    static constexpr int NG = LOCAL_R / EPS;
    float gv[NG], vv[NG];
    int ai[NG];
    uint32_t clash;
};

template <int K, bool WIDE>
__device__ __forceinline__ void local_issue(const int32_t *__restrict__ rec_rc,
                                            const float *__restrict__ rec_v,
                                            const float *__restrict__ grad, uint32_t dim,
                                            const uint8_t *sl, int grp, int l, LocalRound<K> &rd)
{
    constexpr int EPS = kWave / K;
    constexpr int R = LOCAL_R;
    constexpr int NG = R / EPS;
    uint32_t ro[NG], col[NG];
    uint32_t clash = 0;
    const bool hi = EPS == 2 && grp != 0;
    // scalar part: records -> (destination slot, row offset, value) per half,
    // pinned in SGPRs (otherwise the half-select is hoisted above the
    // arithmetic and every lane pays a v_mul_lo_u32); per lane a half-select
    // is a ^ ((a ^ b) & m) with the xor scalar: two VALU ops
    int32_t rcs[R];
    uint32_t vbits[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
        rcs[i] = rec_rc[i];
        vbits[i] = __builtin_bit_cast(uint32_t, rec_v[i]);
    }
    // materialise all records here (two s_load_dwordx16, one wait)
    static_assert(R % 16 == 0, "records are pinned 16 at a time");
#pragma unroll
    for (int c = 0; c < R; c += 16) {
        int32_t *q = rcs + c;
        asm volatile("" : "+s"(q[0]), "+s"(q[1]), "+s"(q[2]), "+s"(q[3]), "+s"(q[4]), "+s"(q[5]),
                     "+s"(q[6]), "+s"(q[7]), "+s"(q[8]), "+s"(q[9]), "+s"(q[10]), "+s"(q[11]),
                     "+s"(q[12]), "+s"(q[13]), "+s"(q[14]), "+s"(q[15]));
    }
    const uint32_t m = hi ? 0xffffffffu : 0u;
#pragma unroll
    for (int u = 0; u < NG; ++u) {
        const int ra = rcs[u * EPS];
        const int rb = EPS == 2 ? rcs[u * EPS + 1] : ra;
        uint32_t sa = ((uint32_t)ra >> 24) * K, sb = ((uint32_t)rb >> 24) * K;
        uint32_t oa = (uint32_t)(ra & 0xffffff) * dim, ob = (uint32_t)(rb & 0xffffff) * dim;
        uint32_t va = vbits[u * EPS], vb = EPS == 2 ? vbits[u * EPS + 1] : va;
        if (EPS == 2 && sa == sb) clash |= 1u << u;
        uint32_t xs = sa ^ sb, xo = oa ^ ob, xv = va ^ vb;
        asm volatile("" : "+s"(sa), "+s"(oa), "+s"(va), "+s"(xs), "+s"(xo), "+s"(xv));
        if constexpr (EPS == 2) {
            rd.ai[u] = (int)(sa ^ (xs & m)) + l;
            ro[u] = oa ^ (xo & m);
            rd.vv[u] = __builtin_bit_cast(float, va ^ (xv & m));
        } else {
            rd.ai[u] = (int)sa + l;
            ro[u] = oa;
            rd.vv[u] = __builtin_bit_cast(float, va);
        }
    }
    rd.clash = clash;
    // selector bytes for all groups, then all gathers back to back
#pragma unroll
    for (int u = 0; u < NG; ++u) {
        col[u] = sl[rd.ai[u]];
    }
#pragma unroll
    for (int u = 0; u < NG; ++u) rd.gv[u] = *g_at<WIDE>(grad, ro[u], col[u]);
}

template <int K>
__device__ __forceinline__ void local_commit(const LocalRound<K> &rd, float *acc, int grp)
{
    constexpr int EPS = kWave / K;
    constexpr int NG = LocalRound<K>::NG;
#pragma unroll
    for (int u = 0; u < NG; ++u) {
        if (!((rd.clash >> u) & 1u)) {
            acc[rd.ai[u]] = fmaf(rd.vv[u], rd.gv[u], acc[rd.ai[u]]);
        } else {  // both halves target one destination: one half at a time
            for (int gg = 0; gg < EPS; ++gg) {
                if (grp == gg) acc[rd.ai[u]] = fmaf(rd.vv[u], rd.gv[u], acc[rd.ai[u]]);
                wave_sync_lds();
            }
        }
    }
}

// One round of the LOCAL loop for K in {32, 64}: R = 16 edge records held in
// SGPRs (wave-uniform loads), NG = R/EPS gathers issued back to back, then the
// NG LDS read-modify-writes.  Row offsets, destination slots and the clash
// test are scalar; per lane only the half-select (EPS = 2), the selector byte
// and the gather remain.  All R records are valid (the tail round of a wave's
// list takes the generic loop).
template <int K, bool WIDE>
__device__ __forceinline__ void local_round(const int32_t *__restrict__ rec_rc,
                                            const float *__restrict__ rec_v,
                                            const float *__restrict__ grad, uint32_t dim,
                                            const uint8_t *sl, float *acc, int grp, int l)
{
    LocalRound<K> rd;
    local_issue<K, WIDE>(rec_rc, rec_v, grad, dim, sl, grp, l, rd);
    local_commit<K>(rd, acc, grp);
}

// The generic LOCAL loop (any K dividing 64): records shuffled out of VGPRs.
template <int K>
__device__ __forceinline__ void local_edges_shfl(int e_beg, int e_end,
                                                 const int32_t *__restrict__ erc,
                                                 const float *__restrict__ evl,
                                                 const float *__restrict__ grad, int dim,
                                                 const uint8_t *sl, float *acc)
{
    constexpr int EPS = kWave / K;                 // edges per wave-instruction
    constexpr int B = EPS * 32 < kWave ? EPS * 32 : kWave;  // edges per batch
    constexpr int NG = B / EPS;                    // groups per batch (<= 32)
    const int lane = lane_id();
    const int grp = lane / K, l = lane % K;
    // records of the next batch are prefetched while the current one gathers
    int nx_rc = 0;
    float nx_v = 0.f;
    if (lane < B && e_beg + lane < e_end) {
        nx_rc = __builtin_nontemporal_load(erc + e_beg + lane);
        nx_v = __builtin_nontemporal_load(evl + e_beg + lane);
    }
    for (int base = e_beg; base < e_end; base += B) {
        const int n = (e_end - base) < B ? (e_end - base) : B;
        const int my_rc = nx_rc;
        const float my_v = nx_v;
        if (lane < B && base + B + lane < e_end) {
            nx_rc = __builtin_nontemporal_load(erc + base + B + lane);
            nx_v = __builtin_nontemporal_load(evl + base + B + lane);
        }
        // U groups of gathers in flight per round (VGPR budget vs memory-level parallelism)
        for (int g0 = 0; g0 < NG; g0 += LOCAL_U) {
            if (g0 * EPS >= n) break;
            float gv[LOCAL_U], vv[LOCAL_U];
            int cc[LOCAL_U];
            uint32_t clash = 0;  // bit u: group u has two edges into one destination
#pragma unroll
            for (int u = 0; u < LOCAL_U; ++u) {
                const int gi = g0 + u;
                const int t = gi * EPS + grp;
                int rc = __shfl(my_rc, t);
                vv[u] = __shfl(my_v, t);
                bool c = false;
#pragma unroll
                for (int j = 1; j < EPS; ++j) {
                    const int other = __shfl(rc, lane >= j * K ? lane - j * K : lane);
                    c |= (lane >= j * K) && ((other >> 24) == (rc >> 24)) && (t < n);
                }
                if (__any(c)) clash |= 1u << u;
                cc[u] = (rc >> 24) & 0xff;
                gv[u] = 0.f;
                if (t < n) {
                    gv[u] = grad[(size_t)(rc & 0xffffff) * dim + sl[cc[u] * K + l]];
                } else {
                    vv[u] = 0.f;
                    cc[u] = -1;
                }
            }
#pragma unroll
            for (int u = 0; u < LOCAL_U; ++u) {
                if ((g0 + u) * EPS >= n) break;
                if (!((clash >> u) & 1u)) {
                    if (cc[u] >= 0) acc[cc[u] * K + l] += vv[u] * gv[u];
                } else {
                    for (int gg = 0; gg < EPS; ++gg) {
                        if (grp == gg && cc[u] >= 0) acc[cc[u] * K + l] += vv[u] * gv[u];
                        wave_sync_lds();
                    }
                }
            }
        }
    }
}

template <int K, bool WIDE>
__device__ __forceinline__ void local_edges_scalar(int e_beg, int e_end,
                                                   const int32_t *__restrict__ erc,
                                                   const float *__restrict__ evl,
                                                   const float *__restrict__ grad, int dim,
                                                   const uint8_t *sl, float *acc)
{
    constexpr int R = LOCAL_R;
    const int lane = lane_id();
    const int grp = lane / K, l = lane % K;
    const int full_end = e_beg + ((e_end - e_beg) / R) * R;
    for (int base = e_beg; base < full_end; base += R) {
        local_round<K, WIDE>(erc + base, evl + base, grad, (uint32_t)dim, sl, acc, grp, l);
    }
    if (full_end < e_end) local_edges_shfl<K>(full_end, e_end, erc, evl, grad, dim, sl, acc);
}

template <int K, bool WIDE>
__global__ __launch_bounds__(kBlock) void bwd_local_kernel(
    const int32_t *__restrict__ seg_beg, const int32_t *__restrict__ seg_end, bool first,
    const int32_t *__restrict__ dstart, int num_waves,
    int dmax, const int32_t *__restrict__ erc, const float *__restrict__ evl,
    const float *__restrict__ grad, const uint8_t *__restrict__ sel, int dim,
    float *__restrict__ dxs)
{
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int wl = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int region = (dmax * K * 5 + 15) & ~15;  // bytes: fp32 dXs block + u8 sel block
    float *acc = reinterpret_cast<float *>(reinterpret_cast<char *>(lds) + wl * region);
    uint8_t *sl = reinterpret_cast<uint8_t *>(acc + dmax * K);
    const int w = blockIdx.x * kWavesPerBlock + wl;
    if (w >= num_waves) return;
    const int lane = lane_id();
    const int e_beg = __builtin_amdgcn_readfirstlane(seg_beg[w]);
    const int e_end = __builtin_amdgcn_readfirstlane(seg_end[w]);
    if (!first && e_beg == e_end) return;  // nothing to add in this band
    const int d0 = dstart[w], D = dstart[w + 1] - d0;
    const int nent = D * K;
    float *dst = dxs + (size_t)d0 * K;
    const uint8_t *srow = sel + (size_t)d0 * K;
    // selector bytes are clamped into the row for the gathers; entries that
    // were out of range are written as 0 below (they receive no contribution)
    for (int i = lane; i < nent; i += kWave) {
        acc[i] = first ? 0.f : dst[i];
        const int c = srow[i];
        sl[i] = (uint8_t)(c < dim ? c : dim - 1);
    }
    wave_sync_lds();
    if constexpr (kWave / K <= 2)
        local_edges_scalar<K, WIDE>(e_beg, e_end, erc, evl, grad, dim, sl, acc);
    else
        local_edges_shfl<K>(e_beg, e_end, erc, evl, grad, dim, sl, acc);
    wave_sync_lds();
    for (int i = lane; i < nent; i += kWave) dst[i] = srow[i] < dim ? acc[i] : 0.f;
}

// Bank-aware CBSR order for the fused multi-relation forward (relation-vector
// kernel: lane = entry j + 32 * relation quad, accumulator word col * S + 4 *
// quad with S / 4 odd).  Its ds_write_b128 goes in groups of 8 contiguous
// lanes = 8 consecutive entries, bank = 16-B unit mod 8 (MI355X_MICROARCH.md
// §LDS), so a group is conflict-free iff its 8 columns differ mod 8.  Rows are
// ordered by (occurrence of the column's residue mod 8, residue): the first 8
// entries take one column of each residue present, and so on.  Measured on
// proteins R=8: LDS bank-conflict cycles -19 %, forward 5.43 -> 5.23 ms; a
// pattern that also spreads the ds_read_b128 16-lane groups over residues mod
// 16 measured the same (random rows rarely have two columns per class).  Any
// entry order is a valid CBSR and the forward's result is bit-identical.
// One wave per row, k <= 64.
__global__ __launch_bounds__(kBlock) void cbsr_bank_order_kernel(const float *__restrict__ data,
                                                                 const uint8_t *__restrict__ sel,
                                                                 int num_rows, int k, int swz,
                                                                 float *__restrict__ odata,
                                                                 uint8_t *__restrict__ osel,
                                                                 uint16_t *__restrict__ opacked)
{
    const int lane = lane_id();
    const int64_t nwaves = (int64_t)gridDim.x * kWavesPerBlock;
    const uint64_t below = (1ull << lane) - 1ull;
    for (int64_t r = (int64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave; r < num_rows;
         r += nwaves) {
        const bool on = lane < k;
        const int c = on ? sel[r * k + lane] : 0;
        const float d = on && odata ? data[r * k + lane] : 0.f;
        if (swz == 2) {
            // the interleaved R = 8, k = 32 layout (FWD_REL8_ILV): the o-th column of
            // class c & 7 (o < 4) goes to a fixed slot of read group o (entries {0, 1,
            // 6, 7, 10..13}, {2..5, 8, 9, 14, 15}, and the same + 16), placed so that
            // every 4-entry write group holds classes of distinct c & 3; the columns
            // past a class's fourth fill the remaining slots in entry order
            const int x = c & 7;
            uint64_t mine = 0;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const uint64_t m = __ballot(on && x == q);
                if (q == x) mine = m;
            }
            const int o = __builtin_popcountll(mine & below);
            // slot of (o, x): read group o, position by class
            const int t0[8] = {0, 1, 6, 7, 10, 11, 12, 13};
            const int t1[8] = {4, 5, 2, 3, 14, 15, 8, 9};
            int slot = -1;
            if (on && o < 4) slot = ((o & 1) ? t1[x] : t0[x]) + ((o >> 1) << 4);
            uint32_t filled = slot >= 0 ? (1u << slot) : 0u;
#pragma unroll
            for (int m = 1; m < kWave; m <<= 1) filled |= (uint32_t)__shfl_xor((int)filled, m);
            const uint64_t over = __ballot(on && o >= 4);
            if (on && o >= 4) {
                int rk = __builtin_popcountll(over & below);   // this overflow entry's rank
                uint32_t holes = ~filled;
                for (; rk > 0; --rk) holes &= holes - 1u;      // drop the rk lowest holes
                slot = __builtin_ctz(holes);
            }
            if (on) {
                if (odata) odata[r * k + slot] = d;
                if (osel) osel[r * k + slot] = (uint8_t)c;
                if (opacked) opacked[r * k + slot] = (uint16_t)(c | (lane << 8));
            }
            continue;
        }
        // the 16-B unit of quad 0 mod 8: (S / 4) c with odd S / 4 (R = 4, 12, 16
        // records: c mod 8), 2c + (c >> 3 & 1) with the swizzled 8-float R = 8 records
        const int res = swz ? (c & 3) | (((c >> 3) & 1) << 2) : c & 7;
        uint64_t mine = 0;
        int cnt[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint64_t m = __ballot(on && res == q);
            cnt[q] = __builtin_popcountll(m);
            if (q == res) mine = m;
        }
        const int occ = __builtin_popcountll(mine & below);
        // entries before this one: all of occurrence < occ, plus occurrence ==
        // occ of a smaller residue
        int pos = 0;
#pragma unroll
        for (int q = 0; q < 8; ++q) pos += (cnt[q] < occ ? cnt[q] : occ) + (q < res && cnt[q] > occ);
        if (on) {
            if (odata) odata[r * k + pos] = d;
            if (osel) osel[r * k + pos] = (uint8_t)c;
            if (opacked) opacked[r * k + pos] = (uint16_t)(c | (lane << 8));
        }
    }
}

// ---------------------------------------------------------------------------
// Multi-relation LOCAL backward for R = 8 relations, k = 32, on the gradient
// interleaved by relation: gt[row][col][q] (fp32[V, h, 8], from
// grad_interleave_kernel).  One edge per wave-instruction: lane (entry l,
// half) loads the 16 B of relations 4*half..4*half+3 at (row, sel[c, l]), so
// an edge's 8 relations cost one 64-lane dwordx4 gather touching ~29 64-B
// sectors, where 8 single-relation calls issue 4 dword gathers touching
// ~112.  The two halves' partial sums meet by a lane swap and lanes 0..31
// update dXs in LDS.  Plan, bands (sized for 8 gradient rows per source row)
// and LDS block are the single-relation LOCAL's; the edge's record and its 8
// values are wave-uniform (scalar loads).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void grad_interleave_kernel(const float *__restrict__ grad,
                                                                 int R, int64_t plane, int64_t n,
                                                                 float *__restrict__ out)
{
    // out[i * R + q] = grad[q * plane + i], i < n = V * h
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        float v[16];
#pragma unroll
        for (int q = 0; q < 16; ++q)
            if (q < R) v[q] = grad[q * plane + i];
        if (R == 8) {
            f4 *o = reinterpret_cast<f4 *>(out + i * 8);
            o[0] = f4{v[0], v[1], v[2], v[3]};
            o[1] = f4{v[4], v[5], v[6], v[7]};
        } else {
            for (int q = 0; q < R; ++q) out[i * R + q] = v[q];
        }
    }
}

__device__ __forceinline__ void local_rel8_edges(int e_beg, int e_end,
                                                 const int32_t *__restrict__ erc,
                                                 const float *__restrict__ evl,
                                                 const float *__restrict__ gt, uint32_t dim,
                                                 const uint8_t *sl, float *acc)
{
    constexpr int K = 32, U = 8;
    const int lane = lane_id();
    const int l = lane & 31, half = lane >> 5;
    for (int base = e_beg; base < e_end; base += U) {
        const int n = (e_end - base) < U ? (e_end - base) : U;   // wave-uniform
        f4 g[U];
        f4 v[U];
        int ai[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (u >= n) break;
            const int e = base + u;
            const int rc = erc[e];                                 // uniform: scalar load
            const uint32_t row = (uint32_t)rc & 0xffffffu;
            ai[u] = (int)(((uint32_t)rc >> 24) * K) + l;
            const uint32_t col = sl[ai[u]];
            const f4 *vp = reinterpret_cast<const f4 *>(evl + (size_t)e * 8);
            const f4 va = vp[0], vb = vp[1];
            v[u] = half ? vb : va;
            g[u] = *reinterpret_cast<const f4 *>(gt + ((size_t)row * dim + col) * 8 + 4 * half);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (u >= n) break;
            float p = v[u].x * g[u].x + v[u].y * g[u].y + v[u].z * g[u].z + v[u].w * g[u].w;
            p += __shfl_xor(p, 32);
            if (half == 0) acc[ai[u]] += p;
        }
    }
}

__global__ __launch_bounds__(kBlock) void bwd_local_rel8_kernel(
    const int32_t *__restrict__ seg_beg, const int32_t *__restrict__ seg_end, bool first,
    const int32_t *__restrict__ dstart, int num_waves, int dmax,
    const int32_t *__restrict__ erc, const float *__restrict__ evl,
    const float *__restrict__ gt, const uint8_t *__restrict__ sel, int dim,
    float *__restrict__ dxs)
{
    constexpr int K = 32;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int wl = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int region = (dmax * K * 5 + 15) & ~15;
    float *acc = reinterpret_cast<float *>(reinterpret_cast<char *>(lds) + wl * region);
    uint8_t *sl = reinterpret_cast<uint8_t *>(acc + dmax * K);
    const int w = blockIdx.x * kWavesPerBlock + wl;
    if (w >= num_waves) return;
    const int lane = lane_id();
    const int e_beg = __builtin_amdgcn_readfirstlane(seg_beg[w]);
    const int e_end = __builtin_amdgcn_readfirstlane(seg_end[w]);
    if (!first && e_beg == e_end) return;
    const int d0 = dstart[w], D = dstart[w + 1] - d0;
    const int nent = D * K;
    float *dst = dxs + (size_t)d0 * K;
    const uint8_t *srow = sel + (size_t)d0 * K;
    for (int i = lane; i < nent; i += kWave) {
        acc[i] = first ? 0.f : dst[i];
        const int c = srow[i];
        sl[i] = (uint8_t)(c < dim ? c : dim - 1);
    }
    wave_sync_lds();
    local_rel8_edges(e_beg, e_end, erc, evl, gt, (uint32_t)dim, sl, acc);
    wave_sync_lds();
    for (int i = lane; i < nent; i += kWave) dst[i] = srow[i] < dim ? acc[i] : 0.f;
}

// ---------------------------------------------------------------------------
// Backward SSpMM, TILE algorithm (k = 32, h = 256; maxk_sspmm_backward_tile).
// LOCAL pays one 64-lane dword gather (~14 scattered 64-B sectors of a 1 KB
// G row) per two edges.  TILE instead reads every G row ONCE per CU: a
// workgroup (16 waves, the whole CU) owns up to 2048 destinations, keeps
// their dXs in VGPRs (64 slot registers per wave, v64..v127; lanes 0-31 one
// destination's 32 entries, lanes 32-63 another's) and their selectors as
// packed bytes (v48..v63), and sweeps the distinct source rows that have
// edges into its destinations through a 3-deep LDS ring of 47-row chunks
// (LDS-DMA, one 1 KB row per wave-instruction; row 47 of each buffer is a
// zero row for padding records).  Per edge: a selector byte picked by
// register index, one ds_read_b32 of the staged row, one v_fma into the
// slot register picked by index (s_set_gpr_idx: the slot is wave-uniform).
// Source rows are split into `splits` ranges (one workgroup per destination
// group and range) so 256 CUs are busy; range 0 writes dxs, the others write
// partial rows that tile_combine_kernel adds.
//
// The plan (spgemm_new_amd/tile.py, MaxKGraph.tile_plan) holds per
// (workgroup, wave) a header stream of int32x4: e(0), e(1) = {0, the rows of
// the wave's three DMA pieces of chunks 0 and 1}, then e(c+2) = {n0 | n1 <<
// 16 of chunk c, rows of chunk c+2} (-1 = the zero row); and a record
// stream: per chunk n0 records of destinations in lane half 0, then n1 of
// half 1, each a multiple of 4 (padding: slot 0, zero row, value 0).
// Record = int32x2 {slot | (buffer * 48 + row) << 24, value bits}.
// Per chunk: the first 4 record groups are s_loaded before the barrier and
// run software-pipelined in pairs; further groups run in an s_load loop.
// ring and chunk sizes: tile_format.h (shared with the plan builder)
constexpr int kTileLead = kTileBufs - 1;  // chunks the DMA runs ahead of the records
// outstanding VMEM ops allowed when a step waits for its chunk's DMA: the
// wave issues exactly kTilePieces DMA + 1 header load + 1 prefetch per step
#ifndef TILE_NO_PREFETCH
constexpr int kTileStepOps = kTilePieces + 2;
#else
constexpr int kTileStepOps = kTilePieces + 1;
#endif
constexpr int kTileVmcnt = (kTileStepOps - kTilePieces) + kTileStepOps * (kTileLead - 1);
static_assert(kTileVmcnt <= 63, "vmcnt field");

typedef float tile_acc_t __attribute__((ext_vector_type(32)));
typedef unsigned tile_sel_t __attribute__((ext_vector_type(16)));
typedef int tile_hdr_t __attribute__((ext_vector_type(4)));
typedef uint32_t tile_g16_t __attribute__((ext_vector_type(16)));

// The wave's three pieces of a chunk by range-checked buffer LDS-DMA: lane l of
// piece i loads 16 B at byte offset off_i (row * 1024 + 16 l) of the gradient
// (descriptor rsrc: base G, num_records = its bytes) into LDS at lds_byte +
// 1024 i + 16 l.  A zero-row piece carries an offset past the end (row -1:
// 0xFFFFFC00 + 16 l >= num_records), which the range check turns into zeros
// without any memory access.  soffset is the constant 0 (it is not range
// checked); the descriptor is built from kernel arguments once (no fresh
// readfirstlane SGPRs, so no VALU->SGPR->VMEM wait states are needed); M0 (the
// LDS address) is written by SALU and read after one wait state (s_nop 0).
// Always three VMEM operations per call, as the counted vmcnt requires.
typedef int32_t tile_rsrc_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void tile_bdma3(tile_rsrc_t rsrc, uint32_t off0, uint32_t off1,
                                           uint32_t off2, uint32_t lds_byte)
{
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\t"
                 "s_mov_b32 m0, %5\n\t"
                 "s_nop 0\n\t"
                 "buffer_load_dwordx4 %1, %4, 0 offen lds\n\t"
                 "s_add_u32 m0, m0, 0x400\n\t"
                 "s_nop 0\n\t"
                 "buffer_load_dwordx4 %2, %4, 0 offen lds\n\t"
                 "s_add_u32 m0, m0, 0x400\n\t"
                 "s_nop 0\n\t"
                 "buffer_load_dwordx4 %3, %4, 0 offen lds\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(off0), "v"(off1), "v"(off2), "s"(rsrc), "s"(lds_byte)
                 : "memory", "scc");
}

__device__ __forceinline__ void tile_glds(const float *g, uint32_t lds_byte)
{
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                 "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(lds_byte)
                 : "memory");
}


// Record = int32x2 {w = slot | row field << 24, value bits}; the slot
// register index reads w[7:0], the selector word is w >> 2, the selector
// byte's bit offset (w << 3) & 24, the staged row's LDS address w >> 14.
// Four records per step, all in one asm block: exec narrowed to the lane
// half (lanes 0-31 while half-0 groups remain, counted by m < 0), selector
// byte = v_bfe_u32 of the selector register picked by s_set_gpr_idx (SRC0),
// one ds_read_b32, v_fma_f32 into the slot register picked by s_set_gpr_idx
// (SRC2 | DST).  The compiler sees neither a divergent branch nor an
// indexed register, so the pinned slot (v64..v127) and selector (v48..v63)
// registers stay in place.  n = -(groups left), m = -(half-0 groups left):
// s_add_u32 sets SCC when a count reaches 0.
// Two of the groups loaded before the chunk's barrier, software-pipelined:
// the second group's selector bytes and LDS reads are issued before the
// first group's FMAs (no SMEM is in flight here, so lgkmcnt(4) waits for
// exactly the first group's reads).  m < -g on entry: group g is a half-0
// group.  The counts saturate: m keeps counting past 0 harmlessly.
__device__ __forceinline__ void tile_groups2(const uint32_t (&g)[16], uint32_t &n, uint32_t &m,
                                             uint64_t lo, uint64_t hi, tile_sel_t &selv,
                                             tile_acc_t &acc0, tile_acc_t &acc1)
{
    uint32_t t0, t1, t2, t3, t4, t5, t6, t7;
    uint64_t ex;
    asm volatile(
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_cmp_eq_u32 %[n], 0\n\t"
        "s_cbranch_scc1 .Ltp_done%=\n\t"
        "s_mov_b64 %[ex], exec\n\t"
        "s_cmp_lt_i32 %[m], 0\n\t"
        "s_cselect_b64 exec, %[lo], %[hi]\n\t"
        "s_lshr_b32 s80, %[g0], 2\n\t"
        "s_lshl_b32 s81, %[g0], 3\n\t"
        "s_lshr_b32 s82, %[g0], 14\n\t"
        "s_lshr_b32 s83, %[g2], 2\n\t"
        "s_lshl_b32 s84, %[g2], 3\n\t"
        "s_lshr_b32 s85, %[g2], 14\n\t"
        "s_lshr_b32 s86, %[g4], 2\n\t"
        "s_lshl_b32 s87, %[g4], 3\n\t"
        "s_lshr_b32 s88, %[g4], 14\n\t"
        "s_lshr_b32 s89, %[g6], 2\n\t"
        "s_lshl_b32 s90, %[g6], 3\n\t"
        "s_lshr_b32 s91, %[g6], 14\n\t"
        "s_set_gpr_idx_on s80, gpr_idx(SRC0)\n\t"
        "v_bfe_u32 %[t0], v48, s81, 8\n\t"
        "s_set_gpr_idx_idx s83\n\t"
        "v_bfe_u32 %[t1], v48, s84, 8\n\t"
        "s_set_gpr_idx_idx s86\n\t"
        "v_bfe_u32 %[t2], v48, s87, 8\n\t"
        "s_set_gpr_idx_idx s89\n\t"
        "v_bfe_u32 %[t3], v48, s90, 8\n\t"
        "s_set_gpr_idx_off\n\t"
        "v_lshl_add_u32 %[t0], %[t0], 2, s82\n\t"
        "v_lshl_add_u32 %[t1], %[t1], 2, s85\n\t"
        "v_lshl_add_u32 %[t2], %[t2], 2, s88\n\t"
        "v_lshl_add_u32 %[t3], %[t3], 2, s91\n\t"
        "ds_read_b32 %[t0], %[t0]\n\t"
        "ds_read_b32 %[t1], %[t1]\n\t"
        "ds_read_b32 %[t2], %[t2]\n\t"
        "ds_read_b32 %[t3], %[t3]\n\t"
        "s_cmp_eq_u32 %[n], -1\n\t"
        "s_cbranch_scc1 .Ltp_one%=\n\t"
        "s_cmp_lt_i32 %[m], -1\n\t"
        "s_cselect_b64 exec, %[lo], %[hi]\n\t"
        "s_lshr_b32 s80, %[g8], 2\n\t"
        "s_lshl_b32 s81, %[g8], 3\n\t"
        "s_lshr_b32 s82, %[g8], 14\n\t"
        "s_lshr_b32 s83, %[g10], 2\n\t"
        "s_lshl_b32 s84, %[g10], 3\n\t"
        "s_lshr_b32 s85, %[g10], 14\n\t"
        "s_lshr_b32 s86, %[g12], 2\n\t"
        "s_lshl_b32 s87, %[g12], 3\n\t"
        "s_lshr_b32 s88, %[g12], 14\n\t"
        "s_lshr_b32 s89, %[g14], 2\n\t"
        "s_lshl_b32 s90, %[g14], 3\n\t"
        "s_lshr_b32 s91, %[g14], 14\n\t"
        "s_set_gpr_idx_on s80, gpr_idx(SRC0)\n\t"
        "v_bfe_u32 %[t4], v48, s81, 8\n\t"
        "s_set_gpr_idx_idx s83\n\t"
        "v_bfe_u32 %[t5], v48, s84, 8\n\t"
        "s_set_gpr_idx_idx s86\n\t"
        "v_bfe_u32 %[t6], v48, s87, 8\n\t"
        "s_set_gpr_idx_idx s89\n\t"
        "v_bfe_u32 %[t7], v48, s90, 8\n\t"
        "s_set_gpr_idx_off\n\t"
        "v_lshl_add_u32 %[t4], %[t4], 2, s82\n\t"
        "v_lshl_add_u32 %[t5], %[t5], 2, s85\n\t"
        "v_lshl_add_u32 %[t6], %[t6], 2, s88\n\t"
        "v_lshl_add_u32 %[t7], %[t7], 2, s91\n\t"
        "ds_read_b32 %[t4], %[t4]\n\t"
        "ds_read_b32 %[t5], %[t5]\n\t"
        "ds_read_b32 %[t6], %[t6]\n\t"
        "ds_read_b32 %[t7], %[t7]\n\t"
        "s_waitcnt lgkmcnt(4)\n\t"
        "s_cmp_lt_i32 %[m], 0\n\t"
        "s_cselect_b64 exec, %[lo], %[hi]\n\t"
        "s_set_gpr_idx_on %[g0], gpr_idx(SRC2,DST)\n\t"
        "v_fma_f32 v64, %[t0], %[g1], v64\n\t"
        "s_set_gpr_idx_idx %[g2]\n\t"
        "v_fma_f32 v64, %[t1], %[g3], v64\n\t"
        "s_set_gpr_idx_idx %[g4]\n\t"
        "v_fma_f32 v64, %[t2], %[g5], v64\n\t"
        "s_set_gpr_idx_idx %[g6]\n\t"
        "v_fma_f32 v64, %[t3], %[g7], v64\n\t"
        "s_set_gpr_idx_off\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_cmp_lt_i32 %[m], -1\n\t"
        "s_cselect_b64 exec, %[lo], %[hi]\n\t"
        "s_set_gpr_idx_on %[g8], gpr_idx(SRC2,DST)\n\t"
        "v_fma_f32 v64, %[t4], %[g9], v64\n\t"
        "s_set_gpr_idx_idx %[g10]\n\t"
        "v_fma_f32 v64, %[t5], %[g11], v64\n\t"
        "s_set_gpr_idx_idx %[g12]\n\t"
        "v_fma_f32 v64, %[t6], %[g13], v64\n\t"
        "s_set_gpr_idx_idx %[g14]\n\t"
        "v_fma_f32 v64, %[t7], %[g15], v64\n\t"
        "s_set_gpr_idx_off\n\t"
        "s_add_u32 %[n], %[n], 2\n\t"
        "s_add_u32 %[m], %[m], 2\n\t"
        "s_branch .Ltp_end%=\n\t"
        ".Ltp_one%=:\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_cmp_lt_i32 %[m], 0\n\t"
        "s_cselect_b64 exec, %[lo], %[hi]\n\t"
        "s_set_gpr_idx_on %[g0], gpr_idx(SRC2,DST)\n\t"
        "v_fma_f32 v64, %[t0], %[g1], v64\n\t"
        "s_set_gpr_idx_idx %[g2]\n\t"
        "v_fma_f32 v64, %[t1], %[g3], v64\n\t"
        "s_set_gpr_idx_idx %[g4]\n\t"
        "v_fma_f32 v64, %[t2], %[g5], v64\n\t"
        "s_set_gpr_idx_idx %[g6]\n\t"
        "v_fma_f32 v64, %[t3], %[g7], v64\n\t"
        "s_set_gpr_idx_off\n\t"
        "s_add_u32 %[n], %[n], 1\n\t"
        "s_add_u32 %[m], %[m], 1\n\t"
        ".Ltp_end%=:\n\t"
        "s_mov_b64 exec, %[ex]\n\t"
        ".Ltp_done%=:\n\t"
        : [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3), [t4] "=&v"(t4),
          [t5] "=&v"(t5), [t6] "=&v"(t6), [t7] "=&v"(t7), [ex] "=&s"(ex), [n] "+s"(n),
          [m] "+s"(m), "+{v[48:63]}"(selv), "+{v[64:95]}"(acc0), "+{v[96:127]}"(acc1)
        : [lo] "s"(lo), [hi] "s"(hi),
          [g0] "s"(g[0]), [g1] "s"(g[1]), [g2] "s"(g[2]), [g3] "s"(g[3]),
          [g4] "s"(g[4]), [g5] "s"(g[5]), [g6] "s"(g[6]), [g7] "s"(g[7]),
          [g8] "s"(g[8]), [g9] "s"(g[9]), [g10] "s"(g[10]), [g11] "s"(g[11]),
          [g12] "s"(g[12]), [g13] "s"(g[13]), [g14] "s"(g[14]), [g15] "s"(g[15])
        : "memory", "scc", "s80", "s81", "s82", "s83", "s84", "s85", "s86", "s87", "s88", "s89",
          "s90", "s91");
}

// the groups after the four loaded before the barrier: s_load, the next group
// in flight while the current one runs; s64..s91 are the loop's
__device__ __forceinline__ void tile_group_loop(const uint32_t *rb, uint32_t ro, uint32_t &n,
                                                uint32_t &m, uint64_t lo, uint64_t hi,
                                                tile_sel_t &selv, tile_acc_t &acc0,
                                                tile_acc_t &acc1)
{
    uint32_t t0, t1, t2, t3;
    uint64_t ex;
    asm volatile(
        "s_cmp_eq_u32 %[n], 0\n\t"
        "s_cbranch_scc1 .Ltile_done%=\n\t"
        "s_mov_b64 %[ex], exec\n\t"
        "s_cmp_lt_i32 %[m], 0\n\t"
        "s_cselect_b64 exec, %[lo], %[hi]\n\t"
        "s_load_dwordx8 s[64:71], %[rb], %[ro]\n\t"
        "s_add_u32 %[ro], %[ro], 32\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        ".Ltile_a%=:\n\t"
        "s_add_u32 %[n], %[n], 1\n\t"
        "s_cbranch_scc1 .Ltile_a_last%=\n\t"
        "s_load_dwordx8 s[72:79], %[rb], %[ro]\n\t"
        "s_add_u32 %[ro], %[ro], 32\n\t"
        "s_lshr_b32 s80, s64, 2\n\t"
        "s_lshl_b32 s81, s64, 3\n\t"
        "s_lshr_b32 s82, s64, 14\n\t"
        "s_lshr_b32 s83, s66, 2\n\t"
        "s_lshl_b32 s84, s66, 3\n\t"
        "s_lshr_b32 s85, s66, 14\n\t"
        "s_lshr_b32 s86, s68, 2\n\t"
        "s_lshl_b32 s87, s68, 3\n\t"
        "s_lshr_b32 s88, s68, 14\n\t"
        "s_lshr_b32 s89, s70, 2\n\t"
        "s_lshl_b32 s90, s70, 3\n\t"
        "s_lshr_b32 s91, s70, 14\n\t"
        "s_set_gpr_idx_on s80, gpr_idx(SRC0)\n\t"
        "v_bfe_u32 %[t0], v48, s81, 8\n\t"
        "s_set_gpr_idx_idx s83\n\t"
        "v_bfe_u32 %[t1], v48, s84, 8\n\t"
        "s_set_gpr_idx_idx s86\n\t"
        "v_bfe_u32 %[t2], v48, s87, 8\n\t"
        "s_set_gpr_idx_idx s89\n\t"
        "v_bfe_u32 %[t3], v48, s90, 8\n\t"
        "s_set_gpr_idx_off\n\t"
        "v_lshl_add_u32 %[t0], %[t0], 2, s82\n\t"
        "v_lshl_add_u32 %[t1], %[t1], 2, s85\n\t"
        "v_lshl_add_u32 %[t2], %[t2], 2, s88\n\t"
        "v_lshl_add_u32 %[t3], %[t3], 2, s91\n\t"
        "ds_read_b32 %[t0], %[t0]\n\t"
        "ds_read_b32 %[t1], %[t1]\n\t"
        "ds_read_b32 %[t2], %[t2]\n\t"
        "ds_read_b32 %[t3], %[t3]\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_set_gpr_idx_on s64, gpr_idx(SRC2,DST)\n\t"
        "v_fma_f32 v64, %[t0], s65, v64\n\t"
        "s_set_gpr_idx_idx s66\n\t"
        "v_fma_f32 v64, %[t1], s67, v64\n\t"
        "s_set_gpr_idx_idx s68\n\t"
        "v_fma_f32 v64, %[t2], s69, v64\n\t"
        "s_set_gpr_idx_idx s70\n\t"
        "v_fma_f32 v64, %[t3], s71, v64\n\t"
        "s_set_gpr_idx_off\n\t"
        "s_add_u32 %[m], %[m], 1\n\t"
        "s_cselect_b64 exec, %[hi], exec\n\t"
        "s_add_u32 %[n], %[n], 1\n\t"
        "s_cbranch_scc1 .Ltile_b_last%=\n\t"
        "s_load_dwordx8 s[64:71], %[rb], %[ro]\n\t"
        "s_add_u32 %[ro], %[ro], 32\n\t"
        "s_lshr_b32 s80, s72, 2\n\t"
        "s_lshl_b32 s81, s72, 3\n\t"
        "s_lshr_b32 s82, s72, 14\n\t"
        "s_lshr_b32 s83, s74, 2\n\t"
        "s_lshl_b32 s84, s74, 3\n\t"
        "s_lshr_b32 s85, s74, 14\n\t"
        "s_lshr_b32 s86, s76, 2\n\t"
        "s_lshl_b32 s87, s76, 3\n\t"
        "s_lshr_b32 s88, s76, 14\n\t"
        "s_lshr_b32 s89, s78, 2\n\t"
        "s_lshl_b32 s90, s78, 3\n\t"
        "s_lshr_b32 s91, s78, 14\n\t"
        "s_set_gpr_idx_on s80, gpr_idx(SRC0)\n\t"
        "v_bfe_u32 %[t0], v48, s81, 8\n\t"
        "s_set_gpr_idx_idx s83\n\t"
        "v_bfe_u32 %[t1], v48, s84, 8\n\t"
        "s_set_gpr_idx_idx s86\n\t"
        "v_bfe_u32 %[t2], v48, s87, 8\n\t"
        "s_set_gpr_idx_idx s89\n\t"
        "v_bfe_u32 %[t3], v48, s90, 8\n\t"
        "s_set_gpr_idx_off\n\t"
        "v_lshl_add_u32 %[t0], %[t0], 2, s82\n\t"
        "v_lshl_add_u32 %[t1], %[t1], 2, s85\n\t"
        "v_lshl_add_u32 %[t2], %[t2], 2, s88\n\t"
        "v_lshl_add_u32 %[t3], %[t3], 2, s91\n\t"
        "ds_read_b32 %[t0], %[t0]\n\t"
        "ds_read_b32 %[t1], %[t1]\n\t"
        "ds_read_b32 %[t2], %[t2]\n\t"
        "ds_read_b32 %[t3], %[t3]\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_set_gpr_idx_on s72, gpr_idx(SRC2,DST)\n\t"
        "v_fma_f32 v64, %[t0], s73, v64\n\t"
        "s_set_gpr_idx_idx s74\n\t"
        "v_fma_f32 v64, %[t1], s75, v64\n\t"
        "s_set_gpr_idx_idx s76\n\t"
        "v_fma_f32 v64, %[t2], s77, v64\n\t"
        "s_set_gpr_idx_idx s78\n\t"
        "v_fma_f32 v64, %[t3], s79, v64\n\t"
        "s_set_gpr_idx_off\n\t"
        "s_add_u32 %[m], %[m], 1\n\t"
        "s_cselect_b64 exec, %[hi], exec\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_branch .Ltile_a%=\n\t"
        ".Ltile_a_last%=:\n\t"
        "s_lshr_b32 s80, s64, 2\n\t"
        "s_lshl_b32 s81, s64, 3\n\t"
        "s_lshr_b32 s82, s64, 14\n\t"
        "s_lshr_b32 s83, s66, 2\n\t"
        "s_lshl_b32 s84, s66, 3\n\t"
        "s_lshr_b32 s85, s66, 14\n\t"
        "s_lshr_b32 s86, s68, 2\n\t"
        "s_lshl_b32 s87, s68, 3\n\t"
        "s_lshr_b32 s88, s68, 14\n\t"
        "s_lshr_b32 s89, s70, 2\n\t"
        "s_lshl_b32 s90, s70, 3\n\t"
        "s_lshr_b32 s91, s70, 14\n\t"
        "s_set_gpr_idx_on s80, gpr_idx(SRC0)\n\t"
        "v_bfe_u32 %[t0], v48, s81, 8\n\t"
        "s_set_gpr_idx_idx s83\n\t"
        "v_bfe_u32 %[t1], v48, s84, 8\n\t"
        "s_set_gpr_idx_idx s86\n\t"
        "v_bfe_u32 %[t2], v48, s87, 8\n\t"
        "s_set_gpr_idx_idx s89\n\t"
        "v_bfe_u32 %[t3], v48, s90, 8\n\t"
        "s_set_gpr_idx_off\n\t"
        "v_lshl_add_u32 %[t0], %[t0], 2, s82\n\t"
        "v_lshl_add_u32 %[t1], %[t1], 2, s85\n\t"
        "v_lshl_add_u32 %[t2], %[t2], 2, s88\n\t"
        "v_lshl_add_u32 %[t3], %[t3], 2, s91\n\t"
        "ds_read_b32 %[t0], %[t0]\n\t"
        "ds_read_b32 %[t1], %[t1]\n\t"
        "ds_read_b32 %[t2], %[t2]\n\t"
        "ds_read_b32 %[t3], %[t3]\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_set_gpr_idx_on s64, gpr_idx(SRC2,DST)\n\t"
        "v_fma_f32 v64, %[t0], s65, v64\n\t"
        "s_set_gpr_idx_idx s66\n\t"
        "v_fma_f32 v64, %[t1], s67, v64\n\t"
        "s_set_gpr_idx_idx s68\n\t"
        "v_fma_f32 v64, %[t2], s69, v64\n\t"
        "s_set_gpr_idx_idx s70\n\t"
        "v_fma_f32 v64, %[t3], s71, v64\n\t"
        "s_set_gpr_idx_off\n\t"
        "s_branch .Ltile_end%=\n\t"
        ".Ltile_b_last%=:\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_lshr_b32 s80, s72, 2\n\t"
        "s_lshl_b32 s81, s72, 3\n\t"
        "s_lshr_b32 s82, s72, 14\n\t"
        "s_lshr_b32 s83, s74, 2\n\t"
        "s_lshl_b32 s84, s74, 3\n\t"
        "s_lshr_b32 s85, s74, 14\n\t"
        "s_lshr_b32 s86, s76, 2\n\t"
        "s_lshl_b32 s87, s76, 3\n\t"
        "s_lshr_b32 s88, s76, 14\n\t"
        "s_lshr_b32 s89, s78, 2\n\t"
        "s_lshl_b32 s90, s78, 3\n\t"
        "s_lshr_b32 s91, s78, 14\n\t"
        "s_set_gpr_idx_on s80, gpr_idx(SRC0)\n\t"
        "v_bfe_u32 %[t0], v48, s81, 8\n\t"
        "s_set_gpr_idx_idx s83\n\t"
        "v_bfe_u32 %[t1], v48, s84, 8\n\t"
        "s_set_gpr_idx_idx s86\n\t"
        "v_bfe_u32 %[t2], v48, s87, 8\n\t"
        "s_set_gpr_idx_idx s89\n\t"
        "v_bfe_u32 %[t3], v48, s90, 8\n\t"
        "s_set_gpr_idx_off\n\t"
        "v_lshl_add_u32 %[t0], %[t0], 2, s82\n\t"
        "v_lshl_add_u32 %[t1], %[t1], 2, s85\n\t"
        "v_lshl_add_u32 %[t2], %[t2], 2, s88\n\t"
        "v_lshl_add_u32 %[t3], %[t3], 2, s91\n\t"
        "ds_read_b32 %[t0], %[t0]\n\t"
        "ds_read_b32 %[t1], %[t1]\n\t"
        "ds_read_b32 %[t2], %[t2]\n\t"
        "ds_read_b32 %[t3], %[t3]\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_set_gpr_idx_on s72, gpr_idx(SRC2,DST)\n\t"
        "v_fma_f32 v64, %[t0], s73, v64\n\t"
        "s_set_gpr_idx_idx s74\n\t"
        "v_fma_f32 v64, %[t1], s75, v64\n\t"
        "s_set_gpr_idx_idx s76\n\t"
        "v_fma_f32 v64, %[t2], s77, v64\n\t"
        "s_set_gpr_idx_idx s78\n\t"
        "v_fma_f32 v64, %[t3], s79, v64\n\t"
        "s_set_gpr_idx_off\n\t"
        ".Ltile_end%=:\n\t"
        "s_mov_b64 exec, %[ex]\n\t"
        ".Ltile_done%=:\n\t"
        : [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3), [ex] "=&s"(ex),
          [ro] "+s"(ro), [m] "+s"(m), [n] "+s"(n), "+{v[48:63]}"(selv), "+{v[64:95]}"(acc0),
          "+{v[96:127]}"(acc1)
        : [rb] "s"(rb), [lo] "s"(lo), [hi] "s"(hi)
        : "memory", "scc", "s64", "s65", "s66", "s67", "s68", "s69", "s70", "s71", "s72", "s73", "s74", "s75", "s76", "s77", "s78", "s79", "s80", "s81", "s82", "s83", "s84", "s85", "s86", "s87", "s88", "s89", "s90", "s91");
}

// TILE_REC_WORDS = 4 (tile_format.h): record = {v_perm control, slot, row's LDS
// byte address, value}.  Per record: the selector byte by one v_perm_b32 of the
// selector register picked by s_set_gpr_idx (SRC0, index = control byte 0,
// the byte picked by control byte 2 lands in byte 2, bytes 1 / 3 are zero), so
// address = (perm >> 14) + row; one ds_read_b32; v_fma_f32 into the slot
// register picked by s_set_gpr_idx (SRC2 | DST).  No scalar shifts: per group
// of four records 10 gpr-index instructions plus the exec and count updates
// (the two-word format spends 12 more on field shifts).  Records sit in
// pinned SGPRs: the two groups loaded before the chunk's barrier in s[64:79]
// and s[80:95] (the loop below reuses them).
__device__ __forceinline__ void tile_groups2_r16(const tile_g16_t &pa, const tile_g16_t &pb,
                                                 uint32_t &n, uint32_t &m, uint64_t lo, uint64_t hi,
                                                 tile_sel_t &selv, tile_acc_t &acc0,
                                                 tile_acc_t &acc1)
{
    uint32_t t0, t1, t2, t3, t4, t5, t6, t7;
    uint64_t ex;
    asm volatile(
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_cmp_eq_u32 %[n], 0\n\t"
        "s_cbranch_scc1 .Lr2_done%=\n\t"
        "s_mov_b64 %[ex], exec\n\t"
        "s_cmp_lt_i32 %[m], 0\n\t"
        "s_cselect_b64 exec, %[lo], %[hi]\n\t"
        "s_set_gpr_idx_on s64, gpr_idx(SRC0)\n\t"
        "v_perm_b32 %[t0], v48, 0, s64\n\t"
        "s_set_gpr_idx_idx s68\n\t"
        "v_perm_b32 %[t1], v48, 0, s68\n\t"
        "s_set_gpr_idx_idx s72\n\t"
        "v_perm_b32 %[t2], v48, 0, s72\n\t"
        "s_set_gpr_idx_idx s76\n\t"
        "v_perm_b32 %[t3], v48, 0, s76\n\t"
        "s_set_gpr_idx_off\n\t"
        "v_lshrrev_b32 %[t0], 14, %[t0]\n\t"
        "v_lshrrev_b32 %[t1], 14, %[t1]\n\t"
        "v_lshrrev_b32 %[t2], 14, %[t2]\n\t"
        "v_lshrrev_b32 %[t3], 14, %[t3]\n\t"
        "v_add_u32 %[t0], s66, %[t0]\n\t"
        "v_add_u32 %[t1], s70, %[t1]\n\t"
        "v_add_u32 %[t2], s74, %[t2]\n\t"
        "v_add_u32 %[t3], s78, %[t3]\n\t"
        "ds_read_b32 %[t0], %[t0]\n\t"
        "ds_read_b32 %[t1], %[t1]\n\t"
        "ds_read_b32 %[t2], %[t2]\n\t"
        "ds_read_b32 %[t3], %[t3]\n\t"
        "s_cmp_eq_u32 %[n], -1\n\t"
        "s_cbranch_scc1 .Lr2_one%=\n\t"
        "s_cmp_lt_i32 %[m], -1\n\t"
        "s_cselect_b64 exec, %[lo], %[hi]\n\t"
        "s_set_gpr_idx_on s80, gpr_idx(SRC0)\n\t"
        "v_perm_b32 %[t4], v48, 0, s80\n\t"
        "s_set_gpr_idx_idx s84\n\t"
        "v_perm_b32 %[t5], v48, 0, s84\n\t"
        "s_set_gpr_idx_idx s88\n\t"
        "v_perm_b32 %[t6], v48, 0, s88\n\t"
        "s_set_gpr_idx_idx s92\n\t"
        "v_perm_b32 %[t7], v48, 0, s92\n\t"
        "s_set_gpr_idx_off\n\t"
        "v_lshrrev_b32 %[t4], 14, %[t4]\n\t"
        "v_lshrrev_b32 %[t5], 14, %[t5]\n\t"
        "v_lshrrev_b32 %[t6], 14, %[t6]\n\t"
        "v_lshrrev_b32 %[t7], 14, %[t7]\n\t"
        "v_add_u32 %[t4], s82, %[t4]\n\t"
        "v_add_u32 %[t5], s86, %[t5]\n\t"
        "v_add_u32 %[t6], s90, %[t6]\n\t"
        "v_add_u32 %[t7], s94, %[t7]\n\t"
        "ds_read_b32 %[t4], %[t4]\n\t"
        "ds_read_b32 %[t5], %[t5]\n\t"
        "ds_read_b32 %[t6], %[t6]\n\t"
        "ds_read_b32 %[t7], %[t7]\n\t"
        "s_waitcnt lgkmcnt(4)\n\t"
        "s_cmp_lt_i32 %[m], 0\n\t"
        "s_cselect_b64 exec, %[lo], %[hi]\n\t"
        "s_set_gpr_idx_on s65, gpr_idx(SRC2,DST)\n\t"
        "v_fma_f32 v64, %[t0], s67, v64\n\t"
        "s_set_gpr_idx_idx s69\n\t"
        "v_fma_f32 v64, %[t1], s71, v64\n\t"
        "s_set_gpr_idx_idx s73\n\t"
        "v_fma_f32 v64, %[t2], s75, v64\n\t"
        "s_set_gpr_idx_idx s77\n\t"
        "v_fma_f32 v64, %[t3], s79, v64\n\t"
        "s_set_gpr_idx_off\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_cmp_lt_i32 %[m], -1\n\t"
        "s_cselect_b64 exec, %[lo], %[hi]\n\t"
        "s_set_gpr_idx_on s81, gpr_idx(SRC2,DST)\n\t"
        "v_fma_f32 v64, %[t4], s83, v64\n\t"
        "s_set_gpr_idx_idx s85\n\t"
        "v_fma_f32 v64, %[t5], s87, v64\n\t"
        "s_set_gpr_idx_idx s89\n\t"
        "v_fma_f32 v64, %[t6], s91, v64\n\t"
        "s_set_gpr_idx_idx s93\n\t"
        "v_fma_f32 v64, %[t7], s95, v64\n\t"
        "s_set_gpr_idx_off\n\t"
        "s_add_u32 %[n], %[n], 2\n\t"
        "s_add_u32 %[m], %[m], 2\n\t"
        "s_branch .Lr2_end%=\n\t"
        ".Lr2_one%=:\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_cmp_lt_i32 %[m], 0\n\t"
        "s_cselect_b64 exec, %[lo], %[hi]\n\t"
        "s_set_gpr_idx_on s65, gpr_idx(SRC2,DST)\n\t"
        "v_fma_f32 v64, %[t0], s67, v64\n\t"
        "s_set_gpr_idx_idx s69\n\t"
        "v_fma_f32 v64, %[t1], s71, v64\n\t"
        "s_set_gpr_idx_idx s73\n\t"
        "v_fma_f32 v64, %[t2], s75, v64\n\t"
        "s_set_gpr_idx_idx s77\n\t"
        "v_fma_f32 v64, %[t3], s79, v64\n\t"
        "s_set_gpr_idx_off\n\t"
        "s_add_u32 %[n], %[n], 1\n\t"
        "s_add_u32 %[m], %[m], 1\n\t"
        ".Lr2_end%=:\n\t"
        "s_mov_b64 exec, %[ex]\n\t"
        ".Lr2_done%=:\n\t"
        : [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3), [t4] "=&v"(t4),
          [t5] "=&v"(t5), [t6] "=&v"(t6), [t7] "=&v"(t7), [ex] "=&s"(ex), [n] "+s"(n),
          [m] "+s"(m), "+{v[48:63]}"(selv), "+{v[64:95]}"(acc0), "+{v[96:127]}"(acc1)
        : [lo] "s"(lo), [hi] "s"(hi), "{s[64:79]}"(pa), "{s[80:95]}"(pb)
        : "memory", "scc");
}

// the groups after the two loaded before the barrier (four-word records): s_load
// into s[64:79] / s[80:95] alternately, the next group in flight
__device__ __forceinline__ void tile_group_loop_r16(const uint32_t *rb, uint32_t ro, uint32_t &n,
                                                    uint32_t &m, uint64_t lo, uint64_t hi,
                                                    tile_sel_t &selv, tile_acc_t &acc0,
                                                    tile_acc_t &acc1)
{
    uint32_t t0, t1, t2, t3;
    uint64_t ex;
    asm volatile(
        "s_cmp_eq_u32 %[n], 0\n\t"
        "s_cbranch_scc1 .Lr4_done%=\n\t"
        "s_mov_b64 %[ex], exec\n\t"
        "s_cmp_lt_i32 %[m], 0\n\t"
        "s_cselect_b64 exec, %[lo], %[hi]\n\t"
        "s_load_dwordx16 s[64:79], %[rb], %[ro]\n\t"
        "s_add_u32 %[ro], %[ro], 64\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        ".Lr4_a%=:\n\t"
        "s_add_u32 %[n], %[n], 1\n\t"
        "s_cbranch_scc1 .Lr4_a_last%=\n\t"
        "s_load_dwordx16 s[80:95], %[rb], %[ro]\n\t"
        "s_add_u32 %[ro], %[ro], 64\n\t"
        "s_set_gpr_idx_on s64, gpr_idx(SRC0)\n\t"
        "v_perm_b32 %[t0], v48, 0, s64\n\t"
        "s_set_gpr_idx_idx s68\n\t"
        "v_perm_b32 %[t1], v48, 0, s68\n\t"
        "s_set_gpr_idx_idx s72\n\t"
        "v_perm_b32 %[t2], v48, 0, s72\n\t"
        "s_set_gpr_idx_idx s76\n\t"
        "v_perm_b32 %[t3], v48, 0, s76\n\t"
        "s_set_gpr_idx_off\n\t"
        "v_lshrrev_b32 %[t0], 14, %[t0]\n\t"
        "v_lshrrev_b32 %[t1], 14, %[t1]\n\t"
        "v_lshrrev_b32 %[t2], 14, %[t2]\n\t"
        "v_lshrrev_b32 %[t3], 14, %[t3]\n\t"
        "v_add_u32 %[t0], s66, %[t0]\n\t"
        "v_add_u32 %[t1], s70, %[t1]\n\t"
        "v_add_u32 %[t2], s74, %[t2]\n\t"
        "v_add_u32 %[t3], s78, %[t3]\n\t"
        "ds_read_b32 %[t0], %[t0]\n\t"
        "ds_read_b32 %[t1], %[t1]\n\t"
        "ds_read_b32 %[t2], %[t2]\n\t"
        "ds_read_b32 %[t3], %[t3]\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_set_gpr_idx_on s65, gpr_idx(SRC2,DST)\n\t"
        "v_fma_f32 v64, %[t0], s67, v64\n\t"
        "s_set_gpr_idx_idx s69\n\t"
        "v_fma_f32 v64, %[t1], s71, v64\n\t"
        "s_set_gpr_idx_idx s73\n\t"
        "v_fma_f32 v64, %[t2], s75, v64\n\t"
        "s_set_gpr_idx_idx s77\n\t"
        "v_fma_f32 v64, %[t3], s79, v64\n\t"
        "s_set_gpr_idx_off\n\t"
        "s_add_u32 %[m], %[m], 1\n\t"
        "s_cselect_b64 exec, %[hi], exec\n\t"
        "s_add_u32 %[n], %[n], 1\n\t"
        "s_cbranch_scc1 .Lr4_b_last%=\n\t"
        "s_load_dwordx16 s[64:79], %[rb], %[ro]\n\t"
        "s_add_u32 %[ro], %[ro], 64\n\t"
        "s_set_gpr_idx_on s80, gpr_idx(SRC0)\n\t"
        "v_perm_b32 %[t0], v48, 0, s80\n\t"
        "s_set_gpr_idx_idx s84\n\t"
        "v_perm_b32 %[t1], v48, 0, s84\n\t"
        "s_set_gpr_idx_idx s88\n\t"
        "v_perm_b32 %[t2], v48, 0, s88\n\t"
        "s_set_gpr_idx_idx s92\n\t"
        "v_perm_b32 %[t3], v48, 0, s92\n\t"
        "s_set_gpr_idx_off\n\t"
        "v_lshrrev_b32 %[t0], 14, %[t0]\n\t"
        "v_lshrrev_b32 %[t1], 14, %[t1]\n\t"
        "v_lshrrev_b32 %[t2], 14, %[t2]\n\t"
        "v_lshrrev_b32 %[t3], 14, %[t3]\n\t"
        "v_add_u32 %[t0], s82, %[t0]\n\t"
        "v_add_u32 %[t1], s86, %[t1]\n\t"
        "v_add_u32 %[t2], s90, %[t2]\n\t"
        "v_add_u32 %[t3], s94, %[t3]\n\t"
        "ds_read_b32 %[t0], %[t0]\n\t"
        "ds_read_b32 %[t1], %[t1]\n\t"
        "ds_read_b32 %[t2], %[t2]\n\t"
        "ds_read_b32 %[t3], %[t3]\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_set_gpr_idx_on s81, gpr_idx(SRC2,DST)\n\t"
        "v_fma_f32 v64, %[t0], s83, v64\n\t"
        "s_set_gpr_idx_idx s85\n\t"
        "v_fma_f32 v64, %[t1], s87, v64\n\t"
        "s_set_gpr_idx_idx s89\n\t"
        "v_fma_f32 v64, %[t2], s91, v64\n\t"
        "s_set_gpr_idx_idx s93\n\t"
        "v_fma_f32 v64, %[t3], s95, v64\n\t"
        "s_set_gpr_idx_off\n\t"
        "s_add_u32 %[m], %[m], 1\n\t"
        "s_cselect_b64 exec, %[hi], exec\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_branch .Lr4_a%=\n\t"
        ".Lr4_a_last%=:\n\t"
        "s_set_gpr_idx_on s64, gpr_idx(SRC0)\n\t"
        "v_perm_b32 %[t0], v48, 0, s64\n\t"
        "s_set_gpr_idx_idx s68\n\t"
        "v_perm_b32 %[t1], v48, 0, s68\n\t"
        "s_set_gpr_idx_idx s72\n\t"
        "v_perm_b32 %[t2], v48, 0, s72\n\t"
        "s_set_gpr_idx_idx s76\n\t"
        "v_perm_b32 %[t3], v48, 0, s76\n\t"
        "s_set_gpr_idx_off\n\t"
        "v_lshrrev_b32 %[t0], 14, %[t0]\n\t"
        "v_lshrrev_b32 %[t1], 14, %[t1]\n\t"
        "v_lshrrev_b32 %[t2], 14, %[t2]\n\t"
        "v_lshrrev_b32 %[t3], 14, %[t3]\n\t"
        "v_add_u32 %[t0], s66, %[t0]\n\t"
        "v_add_u32 %[t1], s70, %[t1]\n\t"
        "v_add_u32 %[t2], s74, %[t2]\n\t"
        "v_add_u32 %[t3], s78, %[t3]\n\t"
        "ds_read_b32 %[t0], %[t0]\n\t"
        "ds_read_b32 %[t1], %[t1]\n\t"
        "ds_read_b32 %[t2], %[t2]\n\t"
        "ds_read_b32 %[t3], %[t3]\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_set_gpr_idx_on s65, gpr_idx(SRC2,DST)\n\t"
        "v_fma_f32 v64, %[t0], s67, v64\n\t"
        "s_set_gpr_idx_idx s69\n\t"
        "v_fma_f32 v64, %[t1], s71, v64\n\t"
        "s_set_gpr_idx_idx s73\n\t"
        "v_fma_f32 v64, %[t2], s75, v64\n\t"
        "s_set_gpr_idx_idx s77\n\t"
        "v_fma_f32 v64, %[t3], s79, v64\n\t"
        "s_set_gpr_idx_off\n\t"
        "s_branch .Lr4_end%=\n\t"
        ".Lr4_b_last%=:\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_set_gpr_idx_on s80, gpr_idx(SRC0)\n\t"
        "v_perm_b32 %[t0], v48, 0, s80\n\t"
        "s_set_gpr_idx_idx s84\n\t"
        "v_perm_b32 %[t1], v48, 0, s84\n\t"
        "s_set_gpr_idx_idx s88\n\t"
        "v_perm_b32 %[t2], v48, 0, s88\n\t"
        "s_set_gpr_idx_idx s92\n\t"
        "v_perm_b32 %[t3], v48, 0, s92\n\t"
        "s_set_gpr_idx_off\n\t"
        "v_lshrrev_b32 %[t0], 14, %[t0]\n\t"
        "v_lshrrev_b32 %[t1], 14, %[t1]\n\t"
        "v_lshrrev_b32 %[t2], 14, %[t2]\n\t"
        "v_lshrrev_b32 %[t3], 14, %[t3]\n\t"
        "v_add_u32 %[t0], s82, %[t0]\n\t"
        "v_add_u32 %[t1], s86, %[t1]\n\t"
        "v_add_u32 %[t2], s90, %[t2]\n\t"
        "v_add_u32 %[t3], s94, %[t3]\n\t"
        "ds_read_b32 %[t0], %[t0]\n\t"
        "ds_read_b32 %[t1], %[t1]\n\t"
        "ds_read_b32 %[t2], %[t2]\n\t"
        "ds_read_b32 %[t3], %[t3]\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "s_set_gpr_idx_on s81, gpr_idx(SRC2,DST)\n\t"
        "v_fma_f32 v64, %[t0], s83, v64\n\t"
        "s_set_gpr_idx_idx s85\n\t"
        "v_fma_f32 v64, %[t1], s87, v64\n\t"
        "s_set_gpr_idx_idx s89\n\t"
        "v_fma_f32 v64, %[t2], s91, v64\n\t"
        "s_set_gpr_idx_idx s93\n\t"
        "v_fma_f32 v64, %[t3], s95, v64\n\t"
        "s_set_gpr_idx_off\n\t"
        ".Lr4_end%=:\n\t"
        "s_mov_b64 exec, %[ex]\n\t"
        ".Lr4_done%=:\n\t"
        : [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3), [ex] "=&s"(ex),
          [ro] "+s"(ro), [m] "+s"(m), [n] "+s"(n), "+{v[48:63]}"(selv), "+{v[64:95]}"(acc0),
          "+{v[96:127]}"(acc1)
        : [rb] "s"(rb), [lo] "s"(lo), [hi] "s"(hi)
        : "memory", "scc", "s64", "s65", "s66", "s67", "s68", "s69", "s70", "s71", "s72", "s73",
          "s74", "s75", "s76", "s77", "s78", "s79", "s80", "s81", "s82", "s83", "s84", "s85",
          "s86", "s87", "s88", "s89", "s90", "s91", "s92", "s93", "s94", "s95");
}

__device__ __forceinline__ tile_hdr_t tile_load_hdr(const tile_hdr_t *p)
{
    tile_hdr_t h;
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(h) : "v"(p) : "memory");
    return h;
}

// pulls a line range into L2; the destination register stays live (the
// caller keeps `d` in every later wait) so nothing else lands in it while the
// load is in flight
__device__ __forceinline__ void tile_prefetch(const uint32_t *p, uint32_t &d)
{
    asm volatile("global_load_dword %0, %1, off" : "+v"(d) : "v"(p) : "memory");
}

// K = 32: slot register s holds destinations (2s + half) * 16 + wave, lanes
// 0-31 / 32-63 their 32 entries; K = 64: destination s * 16 + wave, one entry
// per lane, the records all in "half 0" with exec on every lane.
// BDMA: the DMA pieces by range-checked buffer loads (tile_bdma3: offsets from
// the header VGPRs, ~6 SALU per chunk) instead of one 64-bit address select per
// piece (~9 SALU each); needs the gradient below 4 GiB - 1 KiB.
struct TileArgs {
    const tile_hdr_t *hdrs;
    const int64_t *hdr_start;
    const uint32_t *recs;
    const int64_t *rec_start;
    const int32_t *num_chunks;
    const float *grad;
    const float *zero_row;
    const uint8_t *sel;
    float *dxs;
    float *part;
    int num_cols, group_size, num_groups, num_wgs, num_rows;
};
using TileArgsK = __attribute__((address_space(4))) const TileArgs;

// The kernel's arguments read where they are used, from the kernarg segment
// (scalar loads), through a pointer the compiler cannot see through: values
// used once per piece are not kept in SGPRs across the ring loop, which needs
// all of them (kept live across the piece loop they spilled)
__device__ __forceinline__ TileArgsK *tile_args()
{
    uint64_t p = reinterpret_cast<uint64_t>(__builtin_amdgcn_kernarg_segment_ptr());
    asm volatile("" : "+s"(p));
    return reinterpret_cast<TileArgsK *>(p);
}

template <int K, bool BDMA>
__global__ __launch_bounds__(kTileWaves * kWave) void bwd_tile_kernel(const TileArgs)
{
    __shared__ __attribute__((aligned(16))) float tb[kTileBufs * kTileBufRows * kMaxDim];
    // this workgroup's range of the (group, source row) space: the pieces of
    // groups g_first .. g_last (tile_format.h), one after the other.  The
    // piece loop's state lives in LDS, not in registers: the ring loop below
    // uses every SGPR and VGPR a wave has (state in registers spilled)
    __shared__ int tstate[kTileWaves][4];  // next group, last group, workgroup
    {
        const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        TileArgsK *A = tile_args();
        const int wg = blockIdx.x, num_rows = A->num_rows;
        const int64_t gv = (int64_t)A->num_groups * num_rows;
        const int64_t x0 = tile_wg_start(wg, gv, A->num_wgs);
        const int64_t x1 = tile_wg_start(wg + 1, gv, A->num_wgs);
        if (x1 <= x0) return;
        if (lane_id() == 0) {
            tstate[wv][0] = (int)(x0 / num_rows);
            tstate[wv][1] = (int)((x1 - 1) / num_rows);
            tstate[wv][2] = wg;
        }
    }
    for (;;) {
        // lane constants recomputed per piece from an opaque copy: hoisted out of
        // this loop, the values derived from them (selector and output addresses)
        // stayed live across it and spilled
        const int lane = lane_id();
        int lane_o = lane;
        asm volatile("" : "+v"(lane_o));
        const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        const int half = K == 32 ? lane_o >> 5 : 0, ent = lane_o & (K - 1);
        const uint64_t lo = K == 32 ? 0x00000000ffffffffull : ~0ull;
        const uint64_t hi = K == 32 ? 0xffffffff00000000ull : ~0ull;
        auto dest_of = [&](int slot) { return (K == 32 ? 2 * slot + half : slot) * kTileWaves + wv; };
        TileArgsK *A = tile_args();
        const int grp = __builtin_amdgcn_readfirstlane(tstate[wv][0]);
        const int wg = __builtin_amdgcn_readfirstlane(tstate[wv][2]);
        if (lane == 0) tstate[wv][0] = grp + 1;
        const int pid = grp + wg;
        const int plane = wg - (int)((int64_t)grp * A->num_wgs / A->num_groups);
        const int d0 = grp * A->group_size;
        const int nd = min(A->group_size, A->num_cols - d0);
        const uint8_t *__restrict__ sel = A->sel;
        const float *__restrict__ grad = A->grad;
        const float *__restrict__ zero_row = A->zero_row;
        const int num_rows = A->num_rows;
        // selectors of the group's destinations, staged through LDS (tb is free
        // until the first DMA); slot s = 4t + b of this wave holds destination
        // (2s + half) * 16 + wv, byte b of selector word t
        {
            uint8_t *sb = reinterpret_cast<uint8_t *>(tb);
            constexpr int U = K / 16;  // 16-B units per selector row; 4096 units either way
            for (int i = threadIdx.x; i < 64 * kTileWaves * 4; i += kTileWaves * kWave) {
                const int j = i / U;
                uint4 v = {0u, 0u, 0u, 0u};
                if (j < nd) v = *reinterpret_cast<const uint4 *>(sel + (size_t)(d0 + j) * K + (i % U) * 16);
                *reinterpret_cast<uint4 *>(sb + (size_t)i * 16) = v;
            }
            __syncthreads();
        }
        tile_sel_t selv;
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const uint8_t *sb = reinterpret_cast<const uint8_t *>(tb);
            uint32_t word = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b)
                word |= (uint32_t)sb[dest_of(4 * t + b) * K + ent] << (8 * b);
            selv[t] = word;
            asm volatile("" ::: "memory");  // four LDS reads in flight at a time
        }
        __syncthreads();
        tile_acc_t acc0 = 0.f, acc1 = 0.f;
        const uint32_t tb_base = (uint32_t)reinterpret_cast<uintptr_t>(tb);
        const int bw = pid * kTileWaves + wv;
        const tile_hdr_t *hs = A->hdrs + A->hdr_start[bw];
        const uint32_t *rb = A->recs + kTileRecWords * A->rec_start[bw];
        uint32_t ro = 0;  // byte offset of the next record group in this wave's stream
        const int nch = A->num_chunks[pid];
        // raw buffer descriptor of the gradient: base, stride 0, num_records = its bytes
        const uint64_t gbase = reinterpret_cast<uint64_t>(grad);
        const tile_rsrc_t rsrc = {(int32_t)(uint32_t)gbase, (int32_t)(uint32_t)(gbase >> 32) & 0xffff,
                                  BDMA ? (int32_t)((uint32_t)num_rows * 1024u) : 0, 0x00020000};
        const uint32_t lane16 = (uint32_t)lane * 16u;
        // pieces of rows wv*3 .. wv*3+2 of the chunk's buffer (48 rows = 16 waves x 3)
        static_assert(!BDMA || kTileWaves * kTilePieces == kTileBufRows, "consecutive piece rows");
        auto bdma = [&](int c, const tile_hdr_t &h) {
            const uint32_t buf = tb_base + (uint32_t)(c % kTileBufs) * kTileBufRows * 1024u +
                                 (uint32_t)wv * 3u * 1024u;
            tile_bdma3(rsrc, ((uint32_t)h.y << 10) + lane16, ((uint32_t)h.z << 10) + lane16,
                       ((uint32_t)h.w << 10) + lane16, __builtin_amdgcn_readfirstlane(buf));
        };
        auto dma = [&](int c, int r0, int r1, int r2) {
            static_assert(kTilePieces == 3, "three DMA pieces per wave and chunk");
            const uint32_t buf = tb_base + (uint32_t)(c % kTileBufs) * kTileBufRows * 1024u;
            const int rows[3] = {r0, r1, r2};
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const int r = __builtin_amdgcn_readfirstlane(rows[i]);
                const float *src = r >= 0 ? grad + (size_t)r * kMaxDim : zero_row;
                // pieces past the buffer's rows (a ring of fewer than 48-row buffers)
                // all write the zero row again: same bytes, same place
                const int row = wv * 3 + i < kTileBufRows ? wv * 3 + i : kTileBufRows - 1;
                tile_glds(src + lane * 4,
                          __builtin_amdgcn_readfirstlane(buf + (uint32_t)row * 1024u));
            }
        };
        // records about 1 KB ahead pulled into L2 for the s_loads (one load per chunk)
        uint32_t pf = 0;
#ifndef TILE_PF_AHEAD
#define TILE_PF_AHEAD 128  // dwords: the window starts 512 B past the chunk's records
#endif
#ifndef TILE_KPF
    // record groups 3 and 4 pulled into the scalar cache with the first two (0 or 2; 4
    // measured no better): Reddit k=32 2.81 -> 2.78 ms
#define TILE_KPF 2
#endif
        // the window must stay inside the record stream's padding: 512 records =
        // 1024 dwords after the last wave's stream (kTileRecPad in maxk_plan.hip)
        static_assert(TILE_PF_AHEAD + 4 * kWave <= kTileRecWords * 512,
                      "TILE prefetch past the record padding");
#ifndef TILE_NO_PREFETCH
        auto prefetch = [&]() { tile_prefetch(rb + (ro >> 2) + TILE_PF_AHEAD + lane * 4, pf); };
#else
        auto prefetch = [&]() {};
#endif
        // header e(i) = {n0 | n1 << 16 of chunk i - L, the wave's DMA rows of chunk i},
        // L = kTileLead; queue: H(L); per "iteration" i = -L, ..., -1, 0, 1, ...:
        // DMA(i + L), H(i + 2L + 1), prefetch -- so every step issues the same ops
        tile_hdr_t e[kTileLead];   // plain loads, waited for by the compiler before any DMA
#pragma unroll
        for (int i = 0; i < kTileLead; ++i) e[i] = hs[i];
        tile_hdr_t hh[kTileBufs];
        hh[0] = tile_load_hdr(hs + kTileLead);
#pragma unroll
        for (int i = 0; i < kTileLead; ++i) {
            if constexpr (BDMA)
                bdma(i, e[i]);
            else
                dma(i, e[i].y, e[i].z, e[i].w);
            hh[i + 1] = tile_load_hdr(hs + kTileLead + 1 + i);
            prefetch();
        }
        auto step = [&](int c, tile_hdr_t &h) {
            // the chunk's first record groups, in flight across the barrier (four-word
            // records: pinned to s[64:79] / s[80:95], where the record asm reads them)
            tile_g16_t pa, pb;
#if TILE_KPF
            // groups 3..2+TILE_KPF pulled into the scalar cache with the first two, so
            // that the loop's s_loads hit it (their lgkmcnt waits also wait for the
            // LDS reads; a K$ hit keeps that short); dummies stay live to the wait
            uint32_t kp[4];
            const uint32_t *rp = rb + (ro >> 2);
            if constexpr (kTileRecWords == 4)
                asm volatile("s_load_dwordx16 s[64:79], %6, 0x0\n\t"
                             "s_load_dwordx16 s[80:95], %6, 0x40\n\t"
                             "s_load_dword %2, %6, 0x80\n\t"
                             "s_load_dword %3, %6, 0xc0\n\t"
                             ".if %7 > 2\n\t"
                             "s_load_dword %4, %6, 0x100\n\t"
                             "s_load_dword %5, %6, 0x140\n\t"
                             ".endif"
                             : "=&{s[64:79]}"(pa), "=&{s[80:95]}"(pb), "=&s"(kp[0]), "=&s"(kp[1]),
                               "=&s"(kp[2]), "=&s"(kp[3])
                             : "s"(rp), "n"(TILE_KPF) : "memory");
            else
#else
            if constexpr (kTileRecWords == 4)
                asm volatile("s_load_dwordx16 s[64:79], %2, %3\n\ts_load_dwordx16 s[80:95], %2, %4"
                             : "=&{s[64:79]}"(pa), "=&{s[80:95]}"(pb)
                             : "s"(rb), "s"(ro), "s"(ro + 64) : "memory");
            else
#endif
                asm volatile("s_load_dwordx16 %0, %2, %3\n\ts_load_dwordx16 %1, %2, %4"
                             : "=&s"(pa), "=&s"(pb) : "s"(rb), "s"(ro), "s"(ro + 64) : "memory");
            // this wave's DMA of chunk c and header of chunk c landed; after the
            // barrier everyone's have, and chunk c-1's buffer is free
            asm volatile("s_waitcnt vmcnt(%2)\n\ts_barrier" : "+v"(h), "+v"(pf) : "n"(kTileVmcnt)
                         : "memory");
            const uint32_t cnt = (uint32_t)__builtin_amdgcn_readfirstlane(h.x);
            // (every step must issue exactly 3 DMA + 1 header load + 1 prefetch: the
            // counted vmcnt above relies on it.  A step that issues fewer lets the wave
            // read a header that has not landed -> garbage record counts -> s_loads past
            // the record stream -> memory-access fault; measured with a "no DMA" ablation.)
            if constexpr (BDMA)
                bdma(c + kTileLead, h);
            else
                dma(c + kTileLead, __builtin_amdgcn_readfirstlane(h.y),
                    __builtin_amdgcn_readfirstlane(h.z), __builtin_amdgcn_readfirstlane(h.w));
            h = tile_load_hdr(hs + c + 2 * kTileLead + 1);
            prefetch();
            const uint32_t g0n = (cnt & 0xffffu) >> 2, gn = g0n + (cnt >> 18);
            uint32_t n = 0u - gn, m = 0u - g0n;
            // the record groups must have landed before anything reads (or copies)
            // their SGPRs -- also when this chunk has no records: a skipped wait let
            // the next step's s_loads into the same SGPRs race with these (SMEM
            // returns out of order), i.e. stale records, on graphs with empty
            // wave-chunks (products k=32: runs differed in the last bits)
            if constexpr (kTileRecWords == 4) {
#if TILE_KPF
                asm volatile("s_waitcnt lgkmcnt(0)" : "+{s[64:79]}"(pa), "+{s[80:95]}"(pb),
                             "+s"(kp[0]), "+s"(kp[1]), "+s"(kp[2]), "+s"(kp[3])::"memory");
#else
                asm volatile("s_waitcnt lgkmcnt(0)" : "+{s[64:79]}"(pa), "+{s[80:95]}"(pb)::"memory");
#endif
                tile_groups2_r16(pa, pb, n, m, lo, hi, selv, acc0, acc1);
                tile_group_loop_r16(rb, ro + 128, n, m, lo, hi, selv, acc0, acc1);
                ro += 64 * gn;
                return;
            }
            asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(pa), "+s"(pb)::"memory");
            uint32_t ga[16], gb[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                ga[i] = pa[i];
                gb[i] = pb[i];
            }
            tile_groups2(ga, n, m, lo, hi, selv, acc0, acc1);
            tile_groups2(gb, n, m, lo, hi, selv, acc0, acc1);
            tile_group_loop(rb, ro + 128, n, m, lo, hi, selv, acc0, acc1);
            ro += 32 * gn;
        };
        for (int c = 0; c < nch; c += kTileBufs) {
#pragma unroll
            for (int j = 0; j < kTileBufs; ++j)
                if (c + j < nch) step(c + j, hh[j]);
        }
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(pf)::"memory");
#pragma unroll
        for (int j = 0; j < kTileBufs; ++j) asm volatile("" : "+v"(hh[j])::"memory");
        TileArgsK *Z = tile_args();
        float *out = plane == 0 ? Z->dxs : Z->part + (size_t)(plane - 1) * Z->num_cols * K;
#pragma unroll
        for (int s = 0; s < 64; ++s) {
            const int j = dest_of(s);
            if (j < nd) out[(size_t)(d0 + j) * K + ent] = s < 32 ? acc0[s] : acc1[s - 32];
        }
        if (__builtin_amdgcn_readfirstlane(tstate[wv][0]) >
            __builtin_amdgcn_readfirstlane(tstate[wv][1]))
            break;
        __syncthreads();   // every wave's ring reads of this piece are done
    }
}

// dxs += the partial planes of each destination's group (tile_group_planes of
// them, in plane order: deterministic)
__global__ __launch_bounds__(kBlock) void tile_combine_kernel(float *__restrict__ dxs,
                                                              const float *__restrict__ part,
                                                              int64_t n4, int k, int group_size,
                                                              int num_rows, int num_groups,
                                                              int num_wgs)
{
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n4;
         i += (int64_t)gridDim.x * kBlock) {
        const int g = (int)(i * 4 / k) / group_size;
        const int np = tile_group_planes(g, num_rows, num_groups, num_wgs);
        if (np == 0) continue;
        f4 a = reinterpret_cast<f4 *>(dxs)[i];
        for (int p = 0; p < np; ++p) a += reinterpret_cast<const f4 *>(part)[(int64_t)p * n4 + i];
        reinterpret_cast<f4 *>(dxs)[i] = a;
    }
}

// out = parts[0] + parts[1] + ... (in part order: deterministic), n floats
// per part -- the column-blocked forward's partial outputs (maxk_rows_sum)
template <bool VEC>
__global__ __launch_bounds__(kBlock) void rows_sum_kernel(const float *__restrict__ parts,
                                                          int nparts, int64_t n,
                                                          float *__restrict__ out)
{
    const int64_t items = VEC ? n / 4 : n;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < items;
         i += (int64_t)gridDim.x * kBlock) {
        if constexpr (VEC) {
            const f4 *p = reinterpret_cast<const f4 *>(parts);
            f4 a = __builtin_nontemporal_load(p + i);
            for (int q = 1; q < nparts; ++q)
                a += __builtin_nontemporal_load(p + (int64_t)q * (n / 4) + i);
            __builtin_nontemporal_store(a, reinterpret_cast<f4 *>(out) + i);
        } else {
            float a = parts[i];
            for (int q = 1; q < nparts; ++q) a += parts[(int64_t)q * n + i];
            out[i] = a;
        }
    }
}

template <int K>
__global__ __launch_bounds__(kBlock) void cbsr_pack_kernel(const float *__restrict__ data,
                                                           const uint8_t *__restrict__ sel,
                                                           int num_cols, uint8_t *__restrict__ rec)
{
    constexpr int RS = Packed<K>::RS;
    constexpr int W = RS / 4;  // dwords per record
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // dword of the output
    if (i >= (int64_t)num_cols * W) return;
    const int64_t c = i / W;
    const int w = (int)(i - c * W);
    uint32_t v = 0;
    if (w < K) {
        v = __builtin_bit_cast(uint32_t, data[c * K + w]);
    } else if (w < K + K / 4) {
        v = *reinterpret_cast<const uint32_t *>(sel + c * K + 4 * (w - K));
    }
    reinterpret_cast<uint32_t *>(rec)[i] = v;
}

// Halo records (multi-GPU exchange): record i = the CBSR row rows[i] as k fp32
// values then k selector bytes, 5k bytes unpadded (k a power of two >= 4, so
// records stay 4-B aligned and, for k >= 32, 16-B aligned).  The receiver's
// forward reads the records in place (fwd_panel_kernel<K, 5K>).
template <int K>
__global__ __launch_bounds__(kBlock) void cbsr_records_kernel(const float *__restrict__ data,
                                                              const uint8_t *__restrict__ sel,
                                                              const int32_t *__restrict__ rows,
                                                              int64_t n, uint8_t *__restrict__ rec)
{
    if constexpr (K % 16 == 0) {
        // 16-B pieces: K/4 of data, K/16 of selectors per record (products N=8:
        // 342 MB of records, 0.22 ms with 4-B pieces)
        constexpr int W = 5 * K / 16;
        const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        if (i >= n * W) return;
        const int64_t j = i / W;
        const int w = (int)(i - j * W);
        const int64_t c = rows ? rows[j] : j;
        const f4 v = w < K / 4 ? reinterpret_cast<const f4 *>(data + c * K)[w]
                               : reinterpret_cast<const f4 *>(sel + c * K)[w - K / 4];
        __builtin_nontemporal_store(v, reinterpret_cast<f4 *>(rec) + i);
    } else {
        constexpr int W = 5 * K / 4;  // dwords per record
        const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        if (i >= n * W) return;
        const int64_t j = i / W;
        const int w = (int)(i - j * W);
        const int64_t c = rows ? rows[j] : j;
        const uint32_t v = w < K ? __builtin_bit_cast(uint32_t, data[c * K + w])
                                 : *reinterpret_cast<const uint32_t *>(sel + c * K + 4 * (w - K));
        reinterpret_cast<uint32_t *>(rec)[i] = v;
    }
}

// out[i, :] = the selector bytes of record rows[i] (bytes 4K .. 5K of a 5K-byte
// record): 16-B pieces when K % 16 == 0, else dwords
template <int K>
__global__ __launch_bounds__(kBlock) void records_sel_kernel(const uint8_t *__restrict__ rec,
                                                             const int32_t *__restrict__ rows,
                                                             int64_t n, uint8_t *__restrict__ out)
{
    constexpr int PB = K % 16 == 0 ? 16 : 4;   // piece bytes
    constexpr int W = K / PB;                  // pieces per row
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n * W) return;
    const int64_t j = i / W;
    const int w = (int)(i - j * W);
    const uint8_t *src = rec + (size_t)rows[j] * (5 * K) + 4 * K + (size_t)w * PB;
    if constexpr (PB == 16)
        reinterpret_cast<f4 *>(out)[i] = *reinterpret_cast<const f4 *>(src);
    else
        reinterpret_cast<uint32_t *>(out)[i] = *reinterpret_cast<const uint32_t *>(src);
}

// dst[seg_row[s], :] += sum over j in [seg_off[s], seg_off[s+1]) of src[order[j], :]
// (width floats per row): the owners' sum of the halo partial sums their peers
// returned, in a fixed order (no atomics; index_add_ took 0.23 ms on products
// N=8).  One wave per segment.
// Lanes: 64 / width segments per wave (width <= 64), one column each; the
// segment's source rows are fetched 8 at a time so their loads overlap.
__global__ __launch_bounds__(kBlock) void segment_rows_add_kernel(
    const float *__restrict__ src, int width, const int64_t *__restrict__ order,
    const int64_t *__restrict__ seg_off, const int64_t *__restrict__ seg_row, int64_t num_seg,
    float *__restrict__ dst)
{
    const int spw = width <= kWave ? kWave / width : 1;          // segments per wave
    const int lane = lane_id();
    const int sub = width <= kWave ? lane / width : 0;
    const int64_t s = ((int64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave) * spw + sub;
    if (s >= num_seg || (width <= kWave && sub >= spw)) return;
    const int64_t j0 = seg_off[s], j1 = seg_off[s + 1];
    float *d = dst + seg_row[s] * width;
    for (int c = width <= kWave ? lane % width : lane; c < width; c += kWave) {
        float a = d[c];
        for (int64_t j = j0; j < j1; j += 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = j + u < j1 ? src[order[j + u] * width + c] : 0.f;
#pragma unroll
            for (int u = 0; u < 8; ++u) a += v[u];
        }
        d[c] = a;
    }
}

// dXs zeroing for the ATOMIC backward / empty graphs.  A kernel rather than
// hipMemsetAsync: captured into a hipGraph, the memset node was not reliably
// ordered before the following atomics (wrong results in about half of the
// replays; eager runs always right -- tools/exp_graph_flaky.py).
__global__ __launch_bounds__(kBlock) void zero_kernel(float *__restrict__ p, size_t n)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = 0.f;
}

// ---------------------------------------------------------------------------
// Host-side dispatch
// ---------------------------------------------------------------------------
inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

inline int launch_status()
{
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MAXK_OK : (int)e;
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

inline int zero_floats(float *p, size_t n, hipStream_t st)
{
    if (n == 0) return MAXK_OK;
    const int64_t blocks = ceil_div((int64_t)n, kBlock);
    hipLaunchKernelGGL(zero_kernel, dim3((unsigned)(blocks < 4096 ? blocks : 4096)), dim3(kBlock),
                       0, st, p, n);
    return launch_status();
}

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

inline bool dims_ok(int dim, int k) { return dim >= 1 && dim <= kMaxDim && k >= 1 && k <= dim; }

template <template <int> class F, typename... Args>
int dispatch_k(int k, Args &&...args)
{
    switch (k) {
    case 4: return F<4>::run(args...);
    case 8: return F<8>::run(args...);
    case 16: return F<16>::run(args...);
    case 32: return F<32>::run(args...);
    case 64: return F<64>::run(args...);
    case 128: return F<128>::run(args...);
    case 256: return F<256>::run(args...);
    default: return F<0>::run(args...);
    }
}

size_t row_lds_bytes() { return (size_t)kWavesPerBlock * kMaxDim * sizeof(float); }

template <int K>
size_t fwd_lds_bytes(int k) { return (size_t)kWavesPerBlock * fwd_copies<K>(k) * kMaxDim * sizeof(float); }

inline int fwd_fixup(const int32_t *sched, int64_t P, const float *carry, const float *owner,
                     const int32_t *carry_row, float *out, int dim, bool acc, hipStream_t st,
                     int num_rows = 0, const float *sump = nullptr, int nsump = 0)
{
    const int64_t blocks = ceil_div(P, kWavesPerBlock);
    const int dimp = (dim + 3) & ~3;
    const int2 *sc = reinterpret_cast<const int2 *>(sched);
    if (acc)
        hipLaunchKernelGGL(carry_fixup_owner_kernel<true>, dim3((unsigned)blocks), dim3(kBlock), 0,
                           st, sc, P, carry, owner, carry_row, out, dim, dimp, num_rows,
                           (const float *)nullptr, 0);
    else
        hipLaunchKernelGGL(carry_fixup_owner_kernel<false>, dim3((unsigned)blocks), dim3(kBlock), 0,
                           st, sc, P, carry, owner, carry_row, out, dim, dimp, num_rows, sump, nsump);
    return launch_status();
}

template <int K>
struct FwdPanel {
    static int run(const int32_t *sched, int64_t P, const int32_t *indptr, const int32_t *idx,
                   const float *val, const float *data, const uint8_t *sel, int V, int dim, int k,
                   float *out, float *carry, int32_t *carry_row, float *owner, bool acc,
                   hipStream_t st, uint8_t *esel = nullptr, bool cached = false,
                   const float *sump = nullptr, int nsump = 0)
    {
        const int64_t blocks = ceil_div(P, kWavesPerBlock);
        auto kern = esel ? fwd_panel_kernel<K, 0, false, true>
                    : cached ? (acc ? fwd_panel_kernel<K, 0, true, false, false>
                                    : fwd_panel_kernel<K, 0, false, false, false>)
                    : acc ? fwd_panel_kernel<K, 0, true> : fwd_panel_kernel<K, 0, false>;
        hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kBlock), fwd_lds_bytes<K>(k), st,
                           reinterpret_cast<const int2 *>(sched), P, indptr, idx, val, data, sel,
                           V, dim, k, out, carry, carry_row, owner, esel, sump, nsump);
        int rc = launch_status();
        if (rc) return rc;
        return fwd_fixup(sched, P, carry, owner, carry_row, out, dim, acc, st, V, sump, nsump);
    }
};

template <int K>
struct FwdPanelPacked {
    static int run(const int32_t *sched, int64_t P, const int32_t *indptr, const int32_t *idx,
                   const float *val, const uint8_t *rec, int V, int dim, int k, float *out,
                   float *carry, int32_t *carry_row, float *owner, hipStream_t st,
                   uint8_t *esel = nullptr)
    {
        if constexpr (Packed<K>::RS == 0) {
            return MAXK_E_DIM;
        } else {
            constexpr int RS = Packed<K>::RS;
            const int64_t blocks = ceil_div(P, kWavesPerBlock);
            auto kern = esel ? fwd_panel_kernel<K, RS, false, true> : fwd_panel_kernel<K, RS>;
            hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kBlock),
                               fwd_lds_bytes<K>(k), st, reinterpret_cast<const int2 *>(sched), P,
                               indptr, idx, val, reinterpret_cast<const float *>(rec),
                               rec + 4 * K, V, dim, k, out, carry, carry_row, owner, esel,
                               (const float *)nullptr, 0);
            int rc = launch_status();
            if (rc) return rc;
            return fwd_fixup(sched, P, carry, owner, carry_row, out, dim, false, st);
        }
    }
};

template <int K>
struct FwdRecords {
    static int run(const int32_t *sched, int64_t P, const int32_t *indptr, const int32_t *idx,
                   const float *val, const uint8_t *rec, int V, int dim, int k, bool acc,
                   float *out, float *carry, int32_t *carry_row, float *owner, hipStream_t st)
    {
        if constexpr (K == 0) {
            return MAXK_E_DIM;
        } else {
            constexpr int RS = 5 * K;
            const int64_t blocks = ceil_div(P, kWavesPerBlock);
            auto kern = acc ? fwd_panel_kernel<K, RS, true> : fwd_panel_kernel<K, RS, false>;
            hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kBlock), fwd_lds_bytes<K>(k), st,
                               reinterpret_cast<const int2 *>(sched), P, indptr, idx, val,
                               reinterpret_cast<const float *>(rec), rec + 4 * K, V, dim, k, out,
                               carry, carry_row, owner, (uint8_t *)nullptr, (const float *)nullptr, 0);
            int rc = launch_status();
            if (rc) return rc;
            return fwd_fixup(sched, P, carry, owner, carry_row, out, dim, acc, st);
        }
    }
};

template <int K>
struct CbsrRecords {
    static int run(const float *data, const uint8_t *sel, const int32_t *rows, int64_t n,
                   uint8_t *rec, hipStream_t st)
    {
        if constexpr (K == 0) {
            return MAXK_E_DIM;
        } else {
            const int64_t words = n * (K % 16 == 0 ? 5 * K / 16 : 5 * K / 4);
            hipLaunchKernelGGL(cbsr_records_kernel<K>, dim3((unsigned)ceil_div(words, kBlock)),
                               dim3(kBlock), 0, st, data, sel, rows, n, rec);
            return launch_status();
        }
    }
};

template <int K>
struct CbsrPack {
    static int run(const float *data, const uint8_t *sel, int num_cols, uint8_t *rec, hipStream_t st)
    {
        if constexpr (Packed<K>::RS == 0) {
            return MAXK_E_DIM;
        } else {
            const int64_t n = (int64_t)num_cols * (Packed<K>::RS / 4);
            hipLaunchKernelGGL(cbsr_pack_kernel<K>, dim3((unsigned)ceil_div(n, kBlock)), dim3(kBlock),
                               0, st, data, sel, num_cols, rec);
            return launch_status();
        }
    }
};

template <int K>
struct FwdMulti {
    template <int R4>
    static int launch_rel4(const int2 *sc, int64_t P, const int32_t *indptr, const int32_t *idx,
                           const float *val, const float *data, const uint8_t *sel, int V,
                           int dim, float *out, float *carry, int32_t *carry_row, hipStream_t st)
    {
        using C = Rel4<K, R4>;
        const size_t lds = (size_t)kWavesPerBlock * C::EPS * C::ROW * sizeof(float);
        if (lds > 160 * 1024) return -1;  // nothing launched; the caller falls back
        hipLaunchKernelGGL((fwd_rel4_panel_kernel<K, R4>), dim3((unsigned)ceil_div(P, kWavesPerBlock)),
                           dim3(kBlock), lds, st, sc, P, indptr, idx, val, data, sel, V, dim, out,
                           carry, carry_row);
        return launch_status();
    }

    static int run(const int32_t *sched, int64_t P, const int32_t *indptr, const int32_t *idx,
                   const float *val, int R, const float *data, const uint8_t *sel, int V,
                   int dim, float *out, float *carry, int32_t *carry_row, hipStream_t st)
    {
        if constexpr (K == 0) {
            return MAXK_E_DIM;  // the fused kernel is compiled for k = 4, 8, ..., 256
        } else {
            const int64_t blocks = ceil_div(P, kWavesPerBlock);
            const int2 *sc = reinterpret_cast<const int2 *>(sched);
            int rc = MAXK_OK;
            bool done = false;
            if ((R & 3) == 0 && (reinterpret_cast<uintptr_t>(val) & 15) == 0) {
                done = true;
                switch (R / 4) {
                case 1: rc = launch_rel4<1>(sc, P, indptr, idx, val, data, sel, V, dim, out, carry, carry_row, st); break;
                case 2: rc = launch_rel4<2>(sc, P, indptr, idx, val, data, sel, V, dim, out, carry, carry_row, st); break;
                case 4: rc = launch_rel4<4>(sc, P, indptr, idx, val, data, sel, V, dim, out, carry, carry_row, st); break;
                default: done = false;
                }
                if (rc == -1) done = false;  // LDS too large for this (k, R): generic kernel
            }
            if (!done) {
                const size_t lds = (size_t)kWavesPerBlock * R * kMultiRow * sizeof(float);
                hipLaunchKernelGGL(fwd_multi_panel_kernel<K>, dim3((unsigned)blocks), dim3(kBlock),
                                   lds, st, sc, P, indptr, idx, val, R, data, sel, V, dim, out,
                                   carry, carry_row);
                rc = launch_status();
            }
            if (rc) return rc;
            hipLaunchKernelGGL(carry_fixup_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, st, P,
                               carry, carry_row, out, dim, (dim + 3) & ~3, R, (size_t)V * dim);
            return launch_status();
        }
    }
};

template <int K>
struct FwdWarp4 {
    static int run(const int32_t *warp4, int W, const int32_t *idx, const float *val,
                   const float *data, const uint8_t *sel, int dim, int k, float *out,
                   hipStream_t st)
    {
        const int run = 16;
        const int64_t waves = ceil_div(W, run);
        hipLaunchKernelGGL(fwd_warp4_kernel<K>, dim3((unsigned)ceil_div(waves, kWavesPerBlock)),
                           dim3(kBlock), fwd_lds_bytes<K>(k), st,
                           reinterpret_cast<const int4 *>(warp4), W, run, idx, val, data, sel,
                           dim, k, out);
        return launch_status();
    }
};

template <int K>
struct BwdPanel {
    static int run(bool staged, const int32_t *sched, int64_t P, const int32_t *indptr,
                   const int32_t *idx, const float *val, const float *grad, const uint8_t *sel,
                   const int32_t *csc_pos, int V, int dim, int k, float *dxs, float *Pbuf,
                   hipStream_t st, bool esel = false, int pm = kPmCsc)
    {
        const int64_t blocks = ceil_div(P, kWavesPerBlock);
        if (pm == kPmEdge) {  // EDGE_GATHER phase 1 (edge selectors, P in edge order)
            if constexpr (K == 0) {
                return MAXK_E_DIM;
            } else {
                hipLaunchKernelGGL((bwd_panel_kernel<K, true, true, kPmEdge>), dim3((unsigned)blocks),
                                   dim3(kBlock), row_lds_bytes(), st,
                                   reinterpret_cast<const int2 *>(sched), P, indptr, idx, val,
                                   grad, sel, csc_pos, V, dim, k, dxs, Pbuf);
                return launch_status();
            }
        }
        if (staged && esel)
            hipLaunchKernelGGL((bwd_panel_kernel<K, true, true>), dim3((unsigned)blocks),
                               dim3(kBlock), row_lds_bytes(), st,
                               reinterpret_cast<const int2 *>(sched), P, indptr, idx, val, grad,
                               sel, csc_pos, V, dim, k, dxs, Pbuf);
        else if (staged)
            hipLaunchKernelGGL((bwd_panel_kernel<K, true>), dim3((unsigned)blocks), dim3(kBlock),
                               row_lds_bytes(), st, reinterpret_cast<const int2 *>(sched), P,
                               indptr, idx, val, grad, sel, csc_pos, V, dim, k, dxs, Pbuf);
        else
            hipLaunchKernelGGL((bwd_panel_kernel<K, false>), dim3((unsigned)blocks), dim3(kBlock),
                               row_lds_bytes(), st, reinterpret_cast<const int2 *>(sched), P,
                               indptr, idx, val, grad, sel, csc_pos, V, dim, k, dxs, Pbuf);
        return launch_status();
    }
};

template <int K>
struct BwdSegsum {
    static int run(const int32_t *csched, int64_t CP, const int32_t *cptr, const float *Pbuf,
                   int V, int k, float *dxs, float *carry, int32_t *carry_row, hipStream_t st,
                   const int32_t *perm = nullptr)
    {
        const int64_t blocks = ceil_div(CP, kWavesPerBlock);
        if (perm) {
            if constexpr (K == 0) {
                return MAXK_E_DIM;
            } else {
                hipLaunchKernelGGL((bwd_segsum_kernel<K, true>), dim3((unsigned)blocks),
                                   dim3(kBlock), 0, st, reinterpret_cast<const int2 *>(csched), CP,
                                   cptr, Pbuf, V, k, dxs, carry, carry_row, perm);
            }
        } else {
            hipLaunchKernelGGL(bwd_segsum_kernel<K>, dim3((unsigned)blocks), dim3(kBlock), 0, st,
                               reinterpret_cast<const int2 *>(csched), CP, cptr, Pbuf, V, k, dxs,
                               carry, carry_row, (const int32_t *)nullptr);
        }
        int rc = launch_status();
        if (rc) return rc;
        hipLaunchKernelGGL(carry_fixup_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, st, CP,
                           carry, carry_row, dxs, k, k);
        return launch_status();
    }
};

// APPEND backward (MAXK_BWD_APPEND): per-graph plan = the region base of every
// (bin, XCD group); per call: cursors reset, phase 1 (single relation, node or
// edge selectors; or R in {4, 8, 16} relations summed per edge), phase 2.
// One panel per wave as everywhere; the XCD group of panel w is (w / 4) % 8.
__global__ __launch_bounds__(kBlock) void append_count_kernel(
    const int2 *__restrict__ sched, int64_t num_panels, const int32_t *__restrict__ idx,
    AppendArgs ap, int32_t *__restrict__ counts)
{
    const int64_t w = (int64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave;
    if (w >= num_panels) return;
    const int j0 = sched[w].y, j1 = sched[w + 1].y;
    const int grp = (int)(blockIdx.x & (kAppendGroups - 1));
    for (int e = j0 + lane_id(); e < j1; e += kWave)
        atomicAdd(counts + (size_t)append_bin(idx[e], ap) * kAppendGroups + grp, 1);
}

inline uint32_t append_magic(int bin_size)
{
    const uint64_t m = (1ull << 32) / (uint64_t)bin_size;
    return m > 0xffffffffull ? 0xffffffffu : (uint32_t)m;
}

template <int K>
struct BwdAppend {
    template <int R>
    static void launch_multi(unsigned blocks, const int2 *sc, int64_t P, const int32_t *indptr,
                             const int32_t *idx, const float *val, const float *grad,
                             int64_t plane, const uint8_t *sel, int V, int dim, float *Pbuf,
                             const AppendArgs &ap, hipStream_t st)
    {
        const size_t lds = (size_t)kWavesPerBlock * kMaxDim * R * sizeof(float);
        hipLaunchKernelGGL((bwd_multi_append_kernel<K, R>), dim3(blocks), dim3(kBlock), lds, st,
                           sc, P, indptr, idx, val, grad, plane, sel, V, dim, Pbuf, ap);
    }
    static int run(const int32_t *sched, int64_t P, const int32_t *indptr, const int32_t *idx,
                   const float *val, int num_rel, const float *grad, const uint8_t *sel,
                   bool esel, int V, int C, int dim, const int32_t *region_base, int num_bins,
                   int bin_size, float *dxs, float *Pbuf, int32_t *dst, int32_t *cursor,
                   hipStream_t st)
    {
        if constexpr (K < 4) {
            return MAXK_E_DIM;
        } else {
            const int ng = num_bins * kAppendGroups;
            hipLaunchKernelGGL(append_reset_kernel, dim3((unsigned)ceil_div(ng, kBlock)),
                               dim3(kBlock), 0, st, region_base, ng, cursor);
            int rc = launch_status();
            if (rc) return rc;
            const AppendArgs ap{append_magic(bin_size), bin_size, cursor, dst};
            const unsigned blocks = (unsigned)ceil_div(P, kWavesPerBlock);
            const int2 *sc = reinterpret_cast<const int2 *>(sched);
            if (num_rel == 1) {
                if (esel)
                    hipLaunchKernelGGL((bwd_append_kernel<K, true>), dim3(blocks), dim3(kBlock),
                                       row_lds_bytes(), st, sc, P, indptr, idx, val, grad, sel, V,
                                       dim, Pbuf, ap);
                else
                    hipLaunchKernelGGL((bwd_append_kernel<K, false>), dim3(blocks), dim3(kBlock),
                                       row_lds_bytes(), st, sc, P, indptr, idx, val, grad, sel, V,
                                       dim, Pbuf, ap);
            } else {
                if constexpr (K < 8 || K > 64) {
                    return MAXK_E_DIM;
                } else {
                    const int64_t plane = (int64_t)V * dim;
                    switch (num_rel) {
                    case 4: launch_multi<4>(blocks, sc, P, indptr, idx, val, grad, plane, sel, V, dim, Pbuf, ap, st); break;
                    case 8: launch_multi<8>(blocks, sc, P, indptr, idx, val, grad, plane, sel, V, dim, Pbuf, ap, st); break;
                    case 16: launch_multi<16>(blocks, sc, P, indptr, idx, val, grad, plane, sel, V, dim, Pbuf, ap, st); break;
                    default: return MAXK_E_ARG;
                    }
                }
            }
            rc = launch_status();
            if (rc) return rc;
            hipLaunchKernelGGL(bwd_bin_reduce_kernel<K>, dim3((unsigned)num_bins),
                               dim3(kReduceThreads), (size_t)bin_size * K * sizeof(float), st,
                               region_base, bin_size, C, dst, Pbuf, dxs);
            return launch_status();
        }
    }
};

// Phase 1 of the multi-relation STAGED backward (R in {4, 8, 16}, k in {8, 16,
// 32, 64}); phase 2 is BwdSegsum.
template <int K>
struct BwdMultiStage {
    template <int R>
    static int launch(bool edge_order, const int2 *sc, int64_t P, const int32_t *indptr,
                      const int32_t *idx, const float *val, const float *grad, int64_t plane,
                      const uint8_t *sel, const int32_t *csc_pos, int V, int dim, float *Pbuf,
                      hipStream_t st)
    {
        const unsigned blocks = (unsigned)ceil_div(P, kWavesPerBlock);
        const size_t lds = (size_t)kWavesPerBlock * kMaxDim * R * sizeof(float);
        if (edge_order)
            hipLaunchKernelGGL((bwd_multi_stage_kernel<K, R, kPmEdge>), dim3(blocks), dim3(kBlock),
                               lds, st, sc, P, indptr, idx, val, grad, plane, sel, csc_pos, V, dim,
                               Pbuf);
        else
            hipLaunchKernelGGL((bwd_multi_stage_kernel<K, R, kPmCsc>), dim3(blocks), dim3(kBlock),
                               lds, st, sc, P, indptr, idx, val, grad, plane, sel, csc_pos, V, dim,
                               Pbuf);
        return launch_status();
    }

    static int run(int R, bool edge_order, const int32_t *sched, int64_t P, const int32_t *indptr,
                   const int32_t *idx, const float *val, const float *grad, int64_t plane,
                   const uint8_t *sel, const int32_t *csc_pos, int V, int dim, float *Pbuf,
                   hipStream_t st)
    {
        if constexpr (K != 8 && K != 16 && K != 32 && K != 64) {
            return MAXK_E_DIM;
        } else {
            const int2 *sc = reinterpret_cast<const int2 *>(sched);
            switch (R) {
            case 4: return launch<4>(edge_order, sc, P, indptr, idx, val, grad, plane, sel, csc_pos, V, dim, Pbuf, st);
            case 8: return launch<8>(edge_order, sc, P, indptr, idx, val, grad, plane, sel, csc_pos, V, dim, Pbuf, st);
            case 16: return launch<16>(edge_order, sc, P, indptr, idx, val, grad, plane, sel, csc_pos, V, dim, Pbuf, st);
            default: return MAXK_E_ARG;
            }
        }
    }
};

template <int K>
struct BwdLocal {
    static int run(const int32_t *seg_off, int NS, const int32_t *dstart, int W, int dmax,
                   const int32_t *erc, const float *evl, const float *grad, const uint8_t *sel,
                   int num_rows, int dim, float *dxs, hipStream_t st)
    {
        const size_t region = (size_t)((dmax * K * 5 + 15) & ~15);
        const bool wide = (uint64_t)num_rows * (uint64_t)dim * 4u >= (1ull << 32);
        for (int s = 0; s < NS; ++s) {
            auto kern = wide ? bwd_local_kernel<K, true> : bwd_local_kernel<K, false>;
            hipLaunchKernelGGL(kern, dim3((unsigned)ceil_div(W, kWavesPerBlock)),
                               dim3(kBlock), region * kWavesPerBlock, st,
                               seg_off + (size_t)s * W, seg_off + (size_t)(s + 1) * W, s == 0,
                               dstart, W, dmax, erc, evl, grad, sel, dim, dxs);
            const int rc = launch_status();
            if (rc) return rc;
        }
        return MAXK_OK;
    }
};

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

const char *maxk_version(void) { return MAXK_VERSION_STRING; }

int maxk_abi_version(void) { return MAXK_ABI_VERSION; }

int maxk_schedule_num_panels(int64_t num_rows, int64_t num_edges, int panel_cost, int row_cost,
                             int64_t *num_panels)
{
    if (!num_panels || num_rows < 0 || num_edges < 0 || panel_cost < 1 || row_cost < 1)
        return MAXK_E_ARG;
    const int64_t total = num_edges + num_rows * (int64_t)row_cost;
    int64_t p = ceil_div(total, panel_cost);
    *num_panels = p < 1 ? 1 : p;
    return MAXK_OK;
}

int maxk_schedule_build(const int32_t *indptr, int num_rows, int panel_cost, int row_cost,
                        int32_t *sched, int64_t num_panels, void *stream)
{
    if (!indptr || !sched || num_rows < 0 || panel_cost < 1 || row_cost < 1 || num_panels < 1)
        return MAXK_E_ARG;
    const int64_t n = num_panels + 1;
    hipLaunchKernelGGL(schedule_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0,
                       as_stream(stream), indptr, num_rows, panel_cost, row_cost,
                       reinterpret_cast<int2 *>(sched), num_panels);
    return launch_status();
}

int maxk_warp4_build(const int32_t *indptr, int num_rows, int warp_max_nz, int32_t *chunk_offsets,
                     int32_t *warp4, int64_t warp4_capacity, int64_t *num_warps, void *stream)
{
    if (!indptr || !chunk_offsets || !num_warps || num_rows < 0 || warp_max_nz < 1)
        return MAXK_E_ARG;
    hipStream_t st = as_stream(stream);
    if (num_rows == 0) { *num_warps = 0; return MAXK_OK; }
    hipLaunchKernelGGL(warp4_count_kernel, dim3((unsigned)ceil_div(num_rows, 256)), dim3(256), 0,
                       st, indptr, num_rows, warp_max_nz, chunk_offsets);
    int rc = launch_status();
    if (rc) return rc;
    hipLaunchKernelGGL(exclusive_scan_1block, dim3(1), dim3(256), 0, st, chunk_offsets, num_rows,
                       chunk_offsets + num_rows);
    rc = launch_status();
    if (rc) return rc;
    int32_t total = 0;
    hipError_t e = hipMemcpyAsync(&total, chunk_offsets + num_rows, sizeof(int32_t),
                                  hipMemcpyDeviceToHost, st);
    if (e != hipSuccess) return (int)e;
    e = hipStreamSynchronize(st);
    if (e != hipSuccess) return (int)e;
    *num_warps = total;
    if (!warp4) return MAXK_OK;  // count-only call
    if (warp4_capacity < total) return MAXK_E_WORKSPACE;
    hipLaunchKernelGGL(warp4_fill_kernel, dim3((unsigned)ceil_div(num_rows, 256)), dim3(256), 0,
                       st, indptr, num_rows, warp_max_nz, chunk_offsets,
                       reinterpret_cast<int4 *>(warp4));
    return launch_status();
}

size_t maxk_forward_workspace_bytes(int64_t num_panels, int dim_origin)
{
    // carry rows | carry row ids | owner parts of split rows
    const size_t dimp = (size_t)((dim_origin + 3) & ~3);
    return 2 * align_up((size_t)num_panels * dimp * sizeof(float), 256) +
           align_up((size_t)num_panels * sizeof(int32_t), 256);
}

namespace {
inline float *fwd_owner_slots(void *workspace, int64_t num_panels, int dim_origin)
{
    const size_t dimp = (size_t)((dim_origin + 3) & ~3);
    return reinterpret_cast<float *>(static_cast<char *>(workspace) +
                                     align_up((size_t)num_panels * dimp * sizeof(float), 256) +
                                     align_up((size_t)num_panels * sizeof(int32_t), 256));
}
}  // namespace

int maxk_spgemm_forward(const int32_t *sched, int64_t num_panels, const int32_t *indptr,
                        const int32_t *indices, const float *values, const float *cbsr_data,
                        const uint8_t *cbsr_sel, int num_rows, int dim_origin, int dim_k,
                        float *out, void *workspace, size_t workspace_bytes, void *stream)
{
    return maxk_spgemm_forward_ex(sched, num_panels, indptr, indices, values, cbsr_data, cbsr_sel,
                                  num_rows, dim_origin, dim_k, 0, out, workspace, workspace_bytes,
                                  stream);
}

int maxk_spgemm_forward_ex(const int32_t *sched, int64_t num_panels, const int32_t *indptr,
                           const int32_t *indices, const float *values, const float *cbsr_data,
                           const uint8_t *cbsr_sel, int num_rows, int dim_origin, int dim_k,
                           int flags, float *out, void *workspace, size_t workspace_bytes,
                           void *stream)
{
    if (flags & ~(MAXK_FWD_ACCUMULATE | MAXK_FWD_CACHED_GATHER)) return MAXK_E_ARG;
    if (!sched || !indptr || !out || num_panels < 1 || num_rows < 0) return MAXK_E_ARG;
    if (!dims_ok(dim_origin, dim_k)) return MAXK_E_DIM;
    if (num_rows == 0) return MAXK_OK;
    if (!indices || !values || !cbsr_data || !cbsr_sel) return MAXK_E_ARG;
    if (!workspace || workspace_bytes < maxk_forward_workspace_bytes(num_panels, dim_origin))
        return MAXK_E_WORKSPACE;
    const size_t dimp = (size_t)((dim_origin + 3) & ~3);
    float *carry = static_cast<float *>(workspace);
    int32_t *carry_row = reinterpret_cast<int32_t *>(
        static_cast<char *>(workspace) + align_up((size_t)num_panels * dimp * sizeof(float), 256));
    return dispatch_k<FwdPanel>(dim_k, sched, num_panels, indptr, indices, values, cbsr_data,
                                cbsr_sel, num_rows, dim_origin, dim_k, out, carry, carry_row,
                                fwd_owner_slots(workspace, num_panels, dim_origin),
                                (flags & MAXK_FWD_ACCUMULATE) != 0, as_stream(stream),
                                (uint8_t *)nullptr, (flags & MAXK_FWD_CACHED_GATHER) != 0);
}

int maxk_spgemm_forward_sum_parts(const int32_t *sched, int64_t num_panels, const int32_t *indptr,
                                  const int32_t *indices, const float *values,
                                  const float *cbsr_data, const uint8_t *cbsr_sel, int num_rows,
                                  int dim_origin, int dim_k, int flags, const float *parts,
                                  int num_parts, float *out, void *workspace,
                                  size_t workspace_bytes, void *stream)
{
    if (flags & ~MAXK_FWD_CACHED_GATHER) return MAXK_E_ARG;
    if (num_parts < 0 || (num_parts > 0 && !parts)) return MAXK_E_ARG;
    if (!sched || !indptr || !out || num_panels < 1 || num_rows < 0) return MAXK_E_ARG;
    if (!dims_ok(dim_origin, dim_k)) return MAXK_E_DIM;
    if (num_rows == 0) return MAXK_OK;
    if (!indices || !values || !cbsr_data || !cbsr_sel) return MAXK_E_ARG;
    if (!workspace || workspace_bytes < maxk_forward_workspace_bytes(num_panels, dim_origin))
        return MAXK_E_WORKSPACE;
    const size_t dimp = (size_t)((dim_origin + 3) & ~3);
    float *carry = static_cast<float *>(workspace);
    int32_t *carry_row = reinterpret_cast<int32_t *>(
        static_cast<char *>(workspace) + align_up((size_t)num_panels * dimp * sizeof(float), 256));
    return dispatch_k<FwdPanel>(dim_k, sched, num_panels, indptr, indices, values, cbsr_data,
                                cbsr_sel, num_rows, dim_origin, dim_k, out, carry, carry_row,
                                fwd_owner_slots(workspace, num_panels, dim_origin), false,
                                as_stream(stream), (uint8_t *)nullptr,
                                (flags & MAXK_FWD_CACHED_GATHER) != 0,
                                num_parts > 0 ? parts : (const float *)nullptr, num_parts);
}

int maxk_rows_sum(const float *parts, int num_parts, int64_t n, float *out, void *stream)
{
    if (num_parts < 1 || n < 0 || (n > 0 && (!parts || !out))) return MAXK_E_ARG;
    if (n == 0) return MAXK_OK;
    hipStream_t st = as_stream(stream);
    const bool vec = (n % 4) == 0 && ((uintptr_t)parts % 16) == 0 && ((uintptr_t)out % 16) == 0;
    const int64_t items = vec ? n / 4 : n;
    int64_t blocks = ceil_div(items, kBlock);
    blocks = blocks < 65536 ? blocks : 65536;
    if (vec)
        hipLaunchKernelGGL(rows_sum_kernel<true>, dim3((unsigned)blocks), dim3(kBlock), 0, st, parts,
                           num_parts, n, out);
    else
        hipLaunchKernelGGL(rows_sum_kernel<false>, dim3((unsigned)blocks), dim3(kBlock), 0, st,
                           parts, num_parts, n, out);
    return launch_status();
}

int maxk_spmm_gnna_sag(const int32_t *warp4, int64_t num_parts, const int32_t *indices,
                       const float *values, const float *x, int dim, float *out, void *stream)
{
    if (num_parts < 0 || (num_parts > 0 && (!warp4 || !indices || !x || !out))) return MAXK_E_ARG;
    if (dim < 4 || dim > kMaxDim || (dim & 3)) return MAXK_E_DIM;
    if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(warp4)) & 15) return MAXK_E_ARG;
    if (num_parts == 0) return MAXK_OK;
    const int64_t blocks = ceil_div(num_parts, kWavesPerBlock);
    hipLaunchKernelGGL(gnna_sag_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, as_stream(stream),
                       reinterpret_cast<const int4 *>(warp4), num_parts, indices, values, x, dim,
                       out);
    return launch_status();
}

int maxk_spmm_dense_forward(const int32_t *sched, int64_t num_panels, const int32_t *indptr,
                            const int32_t *indices, const float *values, const float *x,
                            int num_rows, int dim, float *out, void *workspace,
                            size_t workspace_bytes, void *stream)
{
    if (!sched || !indptr || !out || num_panels < 1 || num_rows < 0) return MAXK_E_ARG;
    if (dim < 4 || dim > kMaxDim || (dim & 3)) return MAXK_E_DIM;
    if (num_rows == 0) return MAXK_OK;
    if (!indices || !values || !x) return MAXK_E_ARG;
    if (!workspace || workspace_bytes < maxk_forward_workspace_bytes(num_panels, dim))
        return MAXK_E_WORKSPACE;
    float *carry = static_cast<float *>(workspace);
    int32_t *carry_row = reinterpret_cast<int32_t *>(
        static_cast<char *>(workspace) + align_up((size_t)num_panels * dim * sizeof(float), 256));
    hipStream_t st = as_stream(stream);
    const int64_t blocks = ceil_div(num_panels, kWavesPerBlock);
    const int2 *sc = reinterpret_cast<const int2 *>(sched);
    const int q = dim / 4;  // lanes per edge: the smallest power of two >= dim / 4
    auto k = q > 32 ? dense_panel_kernel<64> : q > 16 ? dense_panel_kernel<32>
           : q > 8 ? dense_panel_kernel<16> : q > 4 ? dense_panel_kernel<8>
           : q > 2 ? dense_panel_kernel<4> : q > 1 ? dense_panel_kernel<2> : dense_panel_kernel<1>;
    hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(kBlock), 0, st, sc, num_panels, indptr,
                       indices, values, x, num_rows, dim, out, carry, carry_row);
    int rc = launch_status();
    if (rc) return rc;
    hipLaunchKernelGGL(carry_fixup_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, st, num_panels,
                       carry, carry_row, out, dim, dim, 1, (size_t)0);
    return launch_status();
}

size_t maxk_cbsr_packed_row_bytes(int dim_k)
{
    return dim_k == 4 ? 32 : (dim_k == 8 ? 64 : (dim_k == 16 ? 128 : 0));
}

int maxk_cbsr_pack(const float *cbsr_data, const uint8_t *cbsr_sel, int num_cols, int dim_k,
                   void *packed, void *stream)
{
    if (maxk_cbsr_packed_row_bytes(dim_k) == 0) return MAXK_E_DIM;
    if (num_cols < 0 || (num_cols > 0 && (!cbsr_data || !cbsr_sel || !packed))) return MAXK_E_ARG;
    if (num_cols == 0) return MAXK_OK;
    uint8_t *rec = static_cast<uint8_t *>(packed);
    hipStream_t st = as_stream(stream);
    switch (dim_k) {
    case 4: return CbsrPack<4>::run(cbsr_data, cbsr_sel, num_cols, rec, st);
    case 8: return CbsrPack<8>::run(cbsr_data, cbsr_sel, num_cols, rec, st);
    default: return CbsrPack<16>::run(cbsr_data, cbsr_sel, num_cols, rec, st);
    }
}

int maxk_spgemm_forward_packed(const int32_t *sched, int64_t num_panels, const int32_t *indptr,
                               const int32_t *indices, const float *values, const void *packed,
                               int num_rows, int dim_origin, int dim_k, float *out,
                               void *workspace, size_t workspace_bytes, void *stream)
{
    if (!sched || !indptr || !out || num_panels < 1 || num_rows < 0) return MAXK_E_ARG;
    if (!dims_ok(dim_origin, dim_k) || maxk_cbsr_packed_row_bytes(dim_k) == 0) return MAXK_E_DIM;
    if (num_rows == 0) return MAXK_OK;
    if (!indices || !values || !packed) return MAXK_E_ARG;
    if (!workspace || workspace_bytes < maxk_forward_workspace_bytes(num_panels, dim_origin))
        return MAXK_E_WORKSPACE;
    const size_t dimp = (size_t)((dim_origin + 3) & ~3);
    float *carry = static_cast<float *>(workspace);
    int32_t *carry_row = reinterpret_cast<int32_t *>(
        static_cast<char *>(workspace) + align_up((size_t)num_panels * dimp * sizeof(float), 256));
    const uint8_t *rec = static_cast<const uint8_t *>(packed);
    float *owner = fwd_owner_slots(workspace, num_panels, dim_origin);
    hipStream_t st = as_stream(stream);
    switch (dim_k) {
    case 4: return FwdPanelPacked<4>::run(sched, num_panels, indptr, indices, values, rec, num_rows, dim_origin, dim_k, out, carry, carry_row, owner, st);
    case 8: return FwdPanelPacked<8>::run(sched, num_panels, indptr, indices, values, rec, num_rows, dim_origin, dim_k, out, carry, carry_row, owner, st);
    default: return FwdPanelPacked<16>::run(sched, num_panels, indptr, indices, values, rec, num_rows, dim_origin, dim_k, out, carry, carry_row, owner, st);
    }
}

int maxk_spgemm_forward_esel(const int32_t *sched, int64_t num_panels, const int32_t *indptr,
                             const int32_t *indices, const float *values, const float *cbsr_data,
                             const uint8_t *cbsr_sel, const void *packed, int num_rows,
                             int dim_origin, int dim_k, float *out, uint8_t *edge_sel,
                             void *workspace, size_t workspace_bytes, void *stream)
{
    if (!sched || !indptr || !out || !edge_sel || num_panels < 1 || num_rows < 0) return MAXK_E_ARG;
    if (!dims_ok(dim_origin, dim_k)) return MAXK_E_DIM;
    if (packed && maxk_cbsr_packed_row_bytes(dim_k) == 0) return MAXK_E_DIM;
    if (num_rows == 0) return MAXK_OK;
    if (!indices || !values || (!packed && (!cbsr_data || !cbsr_sel))) return MAXK_E_ARG;
    if (!workspace || workspace_bytes < maxk_forward_workspace_bytes(num_panels, dim_origin))
        return MAXK_E_WORKSPACE;
    const size_t dimp = (size_t)((dim_origin + 3) & ~3);
    float *carry = static_cast<float *>(workspace);
    int32_t *carry_row = reinterpret_cast<int32_t *>(
        static_cast<char *>(workspace) + align_up((size_t)num_panels * dimp * sizeof(float), 256));
    float *owner = fwd_owner_slots(workspace, num_panels, dim_origin);
    hipStream_t st = as_stream(stream);
    if (packed) {
        const uint8_t *rec = static_cast<const uint8_t *>(packed);
        switch (dim_k) {
        case 4: return FwdPanelPacked<4>::run(sched, num_panels, indptr, indices, values, rec, num_rows, dim_origin, dim_k, out, carry, carry_row, owner, st, edge_sel);
        case 8: return FwdPanelPacked<8>::run(sched, num_panels, indptr, indices, values, rec, num_rows, dim_origin, dim_k, out, carry, carry_row, owner, st, edge_sel);
        default: return FwdPanelPacked<16>::run(sched, num_panels, indptr, indices, values, rec, num_rows, dim_origin, dim_k, out, carry, carry_row, owner, st, edge_sel);
        }
    }
    return dispatch_k<FwdPanel>(dim_k, sched, num_panels, indptr, indices, values, cbsr_data,
                                cbsr_sel, num_rows, dim_origin, dim_k, out, carry, carry_row, owner,
                                false, st, edge_sel);
}

int maxk_records_sel_gather(const uint8_t *records, int dim_k, const int32_t *rows, int64_t n,
                            uint8_t *out_sel, void *stream)
{
    if (n < 0 || (n > 0 && (!records || !rows || !out_sel))) return MAXK_E_ARG;
    if (dim_k < 4 || dim_k > 256 || (dim_k & (dim_k - 1))) return MAXK_E_DIM;
    if (n == 0) return MAXK_OK;
    hipStream_t st = as_stream(stream);
    const int64_t pieces = n * (dim_k % 16 == 0 ? dim_k / 16 : dim_k / 4);
    const dim3 g((unsigned)ceil_div(pieces, kBlock));
    switch (dim_k) {
    case 4: hipLaunchKernelGGL(records_sel_kernel<4>, g, dim3(kBlock), 0, st, records, rows, n, out_sel); break;
    case 8: hipLaunchKernelGGL(records_sel_kernel<8>, g, dim3(kBlock), 0, st, records, rows, n, out_sel); break;
    case 16: hipLaunchKernelGGL(records_sel_kernel<16>, g, dim3(kBlock), 0, st, records, rows, n, out_sel); break;
    case 32: hipLaunchKernelGGL(records_sel_kernel<32>, g, dim3(kBlock), 0, st, records, rows, n, out_sel); break;
    case 64: hipLaunchKernelGGL(records_sel_kernel<64>, g, dim3(kBlock), 0, st, records, rows, n, out_sel); break;
    case 128: hipLaunchKernelGGL(records_sel_kernel<128>, g, dim3(kBlock), 0, st, records, rows, n, out_sel); break;
    default: hipLaunchKernelGGL(records_sel_kernel<256>, g, dim3(kBlock), 0, st, records, rows, n, out_sel); break;
    }
    return launch_status();
}

int maxk_cbsr_gather_records(const float *cbsr_data, const uint8_t *cbsr_sel, const int32_t *rows,
                             int64_t num_records, int dim_k, void *records, void *stream)
{
    if (dim_k < 4 || dim_k > kMaxDim || (dim_k & (dim_k - 1))) return MAXK_E_DIM;
    if (num_records < 0 || (num_records > 0 && (!cbsr_data || !cbsr_sel || !records)))
        return MAXK_E_ARG;
    if (num_records == 0) return MAXK_OK;
    return dispatch_k<CbsrRecords>(dim_k, cbsr_data, cbsr_sel, rows, num_records,
                                   static_cast<uint8_t *>(records), as_stream(stream));
}

int maxk_spgemm_forward_records(const int32_t *sched, int64_t num_panels, const int32_t *indptr,
                                const int32_t *indices, const float *values, const void *records,
                                int num_rows, int dim_origin, int dim_k, int flags, float *out,
                                void *workspace, size_t workspace_bytes, void *stream)
{
    if (!sched || !indptr || !out || num_panels < 1 || num_rows < 0) return MAXK_E_ARG;
    if (flags & ~MAXK_FWD_ACCUMULATE) return MAXK_E_ARG;
    if (!dims_ok(dim_origin, dim_k) || dim_k < 4 || (dim_k & (dim_k - 1))) return MAXK_E_DIM;
    if (num_rows == 0) return MAXK_OK;
    if (!indices || !values || !records) return MAXK_E_ARG;
    if (reinterpret_cast<uintptr_t>(records) & 15) return MAXK_E_ARG;
    if (!workspace || workspace_bytes < maxk_forward_workspace_bytes(num_panels, dim_origin))
        return MAXK_E_WORKSPACE;
    const size_t dimp = (size_t)((dim_origin + 3) & ~3);
    float *carry = static_cast<float *>(workspace);
    int32_t *carry_row = reinterpret_cast<int32_t *>(
        static_cast<char *>(workspace) + align_up((size_t)num_panels * dimp * sizeof(float), 256));
    return dispatch_k<FwdRecords>(dim_k, sched, num_panels, indptr, indices, values,
                                  static_cast<const uint8_t *>(records), num_rows, dim_origin,
                                  dim_k, (flags & MAXK_FWD_ACCUMULATE) != 0, out, carry, carry_row,
                                  fwd_owner_slots(workspace, num_panels, dim_origin),
                                  as_stream(stream));
}

// out_packed (uint16 selector | original entry << 8) serves the ablation
// library's bank-ordered backward (tools/variants_lib)
static int cbsr_bank_order_impl(const float *cbsr_data, const uint8_t *cbsr_sel, int num_rows,
                                int dim_k, int num_rel, float *out_data, uint8_t *out_sel,
                                uint16_t *out_packed, void *stream)
{
    if (dim_k < 1 || dim_k > kWave) return MAXK_E_DIM;
    if (num_rel < 1 || num_rel > 16) return MAXK_E_ARG;
    if (num_rows > 0 && !cbsr_sel) return MAXK_E_ARG;
    if (num_rows > 0 && out_data && !cbsr_data) return MAXK_E_ARG;
    if (num_rows > 0 && !out_data && !out_sel && !out_packed) return MAXK_E_ARG;
    // the store classes follow the record layout maxk_spgemm_forward_multi uses for num_rel
    const int swz = (FWD_REL8_SWZ && num_rel == 8) ? ((FWD_REL8_ILV && dim_k == 32) ? 2 : 1) : 0;
    if (num_rows < 0) return MAXK_E_ARG;
    if (num_rows == 0) return MAXK_OK;
    const int64_t blocks = ceil_div(num_rows, kWavesPerBlock);
    hipLaunchKernelGGL(cbsr_bank_order_kernel, dim3((unsigned)(blocks < 4096 ? blocks : 4096)),
                       dim3(kBlock), 0, as_stream(stream), cbsr_data, cbsr_sel, num_rows, dim_k,
                       swz, out_data, out_sel, out_packed);
    return launch_status();
}

int maxk_cbsr_bank_order(const float *cbsr_data, const uint8_t *cbsr_sel, int num_rows,
                         int dim_k, int num_rel, float *out_data, uint8_t *out_sel, void *stream)
{
    return cbsr_bank_order_impl(cbsr_data, cbsr_sel, num_rows, dim_k, num_rel, out_data, out_sel,
                                nullptr, stream);
}

size_t maxk_forward_multi_workspace_bytes(int64_t num_panels, int dim_origin, int num_rel)
{
    const size_t dimp = (size_t)((dim_origin + 3) & ~3);
    return align_up((size_t)num_panels * num_rel * dimp * sizeof(float), 256) +
           align_up((size_t)num_panels * sizeof(int32_t), 256);
}

int maxk_spgemm_forward_multi(const int32_t *sched, int64_t num_panels, const int32_t *indptr,
                              const int32_t *indices, const float *values, int num_rel,
                              const float *cbsr_data, const uint8_t *cbsr_sel, int num_rows,
                              int dim_origin, int dim_k, float *out, void *workspace,
                              size_t workspace_bytes, void *stream)
{
    if (!sched || !indptr || !out || num_panels < 1 || num_rows < 0) return MAXK_E_ARG;
    if (num_rel < 1 || num_rel > kMaxRel) return MAXK_E_ARG;
    if (!dims_ok(dim_origin, dim_k)) return MAXK_E_DIM;
    if (num_rows == 0) return MAXK_OK;
    if (!indices || !values || !cbsr_data || !cbsr_sel) return MAXK_E_ARG;
    if (!workspace ||
        workspace_bytes < maxk_forward_multi_workspace_bytes(num_panels, dim_origin, num_rel))
        return MAXK_E_WORKSPACE;
    const size_t dimp = (size_t)((dim_origin + 3) & ~3);
    float *carry = static_cast<float *>(workspace);
    int32_t *carry_row = reinterpret_cast<int32_t *>(
        static_cast<char *>(workspace) +
        align_up((size_t)num_panels * num_rel * dimp * sizeof(float), 256));
    return dispatch_k<FwdMulti>(dim_k, sched, num_panels, indptr, indices, values, num_rel,
                                cbsr_data, cbsr_sel, num_rows, dim_origin, out, carry, carry_row,
                                as_stream(stream));
}

size_t maxk_backward_workspace_bytes(int algo, int64_t num_edges, int dim_k,
                                     int64_t csc_num_panels)
{
    if (algo == MAXK_BWD_ATOMIC) return 0;  // STAGED_EDGE: as STAGED
    // P rows padded to 64 B at k = 8 (PRow) when scattered; EDGE_GATHER writes them in order
    const int kp = dim_k == 8 && algo != MAXK_BWD_EDGE_GATHER ? 16 : dim_k;
    return align_up((size_t)num_edges * kp * sizeof(float), 256) +
           align_up((size_t)csc_num_panels * dim_k * sizeof(float), 256) +
           align_up((size_t)csc_num_panels * sizeof(int32_t), 256);
}

int maxk_sspmm_backward(int algo, const int32_t *sched, int64_t num_panels,
                        const int32_t *indptr, const int32_t *indices, const float *values,
                        const float *grad, const uint8_t *cbsr_sel, int num_rows,
                        int num_cols, int64_t num_edges, int dim_origin, int dim_k, float *dxs,
                        const int32_t *csc_pos, const int32_t *csc_sched,
                        int64_t csc_num_panels, const int32_t *csc_indptr, void *workspace,
                        size_t workspace_bytes, void *stream)
{
    if (!sched || !indptr || !dxs || num_panels < 1 || num_rows < 0 || num_cols < 0 ||
        num_edges < 0)
        return MAXK_E_ARG;
    if (!dims_ok(dim_origin, dim_k)) return MAXK_E_DIM;
    hipStream_t st = as_stream(stream);
    if (num_cols == 0) return MAXK_OK;
    if (num_rows == 0 || num_edges == 0)  // no edge: dXs = 0
        return zero_floats(dxs, (size_t)num_cols * dim_k, st);
    if (!indices || !values || !grad || !cbsr_sel) return MAXK_E_ARG;
    const bool staged_ready = csc_pos && csc_sched && csc_indptr && csc_num_panels >= 1 &&
                              workspace;
    if (algo == MAXK_BWD_AUTO) algo = staged_ready ? MAXK_BWD_STAGED : MAXK_BWD_ATOMIC;
    // STAGED_EDGE / EDGE_GATHER: cbsr_sel = edge selectors uint8[E, k];
    // EDGE_GATHER: csc_pos = the CSC slot -> CSR edge permutation (maxk_csc_perm_build)
    const bool gather = algo == MAXK_BWD_EDGE_GATHER;
    const bool esel = algo == MAXK_BWD_STAGED_EDGE || gather;
    const int ws_algo = algo;
    if (esel) algo = MAXK_BWD_STAGED;
    if (algo == MAXK_BWD_ATOMIC) {
        const int e = zero_floats(dxs, (size_t)num_cols * dim_k, st);
        if (e) return e;
        return dispatch_k<BwdPanel>(dim_k, false, sched, num_panels, indptr, indices, values, grad,
                                    cbsr_sel, (const int32_t *)nullptr, num_rows, dim_origin, dim_k,
                                    dxs, (float *)nullptr, st);
    }
    if (algo != MAXK_BWD_STAGED || !staged_ready) return MAXK_E_ARG;
    // workspace: [P rows (E*kp floats)] [carry (CP*k floats)] [carry_row (CP ints)]
    if (workspace_bytes < maxk_backward_workspace_bytes(ws_algo, num_edges, dim_k, csc_num_panels))
        return MAXK_E_WORKSPACE;
    const int kp = dim_k == 8 && !gather ? 16 : dim_k;
    const size_t pbytes = align_up((size_t)num_edges * kp * sizeof(float), 256);
    const size_t carry_bytes = align_up((size_t)csc_num_panels * dim_k * sizeof(float), 256);
    float *Pbuf = static_cast<float *>(workspace);
    float *carry = reinterpret_cast<float *>(static_cast<char *>(workspace) + pbytes);
    int32_t *carry_row = reinterpret_cast<int32_t *>(static_cast<char *>(workspace) + pbytes +
                                                     carry_bytes);
    int rc = dispatch_k<BwdPanel>(dim_k, true, sched, num_panels, indptr, indices, values, grad,
                                  cbsr_sel, csc_pos, num_rows, dim_origin, dim_k, dxs, Pbuf, st,
                                  esel, gather ? kPmEdge : kPmCsc);
    if (rc) return rc;
    return dispatch_k<BwdSegsum>(dim_k, csc_sched, csc_num_panels, csc_indptr, Pbuf, num_cols,
                                 dim_k, dxs, carry, carry_row, st,
                                 gather ? csc_pos : (const int32_t *)nullptr);
}

// Validation, workspace carve-up and phase 2 (the CSC segmented sum) of the
// multi-relation STAGED backward; phase1(edge_order, Pbuf, stream) launches
// phase 1 (here the LDS form; the ablation library, tools/variants_lib, runs
// its register and bank-ordered forms through the same function).
extern "C++" {
template <typename Phase1>
static int sspmm_backward_multi_impl(int algo, int64_t num_panels, const int32_t *sched,
                                     const int32_t *indptr, const int32_t *indices,
                                     const float *values, int num_rel, const float *grad,
                                     const void *cbsr_sel, int num_rows, int num_cols,
                                     int64_t num_edges, int dim_origin, int dim_k, float *dxs,
                                     const int32_t *csc_pos, const int32_t *csc_sched,
                                     int64_t csc_num_panels, const int32_t *csc_indptr,
                                     void *workspace, size_t workspace_bytes, void *stream,
                                     Phase1 phase1)
{
    if (!sched || !indptr || !dxs || num_panels < 1 || num_rows < 0 || num_cols < 0 ||
        num_edges < 0)
        return MAXK_E_ARG;
    if (num_rel != 4 && num_rel != 8 && num_rel != 16) return MAXK_E_ARG;
    if (!dims_ok(dim_origin, dim_k) || (dim_origin & 3) ||
        (dim_k != 8 && dim_k != 16 && dim_k != 32 && dim_k != 64))
        return MAXK_E_DIM;
    if (algo == MAXK_BWD_AUTO) algo = MAXK_BWD_STAGED;
    if (algo != MAXK_BWD_STAGED && algo != MAXK_BWD_EDGE_GATHER) return MAXK_E_ARG;
    hipStream_t st = as_stream(stream);
    if (num_cols == 0) return MAXK_OK;
    if (num_rows == 0 || num_edges == 0) return zero_floats(dxs, (size_t)num_cols * dim_k, st);
    if (!indices || !values || !grad || !cbsr_sel || !csc_pos || !csc_sched || !csc_indptr ||
        csc_num_panels < 1 || !workspace)
        return MAXK_E_ARG;
    if ((reinterpret_cast<uintptr_t>(values) | reinterpret_cast<uintptr_t>(grad)) & 15)
        return MAXK_E_ARG;
    const bool gather = algo == MAXK_BWD_EDGE_GATHER;
    if (workspace_bytes < maxk_backward_workspace_bytes(algo, num_edges, dim_k, csc_num_panels))
        return MAXK_E_WORKSPACE;
    const int kp = dim_k == 8 && !gather ? 16 : dim_k;
    const size_t pbytes = align_up((size_t)num_edges * kp * sizeof(float), 256);
    const size_t carry_bytes = align_up((size_t)csc_num_panels * dim_k * sizeof(float), 256);
    float *Pbuf = static_cast<float *>(workspace);
    float *carry = reinterpret_cast<float *>(static_cast<char *>(workspace) + pbytes);
    int32_t *carry_row = reinterpret_cast<int32_t *>(static_cast<char *>(workspace) + pbytes +
                                                     carry_bytes);
    int rc = phase1(gather, Pbuf, st);
    if (rc) return rc;
    return dispatch_k<BwdSegsum>(dim_k, csc_sched, csc_num_panels, csc_indptr, Pbuf, num_cols,
                                 dim_k, dxs, carry, carry_row, st,
                                 gather ? csc_pos : (const int32_t *)nullptr);
}
}  // extern "C++"

int maxk_sspmm_backward_multi(int algo, const int32_t *sched, int64_t num_panels,
                              const int32_t *indptr, const int32_t *indices, const float *values,
                              int num_rel, const float *grad, const uint8_t *cbsr_sel,
                              int num_rows, int num_cols, int64_t num_edges, int dim_origin,
                              int dim_k, float *dxs, const int32_t *csc_pos,
                              const int32_t *csc_sched, int64_t csc_num_panels,
                              const int32_t *csc_indptr, void *workspace, size_t workspace_bytes,
                              void *stream)
{
    return sspmm_backward_multi_impl(
        algo, num_panels, sched, indptr, indices, values, num_rel, grad, cbsr_sel, num_rows,
        num_cols, num_edges, dim_origin, dim_k, dxs, csc_pos, csc_sched, csc_num_panels,
        csc_indptr, workspace, workspace_bytes, stream,
        [&](bool edge_order, float *Pbuf, hipStream_t st) {
            return dispatch_k<BwdMultiStage>(dim_k, num_rel, edge_order, sched, num_panels, indptr,
                                             indices, values, grad, (int64_t)num_rows * dim_origin,
                                             cbsr_sel, csc_pos, num_rows, dim_origin, Pbuf, st);
        });
}

int maxk_append_bins(int num_cols, int dim_k, int *num_bins, int *bin_size)
{
    if (num_cols < 0 || !num_bins || !bin_size) return MAXK_E_ARG;
    if (dim_k < 4 || dim_k > kMaxDim || (dim_k & (dim_k - 1))) return MAXK_E_DIM;
    if (num_cols == 0) {
        *num_bins = 0;
        *bin_size = 1;
        return MAXK_OK;
    }
    // the bin's rows fill at most 160 KB of LDS; beyond 256 bins, whole rounds of
    // 256 (one workgroup per CU: products k=8 -> 512 bins of 4,784); below, at
    // least ~64 destinations per bin and up to 256 bins for parallelism
    const int cap = (int)(kAppendLds / (4 * dim_k));
    int64_t nb = ceil_div((int64_t)num_cols, cap);
    const int64_t par = ceil_div((int64_t)num_cols, 64) < 256 ? ceil_div((int64_t)num_cols, 64) : 256;
    if (nb > 256) nb = ceil_div(nb, 256) * 256;
    else if (nb < par) nb = par;
    if (nb < 1) nb = 1;
    const int64_t bs = ceil_div((int64_t)num_cols, nb);
    *bin_size = (int)bs;
    *num_bins = (int)ceil_div((int64_t)num_cols, bs);
    return MAXK_OK;
}

int maxk_append_plan_build(const int32_t *sched, int64_t num_panels, const int32_t *indptr,
                           const int32_t *indices, int num_rows, int num_cols, int dim_k,
                           int32_t *region_base, int num_bins, int bin_size, void *stream)
{
    (void)indptr;
    if (!sched || !region_base || num_panels < 1 || num_rows < 0 || num_cols < 0 ||
        num_bins < 0 || bin_size < 1)
        return MAXK_E_ARG;
    int nb = 0, bs = 0;
    const int rc0 = maxk_append_bins(num_cols, dim_k, &nb, &bs);
    if (rc0) return rc0;
    if (nb != num_bins || bs != bin_size) return MAXK_E_ARG;
    hipStream_t st = as_stream(stream);
    const int ng = num_bins * kAppendGroups;
    const hipError_t me = hipMemsetAsync(region_base, 0, (size_t)(ng + 1) * sizeof(int32_t), st);
    if (me != hipSuccess) return (int)me;
    if (num_cols > 0 && num_rows > 0) {
        if (!indices) return MAXK_E_ARG;
        const AppendArgs ap{append_magic(bin_size), bin_size, nullptr, nullptr};
        hipLaunchKernelGGL(append_count_kernel, dim3((unsigned)ceil_div(num_panels, kWavesPerBlock)),
                           dim3(kBlock), 0, st, reinterpret_cast<const int2 *>(sched), num_panels,
                           indices, ap, region_base);
        const int rc = launch_status();
        if (rc) return rc;
    }
    hipLaunchKernelGGL(exclusive_scan_1block, dim3(1), dim3(256), 0, st, region_base, ng,
                       region_base + ng);
    return launch_status();
}

size_t maxk_backward_append_workspace_bytes(int64_t num_edges, int dim_k, int num_bins)
{
    return align_up((size_t)num_edges * dim_k * sizeof(float), 256) +
           align_up((size_t)num_edges * sizeof(int32_t), 256) +
           align_up((size_t)num_bins * kAppendGroups * kCursorStride * sizeof(int32_t), 256);
}

int maxk_sspmm_backward_append(const int32_t *sched, int64_t num_panels, const int32_t *indptr,
                               const int32_t *indices, const float *values, int num_rel,
                               const float *grad, const uint8_t *cbsr_sel, int edge_sel,
                               int num_rows, int num_cols, int64_t num_edges, int dim_origin,
                               int dim_k, const int32_t *region_base, int num_bins, int bin_size,
                               float *dxs, void *workspace, size_t workspace_bytes, void *stream)
{
    if (!sched || !indptr || !dxs || !region_base || num_panels < 1 || num_rows < 0 ||
        num_cols < 0 || num_edges < 0 || num_edges > INT32_MAX)
        return MAXK_E_ARG;
    if (!dims_ok(dim_origin, dim_k) || dim_k < 4 || (dim_k & (dim_k - 1))) return MAXK_E_DIM;
    if (num_rel != 1 && num_rel != 4 && num_rel != 8 && num_rel != 16) return MAXK_E_ARG;
    if (num_rel > 1 && (edge_sel || dim_k < 8 || dim_k > 64 || (dim_origin & 3)))
        return num_rel > 1 && edge_sel ? MAXK_E_ARG : MAXK_E_DIM;
    int nb = 0, bs = 0;
    const int rc0 = maxk_append_bins(num_cols, dim_k, &nb, &bs);
    if (rc0) return rc0;
    if (nb != num_bins || bs != bin_size) return MAXK_E_ARG;
    hipStream_t st = as_stream(stream);
    if (num_cols == 0) return MAXK_OK;
    if (num_rows == 0 || num_edges == 0) return zero_floats(dxs, (size_t)num_cols * dim_k, st);
    if (!indices || !values || !grad || !cbsr_sel) return MAXK_E_ARG;
    if (!workspace || workspace_bytes < maxk_backward_append_workspace_bytes(num_edges, dim_k, num_bins))
        return MAXK_E_WORKSPACE;
    char *ws = static_cast<char *>(workspace);
    float *Pbuf = reinterpret_cast<float *>(ws);
    ws += align_up((size_t)num_edges * dim_k * sizeof(float), 256);
    int32_t *dst = reinterpret_cast<int32_t *>(ws);
    ws += align_up((size_t)num_edges * sizeof(int32_t), 256);
    int32_t *cursor = reinterpret_cast<int32_t *>(ws);
    return dispatch_k<BwdAppend>(dim_k, sched, num_panels, indptr, indices, values, num_rel, grad,
                                 cbsr_sel, edge_sel != 0, num_rows, num_cols, dim_origin,
                                 region_base, num_bins, bin_size, dxs, Pbuf, dst, cursor, st);
}

size_t maxk_backward_local_lds_bytes(int dmax, int dim_k)
{
    return (size_t)kWavesPerBlock * (size_t)((dmax * dim_k * 5 + 15) & ~15);
}

int maxk_sspmm_backward_local(const int32_t *seg_edge_off, int num_segments,
                              const int32_t *wave_dst_start, int num_waves, int dmax,
                              const int32_t *edge_rc, const float *edge_val, const float *grad,
                              const uint8_t *cbsr_sel, int num_rows, int dim_origin, int dim_k,
                              float *dxs, void *stream)
{
    if (!seg_edge_off || !wave_dst_start || !dxs || num_waves < 1 || num_segments < 1 ||
        num_rows < 1 || num_rows >= (1 << 24) || dmax < 1 || dmax > 256)
        return MAXK_E_ARG;
    if (!dims_ok(dim_origin, dim_k) || (kWave % dim_k) != 0) return MAXK_E_DIM;
    if (!edge_rc || !edge_val || !grad || !cbsr_sel) return MAXK_E_ARG;
    if (maxk_backward_local_lds_bytes(dmax, dim_k) > 160 * 1024) return MAXK_E_WORKSPACE;
    hipStream_t st = as_stream(stream);
#define LOCAL_ARGS seg_edge_off, num_segments, wave_dst_start, num_waves, dmax, edge_rc, edge_val, \
                   grad, cbsr_sel, num_rows, dim_origin, dxs, st
    switch (dim_k) {
    case 1: return BwdLocal<1>::run(LOCAL_ARGS);
    case 2: return BwdLocal<2>::run(LOCAL_ARGS);
    case 4: return BwdLocal<4>::run(LOCAL_ARGS);
    case 8: return BwdLocal<8>::run(LOCAL_ARGS);
    case 16: return BwdLocal<16>::run(LOCAL_ARGS);
    case 32: return BwdLocal<32>::run(LOCAL_ARGS);
    default: return BwdLocal<64>::run(LOCAL_ARGS);
    }
#undef LOCAL_ARGS
}

int maxk_grad_interleave(const float *grad, int num_rel, int num_rows, int dim, float *out,
                         void *stream)
{
    if (num_rel < 1 || num_rel > 16 || num_rows < 0 || dim < 1) return MAXK_E_ARG;
    if (num_rows == 0) return MAXK_OK;
    if (!grad || !out) return MAXK_E_ARG;
    const int64_t n = (int64_t)num_rows * dim;
    const int64_t blocks = ceil_div(n, kBlock);
    hipLaunchKernelGGL(grad_interleave_kernel, dim3((unsigned)(blocks < 8192 ? blocks : 8192)),
                       dim3(kBlock), 0, as_stream(stream), grad, num_rel, n, n, out);
    return launch_status();
}

int maxk_sspmm_backward_local_rel8(const int32_t *seg_edge_off, int num_segments,
                                   const int32_t *wave_dst_start, int num_waves, int dmax,
                                   const int32_t *edge_rc, const float *edge_val,
                                   const float *grad_interleaved, const uint8_t *cbsr_sel,
                                   int num_rows, int dim_origin, int dim_k, float *dxs,
                                   void *stream)
{
    if (!seg_edge_off || !wave_dst_start || !dxs || num_waves < 1 || num_segments < 1 ||
        num_rows < 1 || num_rows >= (1 << 24) || dmax < 1 || dmax > 256)
        return MAXK_E_ARG;
    if (dim_k != 32 || !dims_ok(dim_origin, dim_k)) return MAXK_E_DIM;
    if (!edge_rc || !edge_val || !grad_interleaved || !cbsr_sel) return MAXK_E_ARG;
    if ((reinterpret_cast<uintptr_t>(edge_val) | reinterpret_cast<uintptr_t>(grad_interleaved)) & 15)
        return MAXK_E_ARG;
    if (maxk_backward_local_lds_bytes(dmax, dim_k) > 160 * 1024) return MAXK_E_WORKSPACE;
    hipStream_t st = as_stream(stream);
    const size_t region = (size_t)((dmax * 32 * 5 + 15) & ~15);
    for (int s = 0; s < num_segments; ++s) {
        hipLaunchKernelGGL(bwd_local_rel8_kernel, dim3((unsigned)ceil_div(num_waves, kWavesPerBlock)),
                           dim3(kBlock), region * kWavesPerBlock, st,
                           seg_edge_off + (size_t)s * num_waves,
                           seg_edge_off + (size_t)(s + 1) * num_waves, s == 0, wave_dst_start,
                           num_waves, dmax, edge_rc, edge_val, grad_interleaved, cbsr_sel,
                           dim_origin, dxs);
        const int rc = launch_status();
        if (rc) return rc;
    }
    return MAXK_OK;
}

int maxk_sspmm_backward_tile(const void *headers, const int64_t *header_start,
                             const void *records, const int64_t *record_start,
                             const int32_t *num_chunks, int num_groups, int num_workgroups,
                             int group_size, const float *grad, const float *zero_row,
                             const uint8_t *cbsr_sel, int num_rows, int num_cols, int dim_origin,
                             int dim_k, float *dxs, float *part, void *stream)
{
    if ((dim_k != 32 && dim_k != 64) || dim_origin != kMaxDim) return MAXK_E_DIM;
    if (!headers || !header_start || !records || !record_start || !num_chunks || !grad ||
        !zero_row || !cbsr_sel || !dxs || num_groups < 1 || num_workgroups < 1 ||
        num_workgroups > (1 << 20) || group_size < 1 ||
        group_size > (dim_k == 32 ? 128 : 64) * kTileWaves || num_rows < 1 || num_cols < 1 ||
        (int64_t)num_groups * group_size < num_cols ||
        // an empty workgroup range would leave a partial plane unwritten that
        // tile_combine_kernel still adds
        (int64_t)num_workgroups > (int64_t)num_groups * num_rows)
        return MAXK_E_ARG;
    const int planes = maxk_tile_part_planes(num_rows, num_groups, num_workgroups);
    if (planes > 0 && !part) return MAXK_E_ARG;
    if ((reinterpret_cast<uintptr_t>(headers) | reinterpret_cast<uintptr_t>(records) |
         reinterpret_cast<uintptr_t>(grad) | reinterpret_cast<uintptr_t>(zero_row) |
         reinterpret_cast<uintptr_t>(dxs) | reinterpret_cast<uintptr_t>(part) |
         reinterpret_cast<uintptr_t>(cbsr_sel)) & 15)
        return MAXK_E_ARG;
    hipStream_t st = as_stream(stream);
    // buffer DMA while the gradient's bytes and a zero-row offset fit the 32-bit
    // range check (V <= 4 M rows); MAXK_TILE_GDMA=1 keeps the global-address form
    static const bool gdma = [] {
        const char *v = getenv("MAXK_TILE_GDMA");
        return v && v[0] == '1';
    }();
    const bool bdma = !gdma && (int64_t)num_rows * 1024 <= (int64_t)0xFFFFFC00u - 1024;
    auto kern = dim_k == 32 ? (bdma ? bwd_tile_kernel<32, true> : bwd_tile_kernel<32, false>)
                            : (bdma ? bwd_tile_kernel<64, true> : bwd_tile_kernel<64, false>);
    const TileArgs args = {reinterpret_cast<const tile_hdr_t *>(headers), header_start,
                           reinterpret_cast<const uint32_t *>(records), record_start, num_chunks,
                           grad, zero_row, cbsr_sel, dxs, part, num_cols, group_size, num_groups,
                           num_workgroups, num_rows};
    hipLaunchKernelGGL(kern, dim3((unsigned)num_workgroups), dim3(kTileWaves * kWave), 0, st, args);
    int rc = launch_status();
    if (rc || planes == 0) return rc;
    const int64_t n4 = (int64_t)num_cols * dim_k / 4;
    const int64_t blocks = ceil_div(n4, kBlock);
    hipLaunchKernelGGL(tile_combine_kernel, dim3((unsigned)(blocks < 4096 ? blocks : 4096)),
                       dim3(kBlock), 0, st, dxs, part, n4, dim_k, group_size, num_rows, num_groups,
                       num_workgroups);
    return launch_status();
}

int maxk_segment_rows_add(const float *src, int width, const int64_t *order,
                          const int64_t *seg_off, const int64_t *seg_row, int64_t num_segments,
                          float *dst, void *stream)
{
    if (width < 1 || num_segments < 0) return MAXK_E_ARG;
    if (num_segments == 0) return MAXK_OK;
    if (!src || !order || !seg_off || !seg_row || !dst) return MAXK_E_ARG;
    const int64_t spw = width <= kWave ? kWave / width : 1;
    hipLaunchKernelGGL(segment_rows_add_kernel,
                       dim3((unsigned)ceil_div(ceil_div(num_segments, spw), kWavesPerBlock)),
                       dim3(kBlock), 0, as_stream(stream), src, width, order, seg_off, seg_row,
                       num_segments, dst);
    return launch_status();
}

int maxk_spmm_forward_warp4(const int32_t *warp4, const int32_t *idx, const float *val,
                            const float *vin_data, const uint8_t *vin_selector, float *vout,
                            int num_v, int num_e, int feat_in, int dim_sparse, int num_warps,
                            void *stream)
{
    (void)num_e;
    if (num_warps < 0 || num_v < 0) return MAXK_E_ARG;
    if (!dims_ok(feat_in, dim_sparse)) return MAXK_E_DIM;
    if (num_warps == 0) return MAXK_OK;
    if (!warp4 || !idx || !val || !vin_data || !vin_selector || !vout) return MAXK_E_ARG;
    return dispatch_k<FwdWarp4>(dim_sparse, warp4, num_warps, idx, val, vin_data, vin_selector,
                                feat_in, dim_sparse, vout, as_stream(stream));
}

int maxk_spmm_backward_warp4(const int32_t *warp4, const int32_t *idx, const float *val,
                             const float *vin_data, const uint8_t *vin_selector, float *vout,
                             int num_v, int num_e, int feat_in, int dim_sparse, int num_warps,
                             void *stream)
{
    (void)num_e;
    if (num_warps < 0 || num_v < 0) return MAXK_E_ARG;
    if (!dims_ok(feat_in, dim_sparse)) return MAXK_E_DIM;
    if (num_warps == 0) return MAXK_OK;
    if (!warp4 || !idx || !val || !vin_data || !vin_selector || !vout) return MAXK_E_ARG;
    const int run = 16;
    const int64_t waves = ceil_div(num_warps, run);
    hipLaunchKernelGGL(bwd_warp4_kernel, dim3((unsigned)ceil_div(waves, kWavesPerBlock)),
                       dim3(kBlock), row_lds_bytes(), as_stream(stream),
                       reinterpret_cast<const int4 *>(warp4), num_warps, run, idx, val, vin_data,
                       vin_selector, feat_in, dim_sparse, vout);
    return launch_status();
}

}  // extern "C"
