// maxk_topk.hip -- MI355X (gfx950) CBSR producer and dense-gradient scatter.
//
// The MaxK nonlinearity keeps the k largest entries of each feature row
// (reference: utils/models.py:28-59 MaxK, and the CBSR producers
// direct_kernel_interface.py:58-85 / kernels/spmm_bindings.cpp:163-184, all
// torch.topk(X, k, dim=1)).  The SpGEMM consumes them as CBSR: data[r, j] =
// X[r, sel[r, j]], sel uint8.  SpGEMMFunction's backward scatters the
// k-column gradient back to a dense row (utils/models.py:136-141).
//
// topk_kernel: one wave64 per row (dim <= 256: each lane holds 4 entries,
// loaded as one float4 when the row allows).  Entries map to order-preserving
// u32 keys (NaN = the largest key, as torch.topk treats NaN; -0 == +0).  The
// k-th largest key T comes from a counting search: per step, four v_cmp
// produce lane masks and s_bcnt1 counts them (no LDS, no sort); the search
// gallops from the previous row's threshold and bisects with an early stop.
// Selected = key > T, plus the lowest-column entries with key == T until k
// are taken (ties go to the lower column).  Output order:
//   column order: ascending column (prefix counts with v_mbcnt);
//   value order:  descending value, ties by lower column -- torch.topk's
//                 sorted order -- by ranking each selected entry against the
//                 row's k selected (key, column) pairs staged in LDS.
// An optional dense output receives the MaxK forward (selected entries kept,
// the rest 0), utils/models.py:44-50.
//
// scatter_kernel: out[r, :] = 0 except out[r, sel[r, j]] = vals[r, j] (or
// src[r, sel[r, j]] for the masked copy) -- the row is assembled in LDS and
// leaves as one coalesced store per lane.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/maxk_spgemm.h"

namespace {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;
constexpr int kMaxDim = 256;
// first gallop step of the threshold search (key units): 2^18 takes ~25 % fewer
// steps than 2^12 on uniform, normal and ReLU rows (k = 8..64; a CPU
// simulation of this search over 3000 rows)
#ifndef TOPK_GALLOP
#define TOPK_GALLOP 18
#endif

__device__ __forceinline__ void wave_sync_lds()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t float_key(float x)
{
    if (x != x) return 0xffffffffu;      // NaN: largest
    if (x == 0.f) x = 0.f;               // -0 -> +0
    const uint32_t u = __builtin_bit_cast(uint32_t, x);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ int popc64(uint64_t m) { return __builtin_popcountll(m); }

// lanes below this one whose bit is set in m
__device__ __forceinline__ int prefix_count(uint64_t m)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
}

// Lane order (ORDER 2): the column-order rank q is stored at position
// VEC * (q % LPE) + q / LPE, the forward's lane layout (VEC entries per lane,
// LPE = k / VEC lanes per edge): the LPE lanes of one forward wave-step then
// hold consecutive ranks, i.e. columns about 256/k apart, which fall in
// different LDS banks.  Any order is valid CBSR; this one is only faster.
__device__ __forceinline__ int lane_order_pos(int q, int k)
{
    const int vec = k >= 32 ? 4 : (k >= 16 ? 2 : 1);
    if (k % vec) return q;
    const int lpe = k / vec;
    return vec * (q % lpe) + q / lpe;
}

template <int ORDER>
__global__ __launch_bounds__(kBlock) void topk_kernel(const float *__restrict__ x, int num_rows,
                                                      int dim, int64_t ld, int k,
                                                      float *__restrict__ data,
                                                      uint8_t *__restrict__ sel,
                                                      float *__restrict__ dense)
{
    __shared__ uint64_t stage[kWavesPerBlock][kMaxDim];  // value order: (key << 32 | ~col)
    const int lane = threadIdx.x & (kWave - 1);
    const int wl = threadIdx.x / kWave;
    const int64_t nwaves = (int64_t)gridDim.x * kWavesPerBlock;
    const bool vec = (dim & 3) == 0 && (ld & 3) == 0;
    auto load_row = [&](int64_t rr, float *v) {
        const float *row = x + rr * ld;
        if (vec && 4 * lane < dim) {
            const float4 q = *reinterpret_cast<const float4 *>(row + 4 * lane);
            v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = (4 * lane + j < dim) ? row[4 * lane + j] : 0.f;
        }
    };
    int64_t r = (int64_t)blockIdx.x * kWavesPerBlock + wl;
    uint32_t prevT = 0xbf800000u;  // key of 1.0f: a start for the first row
    float nx[4] = {0.f, 0.f, 0.f, 0.f};
    if (r < num_rows) load_row(r, nx);
    for (; r < num_rows; r += nwaves) {
        float v[4];
        uint32_t key[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = nx[j];
        if (r + nwaves < num_rows) load_row(r + nwaves, nx);  // next row in flight
#pragma unroll
        for (int j = 0; j < 4; ++j) key[j] = (4 * lane + j < dim) ? float_key(v[j]) : 0u;
        // T = the largest key value with #{key >= T} >= k (the k-th largest key),
        // or any T with exactly k keys >= T (then those k are the selection).
        // Search: bracket [lo, hi) with count(lo) >= k > count(hi), found by
        // galloping from the previous row's T (rows of one feature matrix have
        // similar distributions), then bisection with an early stop.
        auto count_ge = [&](uint64_t t) -> int {
            if (t > 0xffffffffull) return 0;
            const uint32_t c32 = (uint32_t)t;
            int cnt = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) cnt += popc64(__ballot(key[j] >= c32));
            return cnt;
        };
        uint64_t lo, hi;
        uint32_t T;
        bool exact = false;
        {
            const int c0 = count_ge(prevT);
            if (c0 == k) {
                T = prevT;
                exact = true;
            } else if (c0 > k) {  // gallop up
                lo = prevT;
                uint64_t step = 1u << TOPK_GALLOP;
                for (;;) {
                    const uint64_t t = lo + step;
                    const int c = count_ge(t);
                    if (c == k) { T = (uint32_t)t; exact = true; break; }
                    if (c < k) { hi = t; break; }
                    lo = t;
                    step <<= 2;
                }
            } else {  // gallop down (count(0) = #valid >= k, so this ends)
                hi = prevT;
                uint64_t step = 1u << TOPK_GALLOP;
                for (;;) {
                    const uint64_t t = hi > step ? hi - step : 0;
                    const int c = count_ge(t);
                    if (c == k) { T = (uint32_t)t; exact = true; break; }
                    if (c > k) { lo = t; break; }
                    hi = t;
                    step <<= 2;
                }
            }
            while (!exact && hi - lo > 1) {
                const uint64_t mid = lo + ((hi - lo) >> 1);
                const int c = count_ge(mid);
                if (c == k) { T = (uint32_t)mid; exact = true; break; }
                if (c > k) lo = mid; else hi = mid;
            }
            if (!exact) T = (uint32_t)lo;
            prevT = T;
        }
        uint64_t gt[4], eq[4];
        int n_gt = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            gt[j] = __ballot(key[j] > T);
            eq[j] = __ballot(key[j] == T && 4 * lane + j < dim);
            n_gt += popc64(gt[j]);
        }
        const int need = k - n_gt;  // ties to take, lowest column first
        int eq_before = 0;          // ties at lower columns than this lane's first entry
#pragma unroll
        for (int j = 0; j < 4; ++j) eq_before += prefix_count(eq[j]);
        bool take[4];
        int mine = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const bool t = (eq[j] >> lane) & 1;
            take[j] = ((gt[j] >> lane) & 1) || (t && eq_before < need);
            eq_before += t;
        }
        // column-order position: selected entries at lower columns
        uint64_t sm[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) sm[j] = __ballot(take[j]);
        int pos = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) pos += prefix_count(sm[j]);
        float *drow = data + r * (int64_t)k;
        uint8_t *srow = sel + r * (int64_t)k;
        if constexpr (ORDER != MAXK_TOPK_ORDER_VALUE) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (take[j]) {
                    const int q = pos + mine;
                    const int o = ORDER == MAXK_TOPK_ORDER_LANE ? lane_order_pos(q, k) : q;
                    drow[o] = v[j];
                    srow[o] = (uint8_t)(4 * lane + j);
                    ++mine;
                }
            }
        } else {
            uint64_t *st = stage[wl];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (take[j]) {
                    st[pos + mine] = ((uint64_t)key[j] << 32) | (uint32_t)~(uint32_t)(4 * lane + j);
                    ++mine;
                }
            }
            wave_sync_lds();
            if (k > 16 && k <= kWave) {  // (k <= 16: the rank loop below measured faster)
                // bitonic sort of the k composites (key desc, column asc) across
                // the first n lanes (padding = 0 sorts last); lane i then holds rank i
                uint64_t a = lane < k ? st[lane] : 0ull;
                int n = 1;  // network size: the next power of two >= k (lanes < n)
                while (n < k) n <<= 1;
                for (int size = 2; size <= n; size <<= 1) {
                    for (int stride = size >> 1; stride > 0; stride >>= 1) {
                        const uint64_t b = __shfl_xor(a, stride);
                        // block direction: descending where bit `size` is clear (every
                        // lane below n in the final merge, size = n)
                        const bool desc = (lane & size) == 0;
                        const bool lower = (lane & stride) == 0;
                        a = (desc == lower) ? (a > b ? a : b) : (a < b ? a : b);
                    }
                }
                if (lane < k) {
                    const int col = (int)(~(uint32_t)a);
                    drow[lane] = x[r * ld + col];  // the original value (keeps -0.0)
                    srow[lane] = (uint8_t)col;
                }
            } else {
                // k <= 16 or k > 64: rank = #selected entries ordered before this one
                // (key desc, column asc)
                mine = 0;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (take[j]) {
                        const uint64_t me = st[pos + mine];
                        int rank = 0;
                        for (int t = 0; t < k; ++t) rank += st[t] > me;
                        drow[rank] = v[j];
                        srow[rank] = (uint8_t)(4 * lane + j);
                        ++mine;
                    }
                }
            }
            wave_sync_lds();
        }
        if (dense) {
            float *orow = dense + r * (int64_t)dim;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (4 * lane + j < dim) orow[4 * lane + j] = take[j] ? v[j] : 0.f;
        }
    }
}

// DENSE_SRC: vals is a dense [num_rows, dim] array read at the selected
// columns (MaxK backward: grad masked to the top-k), else [num_rows, k].
template <bool DENSE_SRC>
__global__ __launch_bounds__(kBlock) void scatter_kernel(const float *__restrict__ vals,
                                                         const uint8_t *__restrict__ sel,
                                                         int num_rows, int k, int dim,
                                                         float *__restrict__ out)
{
    typedef float f4v __attribute__((ext_vector_type(4)));
    __shared__ __attribute__((aligned(16))) float rowbuf[kWavesPerBlock][kMaxDim];
    const int lane = threadIdx.x & (kWave - 1);
    const int wl = threadIdx.x / kWave;
    float *rb = rowbuf[wl];
    const int64_t nwaves = (int64_t)gridDim.x * kWavesPerBlock;
    const bool vec = (dim & 3) == 0;
    // the dense row leaves as one 16-B non-temporal store per lane (written
    // once, never re-read here: Reddit 0.060 -> 0.039 ms)
    auto store_row = [&](int64_t r) {
        float *orow = out + r * (int64_t)dim;
        if (vec) {
            if (4 * lane < dim)
                __builtin_nontemporal_store(reinterpret_cast<const f4v *>(rb)[lane],
                                            reinterpret_cast<f4v *>(orow) + lane);
        } else {
            for (int i = lane; i < dim; i += kWave) orow[i] = rb[i];
        }
    };
    auto zero_row = [&]() {
        if (vec) {
            if (4 * lane < dim) reinterpret_cast<f4v *>(rb)[lane] = f4v{0.f, 0.f, 0.f, 0.f};
        } else {
            for (int i = lane; i < dim; i += kWave) rb[i] = 0.f;
        }
    };
    int64_t r = (int64_t)blockIdx.x * kWavesPerBlock + wl;
    if (k <= kWave) {
        // one entry per lane; the next row's entries are loaded while this row
        // is assembled and stored (one row in flight per wave was latency-bound:
        // products 3.4 TB/s of rows written)
        auto fetch = [&](int64_t rr, int &c, float &v) {
            c = dim;
            v = 0.f;
            if (rr < num_rows && lane < k) {
                c = sel[rr * k + lane];
                if (!DENSE_SRC) v = vals[rr * k + lane];
            }
        };
        int nc;
        float nv;
        fetch(r, nc, nv);
        for (; r < num_rows; r += nwaves) {
            const int c = nc;
            float v = nv;
            fetch(r + nwaves, nc, nv);
            if (DENSE_SRC && c < dim) v = vals[r * (int64_t)dim + c];
            zero_row();
            wave_sync_lds();
            if (c < dim) rb[c] = v;
            wave_sync_lds();
            store_row(r);
            wave_sync_lds();
        }
        return;
    }
    for (; r < num_rows; r += nwaves) {
        zero_row();
        wave_sync_lds();
        for (int j = lane; j < k; j += kWave) {
            const int c = sel[r * (int64_t)k + j];
            if (c < dim) rb[c] = DENSE_SRC ? vals[r * (int64_t)dim + c] : vals[r * (int64_t)k + j];
        }
        wave_sync_lds();
        store_row(r);
        wave_sync_lds();
    }
}

inline int launch_status()
{
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MAXK_OK : (int)e;
}

inline unsigned grid_for(int num_rows)
{
    // enough waves to fill 256 CUs x 8 waves; rows beyond are grid-strided
    const int64_t blocks = ((int64_t)num_rows + kWavesPerBlock - 1) / kWavesPerBlock;
    return (unsigned)(blocks < 2048 ? blocks : 2048);
}

}  // namespace

extern "C" {

int maxk_topk_cbsr(const float *x, int num_rows, int dim, int64_t ld, int k, int order,
                   float *cbsr_data, uint8_t *cbsr_sel, float *dense_out, void *stream)
{
    if (num_rows < 0 || (num_rows > 0 && (!x || !cbsr_data || !cbsr_sel))) return MAXK_E_ARG;
    if (dim < 1 || dim > kMaxDim || k < 1 || k > dim || ld < dim) return MAXK_E_DIM;
    if (order != MAXK_TOPK_ORDER_COLUMN && order != MAXK_TOPK_ORDER_VALUE &&
        order != MAXK_TOPK_ORDER_LANE)
        return MAXK_E_ARG;
    if (num_rows == 0) return MAXK_OK;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const dim3 g(grid_for(num_rows)), b(kBlock);
    if (order == MAXK_TOPK_ORDER_VALUE)
        hipLaunchKernelGGL(topk_kernel<MAXK_TOPK_ORDER_VALUE>, g, b, 0, st, x, num_rows, dim, ld,
                           k, cbsr_data, cbsr_sel, dense_out);
    else if (order == MAXK_TOPK_ORDER_LANE)
        hipLaunchKernelGGL(topk_kernel<MAXK_TOPK_ORDER_LANE>, g, b, 0, st, x, num_rows, dim, ld,
                           k, cbsr_data, cbsr_sel, dense_out);
    else
        hipLaunchKernelGGL(topk_kernel<MAXK_TOPK_ORDER_COLUMN>, g, b, 0, st, x, num_rows, dim, ld,
                           k, cbsr_data, cbsr_sel, dense_out);
    return launch_status();
}

int maxk_cbsr_scatter(const float *vals, const uint8_t *cbsr_sel, int num_rows, int k, int dim,
                      float *out, void *stream)
{
    if (num_rows < 0 || (num_rows > 0 && (!vals || !cbsr_sel || !out))) return MAXK_E_ARG;
    if (dim < 1 || dim > kMaxDim || k < 1 || k > dim) return MAXK_E_DIM;
    if (num_rows == 0) return MAXK_OK;
    hipLaunchKernelGGL(scatter_kernel<false>, dim3(grid_for(num_rows)), dim3(kBlock), 0,
                       reinterpret_cast<hipStream_t>(stream), vals, cbsr_sel, num_rows, k, dim,
                       out);
    return launch_status();
}

int maxk_cbsr_mask(const float *src, const uint8_t *cbsr_sel, int num_rows, int k, int dim,
                   float *out, void *stream)
{
    if (num_rows < 0 || (num_rows > 0 && (!src || !cbsr_sel || !out))) return MAXK_E_ARG;
    if (dim < 1 || dim > kMaxDim || k < 1 || k > dim) return MAXK_E_DIM;
    if (num_rows == 0) return MAXK_OK;
    hipLaunchKernelGGL(scatter_kernel<true>, dim3(grid_for(num_rows)), dim3(kBlock), 0,
                       reinterpret_cast<hipStream_t>(stream), src, cbsr_sel, num_rows, k, dim,
                       out);
    return launch_status();
}

}  // extern "C"
