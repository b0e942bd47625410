// maxk_plan.hip -- MI355X (gfx950) once-per-graph plan builders for the
// backward SSpMM, so that a C / C++ caller of the ABI reaches every backward
// algorithm without a Python host:
//
//  * maxk_csc_build: the CSC transpose the STAGED backward scatters into
//    (csc_indptr, and csc_pos[e] = CSC slot of CSR edge e; edges of one
//    column keep CSR order, so the segmented sums are deterministic);
//  * maxk_local_plan_build: the LOCAL backward's destination ranges (cut by
//    in-degree, at most dmax destinations each), every range's in-edges in
//    source-row order packed as (row | c_local << 24, value), and the
//    permutation that produced them;
//  * maxk_local_bands_build: the per-band first edge of every range;
//  * maxk_tile_plan_build: the TILE backward's header and record streams
//    (destination groups x source ranges, 47-row chunks of each workgroup's
//    distinct source rows; format above bwd_tile_kernel in maxk_spgemm.hip),
//    and maxk_tile_plan_set_values, which rewrites the records' edge values
//    in place when the graph's values change.
//
// The reference has no counterpart (its backward takes the same .warp4 chunk
// list as the forward, kernels/spmm_maxk_backward.cu:117-139); these replace
// the torch sort/scan plumbing that spgemm_new_amd/ops.py used before.
// Stable sorts are rocPRIM LSD radix sorts; everything else is one thread per
// output with a binary search.  All builders are asynchronous except the
// count call of maxk_local_plan_build (one host read of the range count).
#include <cstring>
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <stdint.h>

#include "../../include/maxk_spgemm.h"
#include "tile_format.h"

namespace {

constexpr int kThreads = 256;

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
int64_t blocks_for(int64_t n) { return (n + kThreads - 1) / kThreads; }

unsigned bits_for(int64_t n)  // bits to represent every value in [0, n)
{
    unsigned b = 1;
    while (b < 31 && (int64_t(1) << b) < n) ++b;
    return b;
}

int launch_status()
{
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MAXK_OK : (int)e;
}

// first i in [0, n) with a[i] >= x (n if none)
__device__ __forceinline__ int64_t lower_bound(const int32_t *a, int64_t n, int64_t x)
{
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (a[mid] < x) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// first i in [0, n) with a[i] > x (n if none)
__device__ __forceinline__ int64_t upper_bound(const int32_t *a, int64_t n, int64_t x)
{
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (a[mid] <= x) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// ------------------------------------------------------------------ CSC
__global__ void scatter_rank_kernel(const int32_t *__restrict__ perm, int64_t n,
                                    int32_t *__restrict__ pos)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) pos[perm[i]] = (int32_t)i;
}

// inv[pos[i]] = i
__global__ void invert_kernel(const int32_t *__restrict__ pos, int64_t n, int32_t *__restrict__ inv)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) inv[pos[i]] = (int32_t)i;
}

// out[c] = first i with sorted[i] >= c, c in [0, n_out)
__global__ void lower_bounds_kernel(const int32_t *__restrict__ sorted, int64_t n,
                                    int32_t *__restrict__ out, int64_t n_out)
{
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c < n_out) out[c] = (int32_t)lower_bound(sorted, n, c);
}

// ------------------------------------------------------ column-blocked forward
// key of edge e = (column block of its source) * V + (its row): the restacked
// CSR's row.  The row comes from a binary search of e in indptr.
__global__ void blocked_keys_kernel(const int32_t *__restrict__ indptr, int num_rows,
                                    const int32_t *__restrict__ indices, int64_t num_edges,
                                    int num_cols, int num_blocks, int32_t *__restrict__ key)
{
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= num_edges) return;
    int lo = 0, hi = num_rows;  // last row r with indptr[r] <= e
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (indptr[mid] <= e) lo = mid; else hi = mid;
    }
    const int b = (int)(((int64_t)indices[e] * num_blocks) / num_cols);
    key[e] = b * num_rows + lo;
}

// dst[i] = src[perm[i]] (32-bit words)
__global__ void permute32_kernel(const uint32_t *__restrict__ src, const int32_t *__restrict__ perm,
                                 int64_t n, uint32_t *__restrict__ dst)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[perm[i]];
}

// ---------------------------------------------------------------- LOCAL
// cut[w] = first destination i with csc_indptr[i] >= w * E / T (exact integer
// form of the balanced split), cut[0] = 0, cut[T] = V
__global__ void local_cuts_kernel(const int32_t *__restrict__ csc_indptr, int num_cols,
                                  int64_t num_edges, int T, int32_t *__restrict__ cut)
{
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w > T) return;
    if (w == 0) { cut[0] = 0; return; }
    if (w == T) { cut[T] = num_cols; return; }
    // first i with csc_indptr[i] * T >= w * E
    int64_t lo = 0, hi = num_cols;
    const int64_t x = (int64_t)w * num_edges;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if ((int64_t)csc_indptr[mid] * T < x) lo = mid + 1; else hi = mid;
    }
    cut[w] = (int32_t)lo;
}

// pieces[w]: ranges of at most dmax destinations covering [cut[w], cut[w+1])
__global__ void local_pieces_kernel(const int32_t *__restrict__ cut, int T, int dmax,
                                    int32_t *__restrict__ pieces)
{
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w > T) return;
    if (w == T) { pieces[T] = 0; return; }
    const int span = cut[w + 1] - cut[w];
    pieces[w] = span > 0 ? (span + dmax - 1) / dmax : 0;
}

__global__ void local_dstart_kernel(const int32_t *__restrict__ cut, const int32_t *__restrict__ off,
                                    int T, int dmax, int num_cols, int W, int32_t *__restrict__ dstart)
{
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w > T) return;
    if (w == T) { dstart[W] = num_cols; return; }
    const int a = cut[w], b = cut[w + 1];
    for (int j = 0, d = a; d < b; ++j, d += dmax)
        if (off[w] + j < W) dstart[off[w] + j] = d;
}

__global__ void local_owner_kernel(const int32_t *__restrict__ indices, int64_t num_edges,
                                   const int32_t *__restrict__ dstart, int W,
                                   int32_t *__restrict__ owner)
{
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < num_edges) owner[e] = (int32_t)(upper_bound(dstart, (int64_t)W + 1, indices[e]) - 1);
}

// plan slot i: CSR edge perm[i] = (row r, column c) of range owner_sorted[i]
__global__ void local_records_kernel(const int32_t *__restrict__ indptr, int num_rows,
                                     const int32_t *__restrict__ indices,
                                     const float *__restrict__ values,
                                     const int32_t *__restrict__ dstart,
                                     const int32_t *__restrict__ owner_sorted,
                                     const int32_t *__restrict__ perm, int64_t num_edges,
                                     int32_t *__restrict__ edge_rc, float *__restrict__ edge_val)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= num_edges) return;
    const int32_t e = perm[i];
    const int32_t r = (int32_t)(upper_bound(indptr, (int64_t)num_rows + 1, e) - 1);
    const int32_t cl = indices[e] - dstart[owner_sorted[i]];
    edge_rc[i] = r | (cl << 24);
    if (edge_val) edge_val[i] = values[e];
}

// seg[s * W + w] = first edge of range w whose source row >= floor(s * V / NS);
// row NS = the ranges' ends
__global__ void local_bands_kernel(const int32_t *__restrict__ woff,
                                   const int32_t *__restrict__ edge_rc, int W, int num_rows,
                                   int NS, int32_t *__restrict__ seg)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)(NS + 1) * W) return;
    const int s = (int)(t / W), w = (int)(t % W);
    const int b = woff[w], e = woff[w + 1];
    if (s == NS) { seg[t] = e; return; }
    const int64_t cut = (int64_t)s * num_rows / NS;
    int lo = b, hi = e;  // first edge with row >= cut (rows ascend within a range)
    while (lo < hi) {
        const int mid = lo + ((hi - lo) >> 1);
        if ((int64_t)(edge_rc[mid] & 0xffffff) < cut) lo = mid + 1; else hi = mid;
    }
    seg[t] = lo;
}

template <typename T>
T *carve(char *&p, size_t count)
{
    T *r = reinterpret_cast<T *>(p);
    p += align_up(count * sizeof(T), 256);
    return r;
}

size_t sort_temp_bytes(int64_t n, unsigned end_bit)
{
    size_t bytes = 0;
    rocprim::counting_iterator<int32_t> iota(0);
    if (rocprim::radix_sort_pairs(nullptr, bytes, (const int32_t *)nullptr, (int32_t *)nullptr, iota,
                                  (int32_t *)nullptr, (size_t)n, 0u, end_bit) != hipSuccess)
        return 0;
    return bytes;
}

size_t scan_temp_bytes(int64_t n)
{
    size_t bytes = 0;
    if (rocprim::exclusive_scan(nullptr, bytes, (const int32_t *)nullptr, (int32_t *)nullptr, 0,
                                (size_t)n, rocprim::plus<int32_t>()) != hipSuccess)
        return 0;
    return bytes;
}

// ----------------------------------------------------------------- TILE
// Plan of bwd_tile_kernel (format above it in maxk_spgemm.hip).  Edge e =
// (row r, column d): destination group g = d / GS, piece wg = tile_piece(g, r)
// (tile_format.h: the (group, row) space cut into P equal workgroup ranges;
// G + P - 1 piece ids, "wg" below).  Within a piece, the distinct source rows
// (ascending) are cut into 47-row chunks; an edge's segment is (wg, wave,
// chunk, lane half) with wave = (d % GS) % 16.
// Segments are numbered in record-stream order, (wg, wave)-major:
//   seg = ((chunk_base[wg] * 16 + wave * nch[wg] + chunk) * 2 + half),
// and within a segment the records keep CSR edge order (two stable sorts).
constexpr int kTileLead = kTileBufs - 1;  // header entries before chunk 0's counts
constexpr int kTileRecPad = 512;   // records of over-read padding after the stream (the
                                   // kernel's prefetch window is static_asserted against it)
constexpr int kTileHdrPad = 8;     // header entries of padding

__global__ void tile_edge_kernel(const int32_t *__restrict__ indptr, int num_rows,
                                 const int32_t *__restrict__ indices, int64_t num_edges, int GS,
                                 int G, int P, int32_t *__restrict__ wg_key,
                                 int32_t *__restrict__ erow)
{
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= num_edges) return;
    const int r = (int)(upper_bound(indptr, (int64_t)num_rows + 1, e) - 1);
    erow[e] = r;
    wg_key[e] = tile_piece(indices[e] / GS, r, num_rows, G, P);
}

// flag[i] = 1 where the wg-sorted edge i starts a new (workgroup, row) pair
__global__ void tile_flag_kernel(const int32_t *__restrict__ wgs, const int32_t *__restrict__ perm,
                                 const int32_t *__restrict__ erow, int64_t n,
                                 int32_t *__restrict__ flag)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    flag[i] = (i == 0 || wgs[i] != wgs[i - 1] || erow[perm[i]] != erow[perm[i - 1]]) ? 1 : 0;
}

// the distinct (workgroup, row) pairs; uidx = inclusive scan of the flags
__global__ void tile_unique_kernel(const int32_t *__restrict__ uidx, const int32_t *__restrict__ wgs,
                                   const int32_t *__restrict__ perm, const int32_t *__restrict__ erow,
                                   int64_t n, int32_t *__restrict__ urow, int32_t *__restrict__ uwg)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || (i > 0 && uidx[i] == uidx[i - 1])) return;
    const int u = uidx[i] - 1;
    urow[u] = erow[perm[i]];
    uwg[u] = wgs[i];
}

// wg_start[b] = first distinct pair of workgroup b (b in [0, NWG]); nch_in[b] =
// its chunk count (input of the chunk_base scan, nch_in[NWG] = 0)
__global__ void tile_wg_kernel(const int32_t *__restrict__ uwg, const int32_t *__restrict__ num_unique,
                               int NWG, int32_t *__restrict__ wg_start)
{
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b <= NWG) wg_start[b] = (int32_t)lower_bound(uwg, *num_unique, b);
}

__global__ void tile_nch_kernel(const int32_t *__restrict__ wg_start, int NWG,
                                int32_t *__restrict__ nch_in, int32_t *__restrict__ num_chunks)
{
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b > NWG) return;
    const int n = b < NWG ? (wg_start[b + 1] - wg_start[b] + kTileRows - 1) / kTileRows : 0;
    nch_in[b] = n;
    if (num_chunks && b < NWG) num_chunks[b] = n;
}

__device__ __forceinline__ void tile_edge_place(int32_t e, int32_t wg, int32_t u,
                                                const int32_t *__restrict__ indices,
                                                const int32_t *__restrict__ wg_start, int GS, int k,
                                                int &wave, int &slot, int &half, int &chunk, int &rin)
{
    const int ri = u - wg_start[wg];
    chunk = ri / kTileRows;
    rin = ri - chunk * kTileRows;
    const int j = indices[e] % GS;
    wave = j % kTileWaves;
    const int q = j / kTileWaves;
    slot = k == 32 ? q >> 1 : q;
    half = k == 32 ? q & 1 : 0;
}

__global__ void tile_seg_kernel(const int32_t *__restrict__ perm, const int32_t *__restrict__ wgs,
                                const int32_t *__restrict__ uidx, const int32_t *__restrict__ indices,
                                const int32_t *__restrict__ wg_start,
                                const int32_t *__restrict__ chunk_base, int GS, int k, int64_t n,
                                int32_t *__restrict__ seg)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int wg = wgs[i];
    int wave, slot, half, chunk, rin;
    tile_edge_place(perm[i], wg, uidx[i] - 1, indices, wg_start, GS, k, wave, slot, half, chunk, rin);
    const int nch = chunk_base[wg + 1] - chunk_base[wg];
    seg[i] = ((chunk_base[wg] * kTileWaves + wave * nch + chunk) << 1) + half;
}

// pad[s] = record count of segment s rounded up to 4 (s < bound; pad[bound] = 0);
// max over the segments into *max_pad (zeroed before)
__global__ void tile_pad_kernel(const int32_t *__restrict__ segs, int64_t n, int64_t bound,
                                int32_t *__restrict__ pad, int32_t *__restrict__ max_pad)
{
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int p = 0;
    if (s < bound) {
        const int64_t c = lower_bound(segs, n, s + 1) - lower_bound(segs, n, s);
        p = (int)((c + 3) & ~int64_t(3));
        pad[s] = p;
    } else if (s == bound) {
        pad[s] = 0;
    }
    for (int o = 32; o > 0; o >>= 1) p = max(p, __shfl_xor(p, o));
    if ((threadIdx.x & 63) == 0 && p > 0) atomicMax(max_pad, p);
}

// sizes: header entries, records (both with padding), max padded segment
__global__ void tile_sizes_kernel(const int32_t *__restrict__ chunk_base, int NWG,
                                  const int64_t *__restrict__ rec_off,
                                  const int32_t *__restrict__ max_pad, int64_t *__restrict__ sizes)
{
    const int64_t chunks = chunk_base[NWG];
    sizes[0] = kTileWaves * (chunks + kTileLead * (int64_t)NWG) + kTileHdrPad;
    sizes[1] = rec_off[chunks * 2 * kTileWaves] + kTileRecPad;
    sizes[2] = *max_pad;
}

__global__ void tile_starts_kernel(const int32_t *__restrict__ chunk_base,
                                   const int64_t *__restrict__ rec_off, int NWG,
                                   int64_t *__restrict__ header_start,
                                   int64_t *__restrict__ record_start)
{
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= NWG * kTileWaves) return;
    const int b = t / kTileWaves, w = t % kTileWaves;
    const int64_t nch = chunk_base[b + 1] - chunk_base[b];
    header_start[t] =
        kTileWaves * ((int64_t)chunk_base[b] + kTileLead * (int64_t)b) + w * (nch + kTileLead);
    record_start[t] = rec_off[((int64_t)chunk_base[b] * kTileWaves + w * nch) * 2];
}

// header entry t of (workgroup b, wave w), index i: counts of chunk i - kTileLead and
// the source rows of the wave's three DMA pieces of chunk i (-1 = zero row)
__global__ void tile_headers_kernel(const int32_t *__restrict__ chunk_base,
                                    const int32_t *__restrict__ wg_start,
                                    const int32_t *__restrict__ urow,
                                    const int32_t *__restrict__ pad, int NWG, int64_t capacity,
                                    int4 *__restrict__ hdrs)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= capacity) return;
    int4 out = make_int4(0, 0, 0, 0);
    const int64_t total = kTileWaves * ((int64_t)chunk_base[NWG] + kTileLead * (int64_t)NWG);
    if (t < total) {
        int lo = 0, hi = NWG;  // last b with 16 * (chunk_base[b] + 2b) <= t
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (kTileWaves * ((int64_t)chunk_base[mid] + kTileLead * (int64_t)mid) <= t) lo = mid;
            else hi = mid;
        }
        const int b = lo;
        const int64_t nch = chunk_base[b + 1] - chunk_base[b];
        const int64_t local = t - kTileWaves * ((int64_t)chunk_base[b] + kTileLead * (int64_t)b);
        const int w = (int)(local / (nch + kTileLead));
        const int i = (int)(local % (nch + kTileLead));
        if (i >= kTileLead) {
            const int64_t s0 =
                (((int64_t)chunk_base[b] * kTileWaves + w * nch + (i - kTileLead)) << 1);
            out.x = pad[s0] | (pad[s0 + 1] << 16);
        }
        const int nrows = wg_start[b + 1] - wg_start[b];
        int rr[3];
        for (int p = 0; p < kTilePieces; ++p) {
            const int li = w * kTilePieces + p;
            const int64_t r = (int64_t)i * kTileRows + li;
            rr[p] = (li < kTileRows && r < nrows) ? urow[wg_start[b] + r] : -1;
        }
        out.y = rr[0];
        out.z = rr[1];
        out.w = rr[2];
    }
    hdrs[t] = out;
}

// the record of (slot, staged row index in the ring, value) in the build's format
__device__ __forceinline__ void tile_put_record(uint32_t *__restrict__ recs, int64_t pos, int slot,
                                                int ring_row, float value)
{
    uint32_t *r = recs + pos * kTileRecWords;
    if constexpr (kTileRecWords == 2) {
        r[0] = (uint32_t)slot | ((uint32_t)ring_row << 24);
        r[1] = __float_as_uint(value);
    } else {
        // v_perm_b32 selector control: byte 0 = selector register index (slot / 4,
        // M0 for the indexed read; also D's byte 0 selector, don't care), byte 1 =
        // 0x0c (D byte 1 = 0), byte 2 = 4 + slot % 4 (D byte 2 = that byte of the
        // indexed selector register), byte 3 = 0x0c (D byte 3 = 0)
        r[0] = (uint32_t)(slot >> 2) | (0x0cu << 8) | ((uint32_t)(4 + (slot & 3)) << 16) |
               (0x0cu << 24);
        r[1] = (uint32_t)slot;
        r[2] = (uint32_t)ring_row << 10;  // LDS byte address of the staged row
        r[3] = __float_as_uint(value);
    }
}

__global__ void tile_records_init_kernel(uint32_t *__restrict__ recs, int64_t capacity)
{
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < capacity) tile_put_record(recs, t, 0, kTileBufRows - 1, 0.f);  // slot 0, zero row, 0
}

__global__ void tile_records_kernel(const int32_t *__restrict__ segs, const int32_t *__restrict__ perm2,
                                    const int32_t *__restrict__ perm, const int32_t *__restrict__ wgs,
                                    const int32_t *__restrict__ uidx,
                                    const int32_t *__restrict__ wg_start,
                                    const int32_t *__restrict__ indices,
                                    const float *__restrict__ values,
                                    const int64_t *__restrict__ rec_off, int GS, int k, int64_t n,
                                    int64_t capacity, uint32_t *__restrict__ recs,
                                    int32_t *__restrict__ edge_record)
{
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const int32_t s = segs[j];
    const int64_t first = lower_bound(segs, n, s);  // rank within the segment = j - first
    const int32_t i = perm2[j];
    const int32_t e = perm[i];
    int wave, slot, half, chunk, rin;
    tile_edge_place(e, wgs[i], uidx[i] - 1, indices, wg_start, GS, k, wave, slot, half, chunk, rin);
    const int64_t pos = rec_off[s] + (j - first);
    if (pos >= capacity) return;
    tile_put_record(recs, pos, slot, (chunk % kTileBufs) * kTileBufRows + rin, values[e]);
    if (edge_record) edge_record[e] = (int32_t)pos;
}

__global__ void tile_set_values_kernel(const int32_t *__restrict__ edge_record,
                                       const float *__restrict__ values, int64_t n,
                                       uint32_t *__restrict__ recs)
{
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < n)
        recs[(int64_t)edge_record[e] * kTileRecWords + kTileRecWords - 1] = __float_as_uint(values[e]);
}

size_t inclusive_scan_temp_bytes(int64_t n)
{
    size_t bytes = 0;
    if (rocprim::inclusive_scan(nullptr, bytes, (const int32_t *)nullptr, (int32_t *)nullptr,
                                (size_t)n, rocprim::plus<int32_t>()) != hipSuccess)
        return 0;
    return bytes;
}

size_t scan64_temp_bytes(int64_t n)
{
    size_t bytes = 0;
    if (rocprim::exclusive_scan(nullptr, bytes, (const int32_t *)nullptr, (int64_t *)nullptr,
                                int64_t(0), (size_t)n, rocprim::plus<int64_t>()) != hipSuccess)
        return 0;
    return bytes;
}

int64_t tile_seg_bound(int64_t num_edges, int nwg)
{
    // segments = 32 x chunks; chunks <= sum over workgroups of ceil(rows / 47)
    // <= E / 47 + NWG (a workgroup's distinct rows never exceed its edges)
    return 2 * kTileWaves * (num_edges / kTileRows + nwg + 1);
}

int tile_max_group(int k) { return (k == 32 ? 128 : 64) * kTileWaves; }

}  // namespace

extern "C" {

size_t maxk_csc_workspace_bytes(int64_t num_edges, int num_cols)
{
    if (num_edges < 0 || num_cols < 1) return 0;
    return align_up((size_t)num_edges * 4, 256) * 2 +
           align_up(sort_temp_bytes(num_edges, bits_for(num_cols)), 256) + 256;
}

int maxk_csc_build(const int32_t *indices, int64_t num_edges, int num_cols, int32_t *csc_indptr,
                   int32_t *csc_pos, void *workspace, size_t workspace_bytes, void *stream)
{
    if (num_edges < 0 || num_edges > INT32_MAX || num_cols < 1 || !csc_indptr) return MAXK_E_ARG;
    if (num_edges > 0 && (!indices || !csc_pos)) return MAXK_E_ARG;
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (num_edges == 0) {
        return (int)hipMemsetAsync(csc_indptr, 0, sizeof(int32_t) * ((size_t)num_cols + 1), st);
    }
    if (!workspace || workspace_bytes < maxk_csc_workspace_bytes(num_edges, num_cols))
        return MAXK_E_WORKSPACE;
    const unsigned bits = bits_for(num_cols);
    char *p = static_cast<char *>(workspace);
    int32_t *keys_sorted = carve<int32_t>(p, num_edges);
    int32_t *perm = carve<int32_t>(p, num_edges);
    size_t tb = sort_temp_bytes(num_edges, bits);
    rocprim::counting_iterator<int32_t> iota(0);
    hipError_t e = rocprim::radix_sort_pairs(p, tb, indices, keys_sorted, iota, perm,
                                             (size_t)num_edges, 0u, bits, st);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(scatter_rank_kernel, dim3((unsigned)blocks_for(num_edges)), dim3(kThreads),
                       0, st, perm, num_edges, csc_pos);
    int rc = launch_status();
    if (rc) return rc;
    hipLaunchKernelGGL(lower_bounds_kernel, dim3((unsigned)blocks_for((int64_t)num_cols + 1)),
                       dim3(kThreads), 0, st, keys_sorted, num_edges, csc_indptr,
                       (int64_t)num_cols + 1);
    return launch_status();
}

size_t maxk_blocked_plan_workspace_bytes(int64_t num_edges, int num_rows, int num_blocks)
{
    if (num_edges < 0 || num_rows < 1 || num_blocks < 1 ||
        (int64_t)num_rows * num_blocks >= INT32_MAX)
        return 0;
    return align_up((size_t)num_edges * 4, 256) * 2 +
           align_up(sort_temp_bytes(num_edges, bits_for((int64_t)num_rows * num_blocks)), 256) + 256;
}

int maxk_blocked_plan_build(const int32_t *indptr, const int32_t *indices, const float *values,
                            int num_rows, int num_cols, int64_t num_edges, int num_blocks,
                            int32_t *out_indptr, int32_t *out_indices, float *out_values,
                            int32_t *out_order, void *workspace, size_t workspace_bytes,
                            void *stream)
{
    if (num_rows < 1 || num_cols < 1 || num_blocks < 1 || num_edges < 0 || num_edges > INT32_MAX ||
        (int64_t)num_rows * num_blocks >= INT32_MAX || !indptr || !out_indptr)
        return MAXK_E_ARG;
    if (num_edges > 0 && (!indices || !out_indices || !out_order)) return MAXK_E_ARG;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const int64_t R = (int64_t)num_rows * num_blocks;
    if (num_edges == 0)
        return (int)hipMemsetAsync(out_indptr, 0, sizeof(int32_t) * ((size_t)R + 1), st);
    if (!workspace ||
        workspace_bytes < maxk_blocked_plan_workspace_bytes(num_edges, num_rows, num_blocks))
        return MAXK_E_WORKSPACE;
    char *p = static_cast<char *>(workspace);
    int32_t *key = carve<int32_t>(p, num_edges);
    int32_t *key_sorted = carve<int32_t>(p, num_edges);
    const unsigned bits = bits_for(R);
    size_t tb = sort_temp_bytes(num_edges, bits);
    hipLaunchKernelGGL(blocked_keys_kernel, dim3((unsigned)blocks_for(num_edges)), dim3(kThreads),
                       0, st, indptr, num_rows, indices, num_edges, num_cols, num_blocks, key);
    int rc = launch_status();
    if (rc) return rc;
    // LSD radix sort: stable, so a restacked row keeps its edges in CSR order
    rocprim::counting_iterator<int32_t> iota(0);
    hipError_t e = rocprim::radix_sort_pairs(p, tb, key, key_sorted, iota, out_order,
                                             (size_t)num_edges, 0u, bits, st);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(lower_bounds_kernel, dim3((unsigned)blocks_for(R + 1)), dim3(kThreads), 0, st,
                       key_sorted, num_edges, out_indptr, R + 1);
    if ((rc = launch_status())) return rc;
    hipLaunchKernelGGL(permute32_kernel, dim3((unsigned)blocks_for(num_edges)), dim3(kThreads), 0,
                       st, reinterpret_cast<const uint32_t *>(indices), out_order, num_edges,
                       reinterpret_cast<uint32_t *>(out_indices));
    if ((rc = launch_status())) return rc;
    if (values && out_values)
        return maxk_permute_f32(values, out_order, num_edges, out_values, stream);
    return MAXK_OK;
}

int maxk_permute_f32(const float *src, const int32_t *perm, int64_t n, float *dst, void *stream)
{
    if (n < 0 || (n > 0 && (!src || !perm || !dst))) return MAXK_E_ARG;
    if (n == 0) return MAXK_OK;
    hipLaunchKernelGGL(permute32_kernel, dim3((unsigned)blocks_for(n)), dim3(kThreads), 0,
                       static_cast<hipStream_t>(stream), reinterpret_cast<const uint32_t *>(src),
                       perm, n, reinterpret_cast<uint32_t *>(dst));
    return launch_status();
}

int maxk_csc_perm_build(const int32_t *csc_pos, int64_t num_edges, int32_t *csc_perm, void *stream)
{
    if (num_edges < 0 || (num_edges > 0 && (!csc_pos || !csc_perm))) return MAXK_E_ARG;
    if (num_edges == 0) return MAXK_OK;
    hipLaunchKernelGGL(invert_kernel, dim3((unsigned)blocks_for(num_edges)), dim3(kThreads), 0,
                       static_cast<hipStream_t>(stream), csc_pos, num_edges, csc_perm);
    return launch_status();
}

size_t maxk_local_plan_workspace_bytes(int64_t num_edges, int num_cols, int target_waves)
{
    if (num_edges < 0 || num_cols < 1 || target_waves < 1) return 0;
    const size_t t = align_up((size_t)(target_waves + 1) * 4, 256);
    // worst case: every destination its own range
    const size_t sort_b = sort_temp_bytes(num_edges, bits_for((int64_t)num_cols + 1));
    const size_t scan_b = scan_temp_bytes((int64_t)target_waves + 1);
    return 3 * t + align_up((size_t)num_edges * 4, 256) * 2 +
           align_up(sort_b > scan_b ? sort_b : scan_b, 256) + 256;
}

int maxk_local_plan_build(const int32_t *indptr, const int32_t *indices, const float *values,
                          int num_rows, int num_cols, int64_t num_edges,
                          const int32_t *csc_indptr, int dmax, int target_waves,
                          int32_t *dstart, int32_t *woff, int32_t *edge_rc, int32_t *edge_perm,
                          float *edge_val, int32_t *num_waves, void *workspace,
                          size_t workspace_bytes, void *stream)
{
    if (!indptr || !indices || !csc_indptr || !num_waves) return MAXK_E_ARG;
    if (num_rows < 1 || num_rows >= (1 << 24) || num_cols < 1 || num_edges < 1 ||
        num_edges > INT32_MAX || dmax < 1 || dmax > 256 || target_waves < 1)
        return MAXK_E_ARG;
    if (!workspace ||
        workspace_bytes < maxk_local_plan_workspace_bytes(num_edges, num_cols, target_waves))
        return MAXK_E_WORKSPACE;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const int T = target_waves;
    char *p = static_cast<char *>(workspace);
    int32_t *cut = carve<int32_t>(p, (size_t)T + 1);
    int32_t *pieces = carve<int32_t>(p, (size_t)T + 1);
    int32_t *off = carve<int32_t>(p, (size_t)T + 1);
    int32_t *owner = carve<int32_t>(p, num_edges);
    int32_t *owner_sorted = carve<int32_t>(p, num_edges);
    const unsigned tb_blocks = (unsigned)blocks_for((int64_t)T + 1);
    hipLaunchKernelGGL(local_cuts_kernel, dim3(tb_blocks), dim3(kThreads), 0, st, csc_indptr,
                       num_cols, num_edges, T, cut);
    hipLaunchKernelGGL(local_pieces_kernel, dim3(tb_blocks), dim3(kThreads), 0, st, cut, T, dmax,
                       pieces);
    int rc = launch_status();
    if (rc) return rc;
    size_t sb = scan_temp_bytes((int64_t)T + 1);
    hipError_t e = rocprim::exclusive_scan(p, sb, pieces, off, 0, (size_t)T + 1,
                                           rocprim::plus<int32_t>(), st);
    if (e != hipSuccess) return (int)e;
    if (!dstart) {  // count call: W = off[T] (pieces[T] = 0)
        int32_t W = 0;
        e = hipMemcpyAsync(&W, off + T, sizeof(int32_t), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) return (int)e;
        *num_waves = W;
        return MAXK_OK;
    }
    if (!woff || !edge_rc || !edge_perm || (edge_val && !values)) return MAXK_E_ARG;
    const int W = *num_waves;
    if (W < 1) return MAXK_E_ARG;
    hipLaunchKernelGGL(local_dstart_kernel, dim3(tb_blocks), dim3(kThreads), 0, st, cut, off, T,
                       dmax, num_cols, W, dstart);
    hipLaunchKernelGGL(local_owner_kernel, dim3((unsigned)blocks_for(num_edges)), dim3(kThreads), 0,
                       st, indices, num_edges, dstart, W, owner);
    rc = launch_status();
    if (rc) return rc;
    const unsigned bits = bits_for((int64_t)W + 1);
    size_t tb = sort_temp_bytes(num_edges, bits);
    rocprim::counting_iterator<int32_t> iota(0);
    e = rocprim::radix_sort_pairs(p, tb, owner, owner_sorted, iota, edge_perm, (size_t)num_edges,
                                  0u, bits, st);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(lower_bounds_kernel, dim3((unsigned)blocks_for((int64_t)W + 1)),
                       dim3(kThreads), 0, st, owner_sorted, num_edges, woff, (int64_t)W + 1);
    hipLaunchKernelGGL(local_records_kernel, dim3((unsigned)blocks_for(num_edges)), dim3(kThreads),
                       0, st, indptr, num_rows, indices, values, dstart, owner_sorted, edge_perm,
                       num_edges, edge_rc, edge_val);
    return launch_status();
}

int maxk_local_bands_build(const int32_t *woff, const int32_t *edge_rc, int num_waves,
                           int num_rows, int num_bands, int32_t *seg_edge_off, void *stream)
{
    if (!woff || !edge_rc || !seg_edge_off || num_waves < 1 || num_rows < 1 || num_bands < 1)
        return MAXK_E_ARG;
    const int64_t n = (int64_t)(num_bands + 1) * num_waves;
    hipLaunchKernelGGL(local_bands_kernel, dim3((unsigned)blocks_for(n)), dim3(kThreads), 0,
                       static_cast<hipStream_t>(stream), woff, edge_rc, num_waves, num_rows,
                       num_bands, seg_edge_off);
    return launch_status();
}

int maxk_tile_format(int *num_buffers, int *buffer_rows)
{
    if (!num_buffers || !buffer_rows) return MAXK_E_ARG;
    *num_buffers = kTileBufs;
    *buffer_rows = kTileBufRows;
    return MAXK_OK;
}

int maxk_tile_record_words(void) { return kTileRecWords; }

int maxk_tile_plan_shape(int num_rows, int num_cols, int num_cus, int dim_k, int *num_groups,
                         int *group_size, int *num_workgroups)
{
    if (num_rows < 1 || num_cols < 1 || num_cus < 1 || (dim_k != 32 && dim_k != 64) ||
        !num_groups || !group_size || !num_workgroups)
        return MAXK_E_ARG;
    // S equal source ranges per group (num_workgroups = G * S, one piece each):
    // as many groups as fill about one workgroup per CU.  Workgroup ranges that
    // straddle groups (num_workgroups = CUs with full groups) balance the rows
    // swept but measured slower: the workgroups no longer sweep the same rows at
    // the same time, which the L2 serves once
    int64_t groups = (num_cols + (int64_t)tile_max_group(dim_k) - 1) / tile_max_group(dim_k);
    int64_t ns = num_cus / groups;
    ns = ns < 1 ? 1 : ns > 8 ? 8 : ns;
    // at most one source range per source row: with P > G * V some workgroup
    // ranges would be empty, and their partial planes never written
    if (ns > num_rows) ns = num_rows;
    // as many groups as the CUs left over allow: smaller groups, same sweep
    const int64_t g2 = num_cus / ns < num_cols ? num_cus / ns : num_cols;
    if (g2 > groups) groups = g2;
    // more groups than CUs (one source range each): whole rounds of workgroups, the
    // groups made smaller rather than a last round leaving most CUs idle (a group's
    // sweep and records scale with its size on such graphs: products k = 64,
    // 2392 -> 2560 groups, 10.86 -> 10.19 ms)
    if (groups > num_cus) {
        const int64_t whole = (groups + num_cus - 1) / num_cus * num_cus;
        groups = whole < num_cols ? whole : num_cols;
    }
    const int64_t size = (num_cols + groups - 1) / groups;
    groups = (num_cols + size - 1) / size;
    *num_groups = (int)groups;
    *group_size = (int)size;
    *num_workgroups = (int)(groups * ns);
    return MAXK_OK;
}

int maxk_tile_part_planes(int num_rows, int num_groups, int num_workgroups)
{
    if (num_rows < 1 || num_groups < 1 || num_workgroups < 1) return MAXK_E_ARG;
    int m = 0;
    for (int g = 0; g < num_groups; ++g) {
        const int n = tile_group_planes(g, num_rows, num_groups, num_workgroups);
        m = n > m ? n : m;
    }
    return m;
}

size_t maxk_tile_plan_workspace_bytes(int64_t num_edges, int num_groups, int num_workgroups)
{
    if (num_edges < 1 || num_groups < 1 || num_workgroups < 1) return 0;
    const int64_t np = (int64_t)num_groups + num_workgroups - 1;
    if (np > INT32_MAX / 2) return 0;
    const int num_pieces = (int)np;
    const int64_t bound = tile_seg_bound(num_edges, num_pieces);
    const size_t ea = align_up((size_t)num_edges * 4, 256);
    size_t t = sort_temp_bytes(num_edges, bits_for(bound + 1));
    const size_t t2 = inclusive_scan_temp_bytes(num_edges);
    const size_t t3 = scan64_temp_bytes(bound + 1);
    const size_t t4 = scan_temp_bytes((int64_t)num_pieces + 1);
    t = t > t2 ? t : t2;
    t = t > t3 ? t : t3;
    t = t > t4 ? t : t4;
    return 9 * ea + 3 * align_up(((size_t)num_pieces + 1) * 4, 256) +
           align_up((size_t)(bound + 1) * 4, 256) + align_up((size_t)(bound + 1) * 8, 256) + 512 +
           align_up(t, 256) + 256;
}

int maxk_tile_plan_build(const int32_t *indptr, const int32_t *indices, const float *values,
                         int num_rows, int num_cols, int64_t num_edges, int dim_k, int num_groups,
                         int group_size, int num_workgroups, void *headers,
                         int64_t header_capacity, int64_t *header_start, void *records,
                         int64_t record_capacity, int64_t *record_start, int32_t *num_chunks,
                         int32_t *edge_record, int64_t *sizes, void *workspace,
                         size_t workspace_bytes, void *stream)
{
    if (!indptr || !indices || !values || !sizes) return MAXK_E_ARG;
    if ((dim_k != 32 && dim_k != 64) || num_rows < 1 || num_cols < 1 || num_edges < 1 ||
        num_edges > INT32_MAX || num_groups < 1 || num_workgroups < 1 ||
        num_workgroups > (1 << 20) || group_size < 1 || group_size > tile_max_group(dim_k) ||
        (int64_t)num_groups * group_size < num_cols || (int64_t)num_groups + num_workgroups > (1 << 22) ||
        (int64_t)num_workgroups > (int64_t)num_groups * num_rows)
        return MAXK_E_ARG;
    // piece ids (tile_format.h); "workgroup" below is a piece
    const int NWG = num_groups + num_workgroups - 1;
    const int64_t bound = tile_seg_bound(num_edges, NWG);
    if (bound + 1 > INT32_MAX) return MAXK_E_ARG;
    if (!workspace ||
        workspace_bytes < maxk_tile_plan_workspace_bytes(num_edges, num_groups, num_workgroups))
        return MAXK_E_WORKSPACE;
    const bool fill = headers != nullptr;
    if (fill && (!records || !header_start || !record_start || !num_chunks)) return MAXK_E_ARG;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const int64_t E = num_edges;
    char *p = static_cast<char *>(workspace);
    int32_t *key = carve<int32_t>(p, E);    // wg keys, then flags, then segment keys
    int32_t *wgs = carve<int32_t>(p, E);    // wg keys sorted
    int32_t *perm = carve<int32_t>(p, E);   // CSR edge of wg-sorted slot i
    int32_t *erow = carve<int32_t>(p, E);   // source row per CSR edge
    int32_t *uidx = carve<int32_t>(p, E);   // 1 + distinct-pair index of wg-sorted slot i
    int32_t *urow = carve<int32_t>(p, E);
    int32_t *uwg = carve<int32_t>(p, E);
    int32_t *segs = carve<int32_t>(p, E);   // segment keys sorted
    int32_t *perm2 = carve<int32_t>(p, E);  // wg-sorted slot of segment-sorted slot j
    int32_t *wg_start = carve<int32_t>(p, (size_t)NWG + 1);
    int32_t *nch_in = carve<int32_t>(p, (size_t)NWG + 1);
    int32_t *chunk_base = carve<int32_t>(p, (size_t)NWG + 1);
    int32_t *pad = carve<int32_t>(p, (size_t)bound + 1);
    int64_t *rec_off = carve<int64_t>(p, (size_t)bound + 1);
    int32_t *max_pad = carve<int32_t>(p, 2);
    int64_t *dsizes = carve<int64_t>(p, 4);
    void *tmp = p;
    const size_t tmp_bytes = workspace_bytes - (size_t)(p - static_cast<char *>(workspace));
    const unsigned eb = (unsigned)blocks_for(E);
    const unsigned wb = (unsigned)blocks_for((int64_t)NWG + 1);
    rocprim::counting_iterator<int32_t> iota(0);
    size_t tb;
    hipError_t e;
    int rc;

    hipLaunchKernelGGL(tile_edge_kernel, dim3(eb), dim3(kThreads), 0, st, indptr, num_rows, indices,
                       E, group_size, num_groups, num_workgroups, key, erow);
    if ((rc = launch_status())) return rc;
    tb = tmp_bytes;
    e = rocprim::radix_sort_pairs(tmp, tb, key, wgs, iota, perm, (size_t)E, 0u, bits_for(NWG), st);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(tile_flag_kernel, dim3(eb), dim3(kThreads), 0, st, wgs, perm, erow, E, key);
    if ((rc = launch_status())) return rc;
    tb = tmp_bytes;
    e = rocprim::inclusive_scan(tmp, tb, key, uidx, (size_t)E, rocprim::plus<int32_t>(), st);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(tile_unique_kernel, dim3(eb), dim3(kThreads), 0, st, uidx, wgs, perm, erow, E,
                       urow, uwg);
    hipLaunchKernelGGL(tile_wg_kernel, dim3(wb), dim3(kThreads), 0, st, uwg, uidx + (E - 1), NWG,
                       wg_start);
    hipLaunchKernelGGL(tile_nch_kernel, dim3(wb), dim3(kThreads), 0, st, wg_start, NWG, nch_in,
                       fill ? num_chunks : nullptr);
    if ((rc = launch_status())) return rc;
    tb = tmp_bytes;
    e = rocprim::exclusive_scan(tmp, tb, nch_in, chunk_base, 0, (size_t)NWG + 1,
                                rocprim::plus<int32_t>(), st);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(tile_seg_kernel, dim3(eb), dim3(kThreads), 0, st, perm, wgs, uidx, indices,
                       wg_start, chunk_base, group_size, dim_k, E, key);
    if ((rc = launch_status())) return rc;
    tb = tmp_bytes;
    e = rocprim::radix_sort_pairs(tmp, tb, key, segs, iota, perm2, (size_t)E, 0u,
                                  bits_for(bound + 1), st);
    if (e != hipSuccess) return (int)e;
    if ((e = hipMemsetAsync(max_pad, 0, sizeof(int32_t), st)) != hipSuccess) return (int)e;
    hipLaunchKernelGGL(tile_pad_kernel, dim3((unsigned)blocks_for(bound + 1)), dim3(kThreads), 0, st,
                       segs, E, bound, pad, max_pad);
    if ((rc = launch_status())) return rc;
    tb = tmp_bytes;
    e = rocprim::exclusive_scan(tmp, tb, pad, rec_off, int64_t(0), (size_t)bound + 1,
                                rocprim::plus<int64_t>(), st);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(tile_sizes_kernel, dim3(1), dim3(1), 0, st, chunk_base, NWG, rec_off, max_pad,
                       dsizes);
    if ((rc = launch_status())) return rc;
    if (fill) {
        hipLaunchKernelGGL(tile_starts_kernel, dim3((unsigned)blocks_for((int64_t)NWG * kTileWaves)),
                           dim3(kThreads), 0, st, chunk_base, rec_off, NWG, header_start,
                           record_start);
        hipLaunchKernelGGL(tile_headers_kernel, dim3((unsigned)blocks_for(header_capacity)),
                           dim3(kThreads), 0, st, chunk_base, wg_start, urow, pad, NWG,
                           header_capacity, static_cast<int4 *>(headers));
        hipLaunchKernelGGL(tile_records_init_kernel, dim3((unsigned)blocks_for(record_capacity)),
                           dim3(kThreads), 0, st, static_cast<uint32_t *>(records), record_capacity);
        hipLaunchKernelGGL(tile_records_kernel, dim3(eb), dim3(kThreads), 0, st, segs, perm2, perm,
                           wgs, uidx, wg_start, indices, values, rec_off, group_size, dim_k, E,
                           record_capacity, static_cast<uint32_t *>(records), edge_record);
        if ((rc = launch_status())) return rc;
    }
    e = hipMemcpyAsync(sizes, dsizes, 3 * sizeof(int64_t), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return (int)e;
    if (fill && (sizes[0] > header_capacity || sizes[1] > record_capacity)) return MAXK_E_WORKSPACE;
    if (fill && sizes[2] > 0xFFFF) return MAXK_E_ARG;
    return MAXK_OK;
}

int maxk_tile_plan_set_values(const int32_t *edge_record, const float *values, int64_t num_edges,
                              void *records, void *stream)
{
    if (!edge_record || !values || !records || num_edges < 0) return MAXK_E_ARG;
    if (num_edges == 0) return MAXK_OK;
    hipLaunchKernelGGL(tile_set_values_kernel, dim3((unsigned)blocks_for(num_edges)), dim3(kThreads),
                       0, static_cast<hipStream_t>(stream), edge_record, values, num_edges,
                       static_cast<uint32_t *>(records));
    return launch_status();
}

}  // extern "C"
