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
//  * maxk_local_bands_build: the per-band first edge of every range.
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

// out[c] = first i with sorted[i] >= c, c in [0, n_out)
__global__ void lower_bounds_kernel(const int32_t *__restrict__ sorted, int64_t n,
                                    int32_t *__restrict__ out, int64_t n_out)
{
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c < n_out) out[c] = (int32_t)lower_bound(sorted, n, c);
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

}  // extern "C"
