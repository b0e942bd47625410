/*
 * maxk_oracle.c -- CPU restatement of the MaxK-GNN aggregation hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP
 * kernels in spgemm_new_amd/csrc/.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it; the product path never links or
 * calls it (spgemm_new_amd raises if its HIP library is missing).
 *
 * Parity pinning: the reference ships no golden vectors for this path
 *  and its CUDA sources cannot be compiled here (no nvcc),
 * so this restatement is pinned by (a) fixtures produced by importing the
 * reference's own Python MaxK/top-k code (tests/golden/make_golden.py) and
 * (b) torch.sparse.mm, the reference's CPU aggregation op
 * (utils/models.py:281-287).  See DESIGN.md "Oracle".
 *
 * What is restated (reference = /root/reference):
 *   oracle_warp4_count/fill  kernels/generate_meta.py:26-48  (row -> <=64-nnz chunks)
 *   oracle_spmm_forward      kernels/spmm_maxk.cu:17-106     (K1, forward SpGEMM)
 *   oracle_spmm_backward     kernels/spmm_maxk_backward.cu:15-115 (K2, backward SSpMM)
 *
 * The restatement follows the INTENDED math of the kernels,
 * not the tail-block early-exit defect for k<32.
 * Summation order mirrors the reference: K1 sums a chunk's edges in edge
 * order into a chunk-local fp32 row (the shared-memory out_cache,
 * spmm_maxk.cu:66-79) and then adds that row into the output
 * (the atomicAdd writeback, spmm_maxk.cu:101-105), chunks in schedule order.
 * K2 adds each edge's contribution straight into dXs (spmm_maxk_backward.cu:80).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* generate_meta.py:26-48: number of chunks for a CSR row-pointer array. */
long long oracle_warp4_count(const int32_t *indptr, int num_rows, int warp_max_nz)
{
    long long w = 0;
    for (int i = 0; i < num_rows; ++i) {
        int deg = indptr[i + 1] - indptr[i];
        if (deg == 0) continue;                   /* generate_meta.py:32-33 */
        w += (deg + warp_max_nz - 1) / warp_max_nz;
    }
    return w;
}

/* generate_meta.py:34-48: emit (row, loc, len, 0) per chunk.  `loc` is the
 * running edge cursor cur_loc, which equals indptr[row] + offset when
 * indptr[0] == 0. */
long long oracle_warp4_fill(const int32_t *indptr, int num_rows, int warp_max_nz,
                            int32_t *warp4)
{
    long long w = 0;
    int cur_loc = indptr[0];
    for (int i = 0; i < num_rows; ++i) {
        int deg = indptr[i + 1] - indptr[i];
        if (deg == 0) continue;
        int tmp_loc = 0;
        for (;;) {
            warp4[4 * w + 0] = i;
            warp4[4 * w + 1] = cur_loc;
            warp4[4 * w + 3] = 0;
            if (deg - tmp_loc <= warp_max_nz) {
                warp4[4 * w + 2] = deg - tmp_loc;
                cur_loc += deg - tmp_loc;
                ++w;
                break;
            }
            warp4[4 * w + 2] = warp_max_nz;
            cur_loc += warp_max_nz;
            tmp_loc += warp_max_nz;
            ++w;
        }
    }
    return w;
}

/* spmm_maxk.cu:17-106 (intended math).  out must be pre-zeroed by the caller,
 * exactly as the reference binding does (cuda_kernel_bindings.cpp:71). */
int oracle_spmm_forward(const int32_t *warp4, long long num_warps,
                        const int32_t *indices, const float *values,
                        const float *cbsr_data, const uint8_t *cbsr_sel,
                        int num_rows, int dim_origin, int dim_k, float *out)
{
    float *cache = (float *)malloc(sizeof(float) * (size_t)dim_origin);
    if (!cache) return -1;
    for (long long w = 0; w < num_warps; ++w) {
        int row = warp4[4 * w + 0], loc = warp4[4 * w + 1], len = warp4[4 * w + 2];
        if (row < 0 || row >= num_rows) { free(cache); return -2; }
        memset(cache, 0, sizeof(float) * (size_t)dim_origin);     /* spmm_maxk.cu:51-55 */
        for (int i = 0; i < len; ++i) {                            /* spmm_maxk.cu:66-79 */
            int nz = loc + i;
            float left = values[nz];
            const float *d = cbsr_data + (size_t)indices[nz] * dim_k;
            const uint8_t *s = cbsr_sel + (size_t)indices[nz] * dim_k;
            for (int l = 0; l < dim_k; ++l) {
                if (s[l] >= dim_origin) { free(cache); return -3; }
                cache[s[l]] += left * d[l];
            }
        }
        float *o = out + (size_t)row * dim_origin;               /* spmm_maxk.cu:101-105 */
        for (int c = 0; c < dim_origin; ++c) o[c] += cache[c];
    }
    free(cache);
    return 0;
}

/* spmm_maxk_backward.cu:15-115 (intended math).  dxs (num_cols x dim_k: A may be a
 * rectangular row block with halo columns) must be pre-zeroed
 * (cuda_kernel_bindings.cpp:128). */
int oracle_spmm_backward(const int32_t *warp4, long long num_warps,
                         const int32_t *indices, const float *values,
                         const float *grad, const uint8_t *cbsr_sel,
                         int num_rows, int num_cols, int dim_origin, int dim_k, float *dxs)
{
    for (long long w = 0; w < num_warps; ++w) {
        int row = warp4[4 * w + 0], loc = warp4[4 * w + 1], len = warp4[4 * w + 2];
        if (row < 0 || row >= num_rows) return -2;
        const float *g = grad + (size_t)row * dim_origin;       /* staged row, :52-57 */
        for (int i = 0; i < len; ++i) {                          /* :93-104 */
            int col = indices[loc + i];
            if (col < 0 || col >= num_cols) return -4;
            float left = values[loc + i];
            const uint8_t *s = cbsr_sel + (size_t)col * dim_k;
            float *dx = dxs + (size_t)col * dim_k;
            for (int l = 0; l < dim_k; ++l) {
                if (s[l] >= dim_origin) return -3;
                dx[l] += left * g[s[l]];
            }
        }
    }
    return 0;
}

/* Plain CSR restatement used for large property checks: identical math to
 * oracle_spmm_forward with the schedule implied by indptr (one pass per row,
 * rows unsplit).  Threads: none (scalar port). */
int oracle_spmm_forward_csr(const int32_t *indptr, const int32_t *indices,
                            const float *values, const float *cbsr_data,
                            const uint8_t *cbsr_sel, int num_rows, int dim_origin,
                            int dim_k, float *out)
{
    for (int r = 0; r < num_rows; ++r) {
        float *o = out + (size_t)r * dim_origin;
        memset(o, 0, sizeof(float) * (size_t)dim_origin);
        for (int e = indptr[r]; e < indptr[r + 1]; ++e) {
            float left = values[e];
            const float *d = cbsr_data + (size_t)indices[e] * dim_k;
            const uint8_t *s = cbsr_sel + (size_t)indices[e] * dim_k;
            for (int l = 0; l < dim_k; ++l) o[s[l]] += left * d[l];
        }
    }
    return 0;
}

int oracle_spmm_backward_csr(const int32_t *indptr, const int32_t *indices,
                             const float *values, const float *grad,
                             const uint8_t *cbsr_sel, int num_rows, int num_cols,
                             int dim_origin, int dim_k, float *dxs)
{
    memset(dxs, 0, sizeof(float) * (size_t)num_cols * dim_k);
    for (int r = 0; r < num_rows; ++r) {
        const float *g = grad + (size_t)r * dim_origin;
        for (int e = indptr[r]; e < indptr[r + 1]; ++e) {
            int col = indices[e];
            if (col < 0 || col >= num_cols) return -4;
            float left = values[e];
            const uint8_t *s = cbsr_sel + (size_t)col * dim_k;
            float *dx = dxs + (size_t)col * dim_k;
            for (int l = 0; l < dim_k; ++l) dx[l] += left * g[s[l]];
        }
    }
    return 0;
}
