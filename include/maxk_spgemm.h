/*
 * maxk_spgemm.h -- C ABI of the MI355X (gfx950) MaxK-GNN aggregation hot path.
 *
 * This is the drop-in boundary.  It replaces the reference's launch layer,
 *   cuda_kernel_wrappers.cu:36-93   extern "C" spmm_kernel_opt2_sparse_v3_wrapper /
 *                                    spmm_kernel_opt2_sparse_backward_v3_wrapper
 *   cuda_kernel_bindings.cpp:42-161 spmm_maxk_forward / spmm_maxk_backward
 *   kernels/spmm_maxk.cu:108-131, kernels/spmm_maxk_backward.cu:117-139 (SPMM_*::run/do_test)
 *   kernels/generate_meta.py:26-48  (warp4 schedule, now built on the device)
 * and is what a reference-side binding (ctypes / pybind11 / cgo) would bind;
 * see INTEGRATION.md.
 *
 * Conventions
 *  - All pointers are device pointers (hipMalloc / torch CUDA tensors) unless
 *    stated otherwise; sizes are element counts.
 *  - `stream` is a hipStream_t passed as void* (NULL = legacy default stream).
 *    Every call is asynchronous on that stream and performs no allocation and
 *    no host synchronisation, so calls can be captured into a hipGraph.
 *  - Return value: 0 on success; a negative MAXK_E* code for an invalid
 *    argument (nothing launched); a positive hipError_t for a launch failure.
 *  - Layouts (row-major, contiguous).  A is num_rows x num_cols (square in
 *    the single-GPU case; a row block with halo columns on a multi-GPU rank):
 *      CSR    indptr int32[num_rows+1] (indptr[0] may be non-zero),
 *             indices int32[E] (< num_cols), values fp32[E]
 *      CBSR   cbsr_data fp32[num_cols,k], cbsr_sel uint8[num_cols,k] (k distinct
 *             columns < dim_origin per row; the selector is a uint8, so
 *             dim_origin <= 256, as in the reference, spmm_maxk.cu:17)
 *      dense  out / grad fp32[num_rows,dim_origin];  dxs fp32[num_cols,k]
 */
#ifndef MAXK_SPGEMM_H
#define MAXK_SPGEMM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MAXK_OK 0
#define MAXK_E_ARG (-1)        /* bad size / null pointer                  */
#define MAXK_E_DIM (-2)        /* dim_origin > 256 or dim_k outside [1,dim] */
#define MAXK_E_WORKSPACE (-3)  /* workspace too small                       */

/* Default merge-path cost model: one edge costs 1, one output row costs
 * MAXK_DEFAULT_ROW_COST; a panel (one wavefront's work item) costs
 * MAXK_DEFAULT_PANEL_COST. */
#define MAXK_DEFAULT_PANEL_COST 2048
#define MAXK_FWD_ACCUMULATE 1  /* forward flag: out += A . X^ instead of out = A . X^ */
/* forward flag: gather the CBSR data rows with cacheable loads (default:
 * non-temporal).  For a column-blocked call, whose block-major edge order
 * re-reads each source block from L2 (see maxk_rows_sum). */
#define MAXK_FWD_CACHED_GATHER 2
#define MAXK_DEFAULT_ROW_COST 16

/* Library build identification (string, host memory, static). */
const char *maxk_version(void);

/* ABI revision of this header.  Bumped whenever an existing entry point changes
 * its arguments or their meaning (not for added entry points); a binding checks
 * maxk_abi_version() == MAXK_ABI_VERSION at load time and refuses a library
 * built from other sources instead of calling it with the wrong arguments.
 *   5: maxk_tile_plan_shape takes num_rows; num_workgroups <= num_groups *
 *      num_rows is required by maxk_tile_plan_build / maxk_sspmm_backward_tile.
 *   6: the forms measured slower and never chosen (register-accumulator and
 *      bank-ordered multi-relation kernels, BINNED backward) left this library
 *      for the ablation build, tools/variants_lib/maxk_variants.h. */
#define MAXK_ABI_VERSION 6
int maxk_abi_version(void);

/* ---------------------------------------------------------------------------
 * Schedule.  Replaces the offline .warp4 file (generate_meta.py:26-48,
 * loaded by cuda_kernel_bindings.cpp:287-317 / spmm_maxk.cu:117).
 * A schedule is int32[2*(P+1)]: for p = 0..P the merge-path coordinate
 * (row, edge) at cost p*panel_cost over the sequence "edges of row 0, end of
 * row 0, edges of row 1, ...".  Panel p = [coord p, coord p+1) is one
 * wavefront's work; it is balanced in edges + rows by construction.
 * ------------------------------------------------------------------------- */
int maxk_schedule_num_panels(int64_t num_rows, int64_t num_edges, int panel_cost,
                             int row_cost, int64_t *num_panels /* host out */);
int maxk_schedule_build(const int32_t *indptr, int num_rows, int panel_cost, int row_cost,
                        int32_t *sched, int64_t num_panels, void *stream);

/* warp4 schedule on the device (generate_meta.py:26-48 semantics, any
 * warp_max_nz).  chunk_offsets: int32[V+1] scratch.  Count first (returns the
 * chunk count in *num_warps, host memory; this call synchronises the stream),
 * then fill warp4 int32[4*W]. */
int maxk_warp4_build(const int32_t *indptr, int num_rows, int warp_max_nz,
                     int32_t *chunk_offsets, int32_t *warp4, int64_t warp4_capacity,
                     int64_t *num_warps, void *stream);

/* ---------------------------------------------------------------------------
 * Forward SpGEMM  Y = A . scatter(CBSR)      (spmm_maxk.cu:17-106, K1)
 * Writes every row of out (rows of degree 0 become 0); out need not be
 * zeroed.  Workspace: maxk_forward_workspace_bytes(P, dim_origin) bytes.
 * ------------------------------------------------------------------------- */
size_t maxk_forward_workspace_bytes(int64_t num_panels, int dim_origin);
int maxk_spgemm_forward(const int32_t *sched, int64_t num_panels, const int32_t *indptr,
                        const int32_t *indices, const float *values,
                        const float *cbsr_data, const uint8_t *cbsr_sel, int num_rows,
                        int dim_origin, int dim_k, float *out, void *workspace,
                        size_t workspace_bytes, void *stream);
/* The same with flags: MAXK_FWD_ACCUMULATE adds A . X^ into out. */
int maxk_spgemm_forward_ex(const int32_t *sched, int64_t num_panels, const int32_t *indptr,
                           const int32_t *indices, const float *values, const float *cbsr_data,
                           const uint8_t *cbsr_sel, int num_rows, int dim_origin, int dim_k,
                           int flags, float *out, void *workspace, size_t workspace_bytes,
                           void *stream);
/* Column-blocked forward (no reference counterpart; same result up to fp32
 * summation order): the caller restacks the CSR block-major -- row b*V + r
 * holds row r's edges whose sources lie in column block b of NB -- runs
 * maxk_spgemm_forward_ex(..., MAXK_FWD_CACHED_GATHER, ...) on it into
 * partial fp32[NB][V][dim_origin], and sums the parts with maxk_rows_sum
 * (spgemm_new_amd/ops.py, MaxKGraph.blocked_plan).  Pays 2 x NB partial rows
 * per output row; wins where rows are long (Reddit k=32, 4 blocks: 3.29 -> 2.42 ms).
 * out[i] = parts[0][i] + ... + parts[num_parts-1][i] (that order), n floats
 * per part. */
int maxk_rows_sum(const float *parts, int num_parts, int64_t n, float *out, void *stream);
/* The column-blocked forward's last block with the sum fused into its row
 * flush: out[r] = ((parts[0][r] + parts[1][r]) + ... + parts[num_parts-1][r])
 * + (A . X^)[r], parts fp32[num_parts][num_rows][dim_origin] -- bitwise the
 * result of maxk_rows_sum over num_parts + 1 parts, without writing and
 * re-reading the last part or a separate pass.  flags: 0 or
 * MAXK_FWD_CACHED_GATHER; num_parts = 0 is maxk_spgemm_forward_ex. */
int maxk_spgemm_forward_sum_parts(const int32_t *sched, int64_t num_panels, const int32_t *indptr,
                                  const int32_t *indices, const float *values,
                                  const float *cbsr_data, const uint8_t *cbsr_sel, int num_rows,
                                  int dim_origin, int dim_k, int flags, const float *parts,
                                  int num_parts, float *out, void *workspace,
                                  size_t workspace_bytes, void *stream);
/* The column-blocked forward's restacked CSR, built on the device: row b*V + r
 * of out_indptr (int32[num_blocks*V + 1]) holds row r's edges whose source c
 * has c*num_blocks/num_cols == b, in CSR order; out_indices / out_values
 * (int32 / fp32[E]; out_values may be NULL) are indices / values permuted by
 * out_order (int32[E], the CSR edge of each restacked edge).  Needs
 * num_blocks * V < 2^31 and maxk_blocked_plan_workspace_bytes() of device
 * workspace.  Values that change later: maxk_permute_f32(values, out_order, E,
 * out_values, stream). */
size_t maxk_blocked_plan_workspace_bytes(int64_t num_edges, int num_rows, int num_blocks);
int maxk_blocked_plan_build(const int32_t *indptr, const int32_t *indices, const float *values,
                            int num_rows, int num_cols, int64_t num_edges, int num_blocks,
                            int32_t *out_indptr, int32_t *out_indices, float *out_values,
                            int32_t *out_order, void *workspace, size_t workspace_bytes,
                            void *stream);
/* dst[i] = src[perm[i]], n fp32 words. */
int maxk_permute_f32(const float *src, const int32_t *perm, int64_t n, float *dst, void *stream);

/* ---------------------------------------------------------------------------
 * Packed CBSR forward (k = 4, 8, 16).  maxk_cbsr_pack writes one record per
 * node: k fp32 values, then k selector bytes, zero-padded to
 * maxk_cbsr_packed_row_bytes(k) = 32 / 64 / 128 bytes (packed: num_cols x
 * that many bytes, 16-B aligned).  maxk_spgemm_forward_packed is
 * maxk_spgemm_forward reading the records (one cache line per gathered
 * neighbour instead of two); same schedule and workspace.
 * ------------------------------------------------------------------------- */
size_t maxk_cbsr_packed_row_bytes(int dim_k);
int maxk_cbsr_pack(const float *cbsr_data, const uint8_t *cbsr_sel, int num_cols, int dim_k,
                   void *packed, void *stream);
int maxk_spgemm_forward_packed(const int32_t *sched, int64_t num_panels, const int32_t *indptr,
                               const int32_t *indices, const float *values, const void *packed,
                               int num_rows, int dim_origin, int dim_k, float *out,
                               void *workspace, size_t workspace_bytes, void *stream);

/* Forward that also writes the EDGE selectors edge_sel[e * dim_k + l] =
 * cbsr_sel[indices[e] * dim_k + l] for every edge e (CSR order, uint8[E,
 * dim_k]): the selector bytes the forward gathers anyway, stored sequentially,
 * so the backward (MAXK_BWD_STAGED_EDGE) reads them in edge order instead of
 * gathering one selector line per edge again (the dominant cost of the
 * push backward on large graphs, e.g. ogbn-products).  packed = NULL reads
 * cbsr_data / cbsr_sel; packed = maxk_cbsr_pack records (k = 4, 8, 16) reads
 * those.  Same schedule and workspace as maxk_spgemm_forward; overwrites out. */
int maxk_spgemm_forward_esel(const int32_t *sched, int64_t num_panels, const int32_t *indptr,
                             const int32_t *indices, const float *values, const float *cbsr_data,
                             const uint8_t *cbsr_sel, const void *packed, int num_rows,
                             int dim_origin, int dim_k, float *out, uint8_t *edge_sel,
                             void *workspace, size_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------------------
 * Halo records (the multi-GPU path; the reference is
 * single-GPU and has no counterpart).  maxk_cbsr_gather_records writes record
 * i = CBSR row rows[i] (rows == NULL: row i) as dim_k fp32 values followed by
 * dim_k selector bytes, 5*dim_k bytes per record, unpadded -- the all-to-all-v
 * message of packed halo rows.  maxk_spgemm_forward_records is
 * maxk_spgemm_forward reading its CBSR from such records in place (column c =
 * record c; records 16-B aligned); with flags = MAXK_FWD_ACCUMULATE it adds
 * A . X^ into out (out += ...) instead of overwriting it, so a rank's halo
 * column block adds onto the rows its own block wrote.  dim_k a power of two
 * in [4, 256]; same schedule and workspace as maxk_spgemm_forward.
 * ------------------------------------------------------------------------- */
/* dst[seg_row[s], :] += sum_{j in [seg_off[s], seg_off[s+1])} src[order[j], :] for
 * rows of `width` floats: the owners' add of the halo partial sums returned by
 * the peers (reverse exchange of the partitioned backward), in a fixed order
 * (no atomics).  seg_row distinct. */
int maxk_segment_rows_add(const float *src, int width, const int64_t *order,
                          const int64_t *seg_off, const int64_t *seg_row, int64_t num_segments,
                          float *dst, void *stream);
/* out_sel[i, :] = the dim_k selector bytes of record rows[i] of a records array
 * (5*dim_k bytes per record, as maxk_cbsr_gather_records writes them): the halo
 * columns' selectors out of an all-gathered table (PartitionedMaxK halo_mode
 * "allgather"). */
int maxk_records_sel_gather(const uint8_t *records, int dim_k, const int32_t *rows, int64_t n,
                            uint8_t *out_sel, void *stream);
int maxk_cbsr_gather_records(const float *cbsr_data, const uint8_t *cbsr_sel, const int32_t *rows,
                             int64_t num_records, int dim_k, void *records, void *stream);
int maxk_spgemm_forward_records(const int32_t *sched, int64_t num_panels, const int32_t *indptr,
                                const int32_t *indices, const float *values, const void *records,
                                int num_rows, int dim_origin, int dim_k, int flags, float *out,
                                void *workspace, size_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------------------
 * Plan builders (once per graph; spgemm_new_amd/csrc/maxk_plan.hip).  The
 * reference's backward reuses the forward's .warp4 chunks
 * (kernels/spmm_maxk_backward.cu:117-139); the STAGED and LOCAL algorithms
 * need these instead.  CSR with indptr[0] == 0, num_edges = indptr[num_rows].
 *
 * maxk_csc_build: csc_indptr int32[num_cols + 1] and csc_pos int32[num_edges]
 *   (CSC slot of CSR edge e; edges of one column keep CSR order).
 * maxk_local_plan_build: destinations cut into ranges of <= dmax (<= 256)
 *   columns balanced by in-degree (about target_waves ranges); call once with
 *   dstart == NULL to get *num_waves (W; synchronises the stream once), then
 *   with dstart int32[W+1], woff int32[W+1], edge_rc int32[E] (row | c_local
 *   << 24, each range's in-edges in source-row order), edge_perm int32[E]
 *   (the CSR edge of each slot) and edge_val fp32[E] (values[edge_perm], or
 *   NULL) -- the inputs of maxk_sspmm_backward_local.  num_rows < 2^24.
 * maxk_local_bands_build: seg_edge_off int32[(num_bands + 1) * W], source
 *   rows cut into num_bands equal bands (see maxk_sspmm_backward_local).
 * ------------------------------------------------------------------------- */
size_t maxk_csc_workspace_bytes(int64_t num_edges, int num_cols);
int maxk_csc_build(const int32_t *indices, int64_t num_edges, int num_cols, int32_t *csc_indptr,
                   int32_t *csc_pos, void *workspace, size_t workspace_bytes, void *stream);
/* csc_perm[csc_pos[e]] = e: the CSC slot -> CSR edge permutation (MAXK_BWD_EDGE_GATHER). */
int maxk_csc_perm_build(const int32_t *csc_pos, int64_t num_edges, int32_t *csc_perm, void *stream);
size_t maxk_local_plan_workspace_bytes(int64_t num_edges, int num_cols, int target_waves);
int maxk_local_plan_build(const int32_t *indptr, const int32_t *indices, const float *values,
                          int num_rows, int num_cols, int64_t num_edges,
                          const int32_t *csc_indptr, int dmax, int target_waves,
                          int32_t *dstart, int32_t *woff, int32_t *edge_rc, int32_t *edge_perm,
                          float *edge_val, int32_t *num_waves, void *workspace,
                          size_t workspace_bytes, void *stream);
int maxk_local_bands_build(const int32_t *woff, const int32_t *edge_rc, int num_waves,
                           int num_rows, int num_bands, int32_t *seg_edge_off, void *stream);

/* GNNAdvisor-style SAG baseline (kernels/spmm_gnna.cu:60-140, the reference's
 * speedup table README.md:136; not on the MaxK path): out[row] += sum over a
 * part's neighbours of (values[e] or 1) * x[indices[e]], one wave per part of
 * the warp4 schedule built with warp_max_nz = part size (maxk_warp4_build;
 * the reference uses E / V, spmm_gnna.cu:149), float atomics into out (zero it
 * first).  values NULL: unweighted as the reference.  x fp32[num_cols, dim],
 * 16-B aligned, dim % 4 == 0, dim <= 256; warp4 16-B aligned. */
int maxk_spmm_gnna_sag(const int32_t *warp4, int64_t num_parts, const int32_t *indices,
                       const float *values, const float *x, int dim, float *out, void *stream);
/* ---------------------------------------------------------------------------
 * Dense SpMM baseline: out = A . x with x fp32[num_cols, dim] dense, 4 <= dim
 * <= 256, dim % 4 == 0 (the comparison kernels of the reference's speedup
 * table: GNNAdvisor SAG kernels/spmm_gnna.cu:60-140 -- unweighted, pass
 * values = 1 -- and cusparse_spmm, cuda_kernel_bindings.cpp:253-284).  Same
 * schedule as maxk_spgemm_forward, workspace maxk_forward_workspace_bytes(P,
 * dim); out need not be zeroed.
 * ------------------------------------------------------------------------- */
int maxk_spmm_dense_forward(const int32_t *sched, int64_t num_panels, const int32_t *indptr,
                            const int32_t *indices, const float *values, const float *x,
                            int num_rows, int dim, float *out, void *workspace,
                            size_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------------------
 * Fused multi-relation forward (ogbn-proteins, BASELINE config 5; no
 * reference function -- the reference sums proteins' 8 edge features into
 * node features, utils/proteins_loader.py:41-44).  Y[q] = A_q . scatter(CBSR)
 * for q < num_rel <= 16 relations sharing one CSR and one CBSR; values is
 * fp32[num_edges, num_rel] (row-major), out is fp32[num_rel, num_rows,
 * dim_origin].  Equals num_rel calls of maxk_spgemm_forward with values[:, q]
 * (up to fp32 summation order).  dim_k must be a power of two in [4, 256].
 * Same schedule as maxk_spgemm_forward; workspace from
 * maxk_forward_multi_workspace_bytes.
 * ------------------------------------------------------------------------- */
size_t maxk_forward_multi_workspace_bytes(int64_t num_panels, int dim_origin, int num_rel);
/* The same CBSR with each row's entries in bank-aware order for the fused
 * forward over num_rel relations (its LDS stores go 8 entries at a time; the
 * store classes follow the num_rel record layout).  Any order is a valid CBSR
 * and the forward's result is bit-identical; dim_k <= 64, 1 <= num_rel <= 16.
 * out_data / out_sel: num_rows x dim_k. */
int maxk_cbsr_bank_order(const float *cbsr_data, const uint8_t *cbsr_sel, int num_rows,
                         int dim_k, int num_rel, float *out_data, uint8_t *out_sel, void *stream);
int maxk_spgemm_forward_multi(const int32_t *sched, int64_t num_panels, const int32_t *indptr,
                              const int32_t *indices, const float *values, int num_rel,
                              const float *cbsr_data, const uint8_t *cbsr_sel, int num_rows,
                              int dim_origin, int dim_k, float *out, void *workspace,
                              size_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------------------
 * Backward SSpMM  dXs[c,l] = sum_{e: idx[e]=c} val[e] * G[row(e), sel[c,l]]
 * (spmm_maxk_backward.cu:15-115, K2).  Writes every element of dxs (no
 * pre-zeroing needed).  Workspace: maxk_backward_workspace_bytes(...).
 * algo: MAXK_BWD_AUTO = STAGED when the CSC inputs and a workspace are given,
 * else ATOMIC (the measured per-shape choice, LOCAL included, is made above
 * the ABI: MaxKGraph.autotune_backward, or the harness's timing loop).
 * ------------------------------------------------------------------------- */
#define MAXK_BWD_AUTO 0
#define MAXK_BWD_ATOMIC 1      /* push + global float atomics (reference's scheme) */
#define MAXK_BWD_STAGED 2      /* push to per-edge staging rows + CSC segmented sum */
#define MAXK_BWD_LOCAL 3       /* destination-owned LDS accumulation (maxk_sspmm_backward_local) */
#define MAXK_BWD_TILE 4        /* gradient rows staged once per CU (maxk_sspmm_backward_tile) */
#define MAXK_BWD_STAGED_EDGE 5 /* STAGED reading EDGE selectors: cbsr_sel is uint8[num_edges,
                                  dim_k] in CSR edge order (maxk_spgemm_forward_esel's edge_sel)
                                  instead of the node CBSR selectors; workspace as STAGED */
#define MAXK_BWD_EDGE_GATHER 6 /* as STAGED_EDGE, but the per-edge products are written in edge
                                  (CSR) order -- one sequential stream -- and the segmented sum
                                  gathers them per destination: csc_pos is then the CSC slot ->
                                  CSR edge permutation (maxk_csc_perm_build); k a power of
                                  two in [4, 256] */
size_t maxk_backward_workspace_bytes(int algo, int64_t num_edges, int dim_k,
                                     int64_t csc_num_panels);
int maxk_sspmm_backward(int algo, const int32_t *sched, int64_t num_panels,
                        const int32_t *indptr, const int32_t *indices, const float *values,
                        const float *grad, const uint8_t *cbsr_sel, int num_rows,
                        int num_cols, int64_t num_edges, int dim_origin, int dim_k, float *dxs,
                        const int32_t *csc_pos, const int32_t *csc_sched,
                        int64_t csc_num_panels, const int32_t *csc_indptr,
                        void *workspace, size_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------------------
 * Backward SSpMM, APPEND algorithm (write-combined propagation blocking; no
 * reference counterpart -- it replaces K2's atomicAdd push,
 * spmm_maxk_backward.cu:80,101, and is NON-DETERMINISTIC like it: the sum order
 * of a destination follows the arrival order of its products).
 * Destinations are cut into num_bins bins of bin_size columns
 * (maxk_append_bins: a bin's k-vectors fit 160 KB of LDS).  Phase 1 pushes every
 * edge's k products, with its destination, to the region of (its destination's
 * bin, the pushing workgroup's XCD group) through an atomic cursor; the regions
 * of one bin are consecutive, so phase 2 streams each bin once into LDS and
 * writes its dXs rows.  Plan (once per graph and k, maxk_append_plan_build):
 * region_base int32[num_bins * 8 + 1], the first entry of every region in the
 * panel schedule `sched` the backward will use -- the plan belongs to that graph
 * and schedule.  num_rel: 1 (values fp32[E], cbsr_sel node selectors, or edge
 * selectors uint8[E, k] in CSR order when edge_sel != 0), or 4 / 8 / 16 relations
 * (values fp32[E, num_rel], grad fp32[num_rel, num_rows, dim_origin], node
 * selectors; dim_k in {8, 16, 32, 64}: the backward of maxk_spgemm_forward_multi,
 * relations summed per edge).  dim_k a power of two in [4, 256].  Workspace:
 * maxk_backward_append_workspace_bytes.  Writes every element of dxs.
 * ------------------------------------------------------------------------- */
#define MAXK_BWD_APPEND 7
int maxk_append_bins(int num_cols, int dim_k, int *num_bins, int *bin_size);
int maxk_append_plan_build(const int32_t *sched, int64_t num_panels, const int32_t *indptr,
                           const int32_t *indices, int num_rows, int num_cols, int dim_k,
                           int32_t *region_base, int num_bins, int bin_size, void *stream);
size_t maxk_backward_append_workspace_bytes(int64_t num_edges, int dim_k, int num_bins);
int maxk_sspmm_backward_append(const int32_t *sched, int64_t num_panels, const int32_t *indptr,
                               const int32_t *indices, const float *values, int num_rel,
                               const float *grad, const uint8_t *cbsr_sel, int edge_sel,
                               int num_rows, int num_cols, int64_t num_edges, int dim_origin,
                               int dim_k, const int32_t *region_base, int num_bins, int bin_size,
                               float *dxs, void *workspace, size_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------------------
 * Backward SSpMM, LOCAL algorithm: destination-owned dXs in LDS, no atomics
 * and no staging rows.  Needs a plan (built once per graph, ops.py
 * MaxKGraph.local_plan): destinations split into `num_waves` ranges
 * wave_dst_start[0..W] (<= dmax <= 256 each); each range's in-edges sorted by
 * source row, packed as edge_rc = row | (dest - range_start) << 24 and
 * edge_val.  The source rows are cut into `num_segments` bands, one launch
 * each, so the gradient rows in flight stay cache-resident:
 * seg_edge_off[s * W + w] is the first edge of wave w in band s, and row
 * s = num_segments holds each wave's end (for one band: the wave offsets
 * without the last, then without the first).  Band 0 writes the owned dXs
 * rows, later bands add to them.  num_rows < 2^24; dim_k must divide 64; LDS
 * per 4-wave block = maxk_backward_local_lds_bytes(dmax, k) <= 160 KiB.
 * Writes every element of dxs.
 * ------------------------------------------------------------------------- */
size_t maxk_backward_local_lds_bytes(int dmax, int dim_k);
int maxk_sspmm_backward_local(const int32_t *seg_edge_off, int num_segments,
                              const int32_t *wave_dst_start, int num_waves, int dmax,
                              const int32_t *edge_rc, const float *edge_val, const float *grad,
                              const uint8_t *cbsr_sel, int num_rows, int dim_origin, int dim_k,
                              float *dxs, void *stream);

/* Multi-relation LOCAL backward for 8 relations, dim_k = 32 (the backward of
 * maxk_spgemm_forward_multi at ogbn-proteins' R = 8): dxs[c,l] = sum_q sum_e
 * val[e,q] * grad[q, row(e), sel[c,l]].  maxk_grad_interleave turns grad
 * fp32[num_rel, num_rows, dim] into fp32[num_rows, dim, num_rel] (relation
 * innermost); the kernel then fetches an edge's 8 relations at a selected
 * column as 32 contiguous bytes.  edge_val: fp32[E, 8] in the plan's edge
 * order (values[edge_perm, :]), 16-B aligned; same plan as
 * maxk_sspmm_backward_local, bands sized for 8 gradient rows per source row. */
int maxk_grad_interleave(const float *grad, int num_rel, int num_rows, int dim, float *out,
                         void *stream);
int maxk_sspmm_backward_local_rel8(const int32_t *seg_edge_off, int num_segments,
                                   const int32_t *wave_dst_start, int num_waves, int dmax,
                                   const int32_t *edge_rc, const float *edge_val,
                                   const float *grad_interleaved, const uint8_t *cbsr_sel,
                                   int num_rows, int dim_origin, int dim_k, float *dxs,
                                   void *stream);

/* Multi-relation STAGED backward (the backward of maxk_spgemm_forward_multi;
 * config 5, ogbn-proteins R = 8): dxs[c,l] = sum_q sum_e val[e,q] *
 * grad[q, row(e), sel[c,l]] with values fp32[E, num_rel] and grad
 * fp32[num_rel, num_rows, dim_origin] as the forward's (both 16-B aligned).
 * The relations are summed per edge inside phase 1, which writes one staging
 * row per edge; phase 2 is the single-relation segmented sum.  algo
 * MAXK_BWD_STAGED (or AUTO): rows in CSC order, csc_pos = maxk_csc_build's;
 * MAXK_BWD_EDGE_GATHER: rows in edge order, csc_pos = the CSC slot -> edge
 * permutation (maxk_csc_perm_build).  Selectors are always the node CBSR
 * selectors here.  num_rel in {4, 8, 16}; dim_k in {8, 16, 32, 64};
 * dim_origin % 4 == 0.  Workspace: maxk_backward_workspace_bytes(algo, ...).
 * No counterpart in the reference (its proteins model makes one SSpMM call
 * per relation); equals the sum of num_rel maxk_sspmm_backward calls up to
 * fp32 summation order.  Writes every element of dxs. */
int maxk_sspmm_backward_multi(int algo, const int32_t *sched, int64_t num_panels,
                              const int32_t *indptr, const int32_t *indices, const float *values,
                              int num_rel, const float *grad, const uint8_t *cbsr_sel,
                              int num_rows, int num_cols, int64_t num_edges, int dim_origin,
                              int dim_k, float *dxs, const int32_t *csc_pos,
                              const int32_t *csc_sched, int64_t csc_num_panels,
                              const int32_t *csc_indptr, void *workspace, size_t workspace_bytes,
                              void *stream);

/* ---------------------------------------------------------------------------
 * Backward SSpMM, TILE algorithm (dim_k = 32 or 64, dim_origin = 256): every
 * gradient row is read once per CU into an LDS ring instead of being
 * gathered per edge; destinations' dXs live in registers.  Destinations are cut
 * into num_groups groups of group_size <= 2048 (k = 64: 1024) columns; the
 * (group, source row) space is cut into num_workgroups equal ranges, one per
 * workgroup (grid = num_workgroups), a range crossing a group boundary being
 * two or more PIECES run one after the other (csrc/tile_format.h; piece ids
 * 0 .. num_groups + num_workgroups - 2).  Inputs from the plan
 * (maxk_tile_plan_build below; format in csrc/maxk_spgemm.hip above
 * bwd_tile_kernel), one stream per (piece, wave) w = piece * 16 + wave: headers
 * int32[.., 4] from header_start[w] (16-B aligned), records int32[.., 2|4] from
 * record_start[w] (16-B aligned, padded by 4 KB); num_chunks int32[pieces];
 * zero_row: 1 KB of zeros (16-B aligned).  part: fp32[planes * num_cols *
 * dim_k] scratch, planes = maxk_tile_part_planes (NULL when 0): a group's
 * later pieces' partial sums, added into dxs in piece order.  Writes every
 * element of dxs; same result as the other algorithms up to fp32 summation
 * order (deterministic).
 * ------------------------------------------------------------------------- */
int maxk_sspmm_backward_tile(const void *headers, const int64_t *header_start,
                             const void *records, const int64_t *record_start,
                             const int32_t *num_chunks, int num_groups, int num_workgroups,
                             int group_size, const float *grad, const float *zero_row,
                             const uint8_t *cbsr_sel, int num_rows, int num_cols, int dim_origin,
                             int dim_k, float *dxs, float *part, void *stream);

/* TILE plan, built on the device (spgemm_new_amd/csrc/maxk_plan.hip; no
 * reference counterpart: the reference backward reuses the forward's .warp4
 * chunks, kernels/spmm_maxk_backward.cu:117-139).  CSR with indptr[0] == 0.
 *  maxk_tile_plan_shape: (num_groups, group_size, num_workgroups) for num_cus
 *    CUs -- groups of <= 2048 (k = 32) / 1024 (k = 64) destinations and S <= 8
 *    equal source ranges per group (num_workgroups = num_groups * S, one piece
 *    each, S <= num_rows) so that about one workgroup runs per CU; when the
 *    groups outnumber the CUs (S = 1), their count is rounded up to whole
 *    rounds of num_cus workgroups (smaller groups, no idle last round).  Any other
 *    num_workgroups <= num_groups * num_rows is valid (ranges straddling
 *    groups), measured slower on Reddit; more would leave empty workgroup
 *    ranges and is refused (MAXK_E_ARG) by the build and the backward.
 *  maxk_tile_plan_build: call once with headers == NULL (count call): writes
 *    sizes (host int64[3]) = {header entries, records, largest
 *    padded per-segment record count}; the plan is usable only if sizes[2] <=
 *    65535.  Then call with headers int32x4[sizes[0]], header_start
 *    int64[NP*16], records int32 x maxk_tile_record_words() each [sizes[1]],
 *    record_start int64[NP*16], num_chunks int32[NP] (NP = num_groups +
 *    num_workgroups - 1 pieces) and optionally edge_record int32[E] (the record of
 *    each CSR edge, for maxk_tile_plan_set_values).  Both calls synchronise
 *    the stream once.  Deterministic: records keep CSR order per segment.
 *  maxk_tile_plan_set_values: records' values := values (after the graph's
 *    edge values changed; the plan's structure does not depend on them). */
int maxk_tile_plan_shape(int num_rows, int num_cols, int num_cus, int dim_k, int *num_groups,
                         int *group_size, int *num_workgroups);
/* The plan format the library was built with (host out): LDS ring buffers and rows per
 * buffer (chunks hold rows - 1 source rows; the header stream leads by buffers - 1). */
int maxk_tile_format(int *num_buffers, int *buffer_rows);
/* int32 words per TILE record in this build (2 or 4; tile_format.h). */
int maxk_tile_record_words(void);
size_t maxk_tile_plan_workspace_bytes(int64_t num_edges, int num_groups, int num_workgroups);
/* Partial planes the backward needs (fp32[planes * num_cols * dim_k] `part`):
 * the most pieces any destination group spans, minus one. */
int maxk_tile_part_planes(int num_rows, int num_groups, int num_workgroups);
int maxk_tile_plan_build(const int32_t *indptr, const int32_t *indices, const float *values,
                         int num_rows, int num_cols, int64_t num_edges, int dim_k, int num_groups,
                         int group_size, int num_workgroups, void *headers, int64_t header_capacity,
                         int64_t *header_start, void *records, int64_t record_capacity,
                         int64_t *record_start, int32_t *num_chunks, int32_t *edge_record,
                         int64_t *sizes, void *workspace, size_t workspace_bytes, void *stream);
int maxk_tile_plan_set_values(const int32_t *edge_record, const float *values, int64_t num_edges,
                              void *records, void *stream);

/* ---------------------------------------------------------------------------
 * CBSR producer (MaxK top-k) and dense-gradient scatter.
 * Replace torch.topk in the CBSR producers (direct_kernel_interface.py:58-85,
 * kernels/spmm_bindings.cpp:163-184, utils/models.py:72) and the host scatter
 * loop of SpGEMMFunction.backward (utils/models.py:136-141).
 *   maxk_topk_cbsr: per row of x (num_rows x dim, row stride ld floats,
 *   dim <= 256) the k largest entries -> cbsr_data[r, j] = x[r, cbsr_sel[r, j]]
 *   (num_rows x k, fp32 / uint8).  NaN counts as the largest value, -0 == +0,
 *   ties at the k-th value go to the lower column.  order: COLUMN = ascending
 *   column, VALUE = descending value (torch.topk's sorted order), LANE = column
 *   ranks interleaved for the forward kernel's lane layout.  dense_out
 *   (nullable, num_rows x dim): the MaxK forward (selected kept, rest 0).
 *   maxk_cbsr_scatter: out[r, :] = 0 except out[r, cbsr_sel[r, j]] = vals[r, j].
 *   maxk_cbsr_mask: out[r, :] = 0 except out[r, c] = src[r, c] for c in
 *   cbsr_sel[r, :] (src, out: num_rows x dim) -- the MaxK backward.
 * ------------------------------------------------------------------------- */
#define MAXK_TOPK_ORDER_COLUMN 0
#define MAXK_TOPK_ORDER_VALUE 1
#define MAXK_TOPK_ORDER_LANE 2  /* column rank q at VEC*(q % LPE) + q/LPE: the forward's lane layout */
int maxk_topk_cbsr(const float *x, int num_rows, int dim, int64_t ld, int k, int order,
                   float *cbsr_data, uint8_t *cbsr_sel, float *dense_out, void *stream);
int maxk_cbsr_scatter(const float *vals, const uint8_t *cbsr_sel, int num_rows, int k, int dim,
                      float *out, void *stream);
int maxk_cbsr_mask(const float *src, const uint8_t *cbsr_sel, int num_rows, int k, int dim,
                   float *out, void *stream);

/* ---------------------------------------------------------------------------
 * Exact drop-ins for the reference's extern "C" launchers
 * (cuda_kernel_wrappers.cu:38-56 and :58-76), minus the CUDA launch geometry
 * (grid/block/shared_size), which the implementation chooses.  They consume
 * the reference's warp4 chunks and, like the reference, ACCUMULATE into the
 * caller's (normally zeroed, cuda_kernel_bindings.cpp:71,128) output.
 * Defects of the reference are not reproduced (SURVEY.md §2.4-1,-7).
 * ------------------------------------------------------------------------- */
int maxk_spmm_forward_warp4(const int32_t *warp4, const int32_t *idx, const float *val,
                            const float *vin_data, const uint8_t *vin_selector, float *vout,
                            int num_v, int num_e, int feat_in, int dim_sparse,
                            int num_warps, void *stream);
int maxk_spmm_backward_warp4(const int32_t *warp4, const int32_t *idx, const float *val,
                             const float *vin_data, const uint8_t *vin_selector, float *vout,
                             int num_v, int num_e, int feat_in, int dim_sparse,
                             int num_warps, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* MAXK_SPGEMM_H */
