/*
 * maxk_variants.h -- entry points of the ABLATION build (libmaxk_variants.so,
 * tools/variants_lib): kernels that were built, tested bit-exact against the
 * product kernels and measured slower on every BASELINE shape,
 * so the product library (include/maxk_spgemm.h) no longer carries them.  The
 * ablation library is the product sources plus these; it exports the whole
 * product ABI as well.  Development and regression-test use only.
 */
#ifndef MAXK_VARIANTS_H
#define MAXK_VARIANTS_H

#include "../../include/maxk_spgemm.h"

#ifdef __cplusplus
extern "C" {
#endif

/* The same with each output optional (NULL: not written; cbsr_data may be NULL
 * when out_data is) plus out_packed uint16[num_rows, dim_k]: the reordered
 * selector | its ORIGINAL entry index << 8 -- the input of
 * maxk_sspmm_backward_multi_banked. */
int maxk_cbsr_bank_order_ex(const float *cbsr_data, const uint8_t *cbsr_sel, int num_rows,
                            int dim_k, int num_rel, float *out_data, uint8_t *out_sel,
                            uint16_t *out_packed, void *stream);

/* Register-accumulator form of the fused forward for num_rel = 8, dim_origin =
 * 256, dim_k in {4, 8, 16, 32} (the proteins shape): each destination row's 8 x
 * 256 sums stay in registers and an edge's CBSR values reach them by a gather
 * over the source's column bitmask.  Needs the CBSR in the form
 * maxk_cbsr_colmask writes: sorted_data fp32[V, k] (each row's values in
 * ascending column order) and mask_rec uint32[V, 16] (per 32-column word: the
 * bitmask of selected columns, then the number selected below it; 8-B aligned).
 * Same result as maxk_spgemm_forward_multi -- bit for bit at dim_k = 32 (both
 * add each element's contributions in edge order; at smaller k that kernel
 * sums per-edge-slot copies, another fp32 order) -- same schedule and
 * workspace size. */
int maxk_cbsr_colmask(const float *cbsr_data, const uint8_t *cbsr_sel, int num_rows, int dim_k,
                      float *sorted_data, uint32_t *mask_rec, void *stream);
int maxk_spgemm_forward_multi_gather(const int32_t *sched, int64_t num_panels,
                                     const int32_t *indptr, const int32_t *indices,
                                     const float *values, int num_rel, const float *sorted_data,
                                     const uint32_t *mask_rec, int num_rows, int dim_origin,
                                     int dim_k, float *out, void *workspace,
                                     size_t workspace_bytes, void *stream);

#define MAXK_BWD_BINNED 7      /* destination bins summed in LDS (maxk_sspmm_backward_binned,
                                  node selectors); not accepted by maxk_sspmm_backward */
#define MAXK_BWD_BINNED_EDGE 8 /* BINNED reading edge selectors (as STAGED_EDGE) */

/* The same for num_rel = 8, dim_k = 32 with bank-ordered selectors
 * (sel_banked = maxk_cbsr_bank_order_ex's out_packed of cbsr_sel, R = 8): phase
 * 1 reads one edge per wave-instruction, lane 2p + q the quad q of its p-th
 * column, so LDS reads of a 16-lane group cover 8 columns the bank order made
 * distinct mod 8; products are stored at the columns' original entries.  Same
 * FMAs in the same order as maxk_sspmm_backward_multi: the same bits. */
int maxk_sspmm_backward_multi_banked(int algo, const int32_t *sched, int64_t num_panels,
                                     const int32_t *indptr, const int32_t *indices,
                                     const float *values, int num_rel, const float *grad,
                                     const uint16_t *sel_banked, int num_rows, int num_cols,
                                     int64_t num_edges, int dim_origin, int dim_k, float *dxs,
                                     const int32_t *csc_pos, const int32_t *csc_sched,
                                     int64_t csc_num_panels, const int32_t *csc_indptr,
                                     void *workspace, size_t workspace_bytes, void *stream);

/* The same with phase 1 in register form (num_rel = 8, dim_origin = 256, dim_k
 * in {8, 16, 32}): the source row's 8 gradient rows in registers, per edge the
 * relations folded for every column and the selected ones fetched by lane
 * permutes -- the same FMAs in the same order, so the same bits; same
 * arguments, workspace and phase 2. */
int maxk_sspmm_backward_multi_gather(int algo, const int32_t *sched, int64_t num_panels,
                                     const int32_t *indptr, const int32_t *indices,
                                     const float *values, int num_rel, const float *grad,
                                     const uint8_t *cbsr_sel, int num_rows, int num_cols,
                                     int64_t num_edges, int dim_origin, int dim_k, float *dxs,
                                     const int32_t *csc_pos, const int32_t *csc_sched,
                                     int64_t csc_num_panels, const int32_t *csc_indptr,
                                     void *workspace, size_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------------------
 * Backward SSpMM, BINNED algorithm (propagation blocking; no counterpart in the
 * reference, whose backward scatters with atomics, spmm_maxk_backward.cu:
 * 86-112).  Phase 1 pushes over the CSR panels (sched, as the forward and
 * STAGED) and writes each edge's k products, unpadded, to slot bin_pos[e] of
 * destination bin idx[e] / MAXK_BIN_DESTS; phase 2 sums every bin in LDS (one
 * wave per bin) and stores its rows of dxs.  Versus STAGED it writes k*4 B
 * instead of a 64-B row per edge at k = 8, in streams its XCD's L2 completes
 * line by line, and replaces the segmented sum's CSC panels by one pass.
 * dim_k in {8, 16, 32}; sel = node CBSR selectors, or edge selectors (uint8
 * [E, k] from maxk_spgemm_forward_esel) when edge_selectors != 0.
 * Deterministic (the slot order is fixed by the plan).  Workspace:
 * maxk_backward_binned_workspace_bytes(num_slots, dim_k) (the products).
 *  maxk_bin_plan_build: bins of MAXK_BIN_DESTS destinations; a bin's slots hold
 *    its in-edges ordered by (XCD of the panel's workgroup, edge), packed
 *    first-fit into windows of 64 slots with distinct destinations (at most 8
 *    windows open; padding slots have bin_dst 0xFF).  Count call
 *    (bin_pos == NULL): writes *num_slots (host) and synchronises; fill call:
 *    bin_pos int32[E], bin_ptr int32[num_bins + 1] (slot offsets, multiples of
 *    64), bin_dst uint8[num_slots].  The plan is tied to `sched` (the XCD
 *    order follows its panels).  num_bins = ceil(num_cols / MAXK_BIN_DESTS).
 * ------------------------------------------------------------------------- */
#define MAXK_BIN_DESTS 255
#define MAXK_BIN_WINDOW 64
size_t maxk_bin_plan_workspace_bytes(int64_t num_edges, int num_cols);
int maxk_bin_plan_build(const int32_t *sched, int64_t num_panels, const int32_t *indices,
                        int64_t num_edges, int num_cols, int32_t *bin_pos, int32_t *bin_ptr,
                        uint8_t *bin_dst, int64_t slot_capacity, int64_t *num_slots,
                        void *workspace, size_t workspace_bytes, void *stream);
size_t maxk_backward_binned_workspace_bytes(int64_t num_slots, int dim_k);
int maxk_sspmm_backward_binned(const int32_t *sched, int64_t num_panels, const int32_t *indptr,
                               const int32_t *indices, const float *values, const float *grad,
                               const uint8_t *sel, int edge_selectors, int num_rows, int num_cols,
                               int64_t num_edges, int dim_origin, int dim_k, float *dxs,
                               const int32_t *bin_pos, const int32_t *bin_ptr,
                               const uint8_t *bin_dst, int num_bins, int64_t num_slots,
                               void *workspace, size_t workspace_bytes, void *stream);


#ifdef __cplusplus
}
#endif

#endif
