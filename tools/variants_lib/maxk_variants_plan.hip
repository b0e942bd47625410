// maxk_variants_plan.hip -- the ablation build's plan builders: the product
// plan builders (spgemm_new_amd/csrc/maxk_plan.hip) plus the BINNED backward's
// bin plan (maxk_bin_plan_build; round 3, measured slower than STAGED /
// EDGE_GATHER at every k).
#include "../../spgemm_new_amd/csrc/maxk_plan.hip"
#include "maxk_variants.h"

// --------------------------------------------------------------- BINNED
// The BINNED backward's phase 1 launches 4 waves (panels) per workgroup and
// the hardware deals workgroups to the 8 XCDs round-robin, so panel w runs on
// XCD (w / 4) % 8 (cdna_hip_programming.md, XCD dispatch).  A bin's slots are
// ordered by that XCD first, so each 128-B line of a bin is written by one
// XCD's L2.  (A wrong guess costs only line merging, never correctness.)
constexpr int kBinPanelWaves = 4;   // kWavesPerBlock of maxk_spgemm.hip
constexpr int kBinXcds = 8;
constexpr int kBinOpen = 8;         // windows open at once while packing

// key[e] = bin(idx[e]) * 8 + XCD of e's panel (last panel starting at or
// before e: panels with no edges share their start with the next one)
__global__ void bin_keys_kernel(const int2 *__restrict__ sched, int64_t num_panels,
                                const int32_t *__restrict__ indices, int64_t num_edges,
                                int32_t *__restrict__ key)
{
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= num_edges) return;
    int64_t lo = 0, hi = num_panels;   // first w with sched[w].y > e
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (sched[mid].y <= e) lo = mid + 1; else hi = mid;
    }
    const int64_t w = lo - 1;
    const int xcd = (int)((w / kBinPanelWaves) % kBinXcds);
    key[e] = (indices[e] / MAXK_BIN_DESTS) * kBinXcds + xcd;
}

// start[b] = first sorted slot of bin b (b in [0, nbins])
__global__ void bin_bounds_kernel(const int32_t *__restrict__ keys_sorted, int64_t n, int nbins,
                                  int32_t *__restrict__ start)
{
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b <= nbins) start[b] = (int32_t)lower_bound(keys_sorted, n, b * kBinXcds);
}

// destination within its bin, in sorted order
__global__ void bin_dloc_kernel(const int32_t *__restrict__ keys_sorted,
                                const int32_t *__restrict__ order,
                                const int32_t *__restrict__ indices, int64_t n,
                                uint8_t *__restrict__ dloc)
{
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q < n)
        dloc[q] = (uint8_t)(indices[order[q]] - (keys_sorted[q] / kBinXcds) * MAXK_BIN_DESTS);
}

// One thread per bin: first-fit packing of the bin's in-edges (sorted order)
// into windows of 64 slots with distinct destinations, at most kBinOpen open
// (the oldest is closed, padded, when a record fits none).  Windows are
// numbered in opening order.  FILL = false: nwin[b] = windows used; FILL: the
// slots (bin_pos of each edge, bin_dst of each slot).
template <bool FILL>
__global__ void bin_pack_kernel(const int32_t *__restrict__ start, int nbins,
                                const uint8_t *__restrict__ dloc, const int32_t *__restrict__ order,
                                int32_t *__restrict__ nwin, const int32_t *__restrict__ bin_ptr,
                                int32_t *__restrict__ bin_pos, uint8_t *__restrict__ bin_dst)
{
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nbins) return;
    uint64_t m[kBinOpen][4];
    int fill[kBinOpen], wid[kBinOpen];
    int nopen = 0, next = 0;
    const int base = FILL ? bin_ptr[b] : 0;
    for (int q = start[b]; q < start[b + 1]; ++q) {
        const int d = dloc[q];
        const uint64_t bit = uint64_t(1) << (d & 63);
        int i = 0;
        while (i < nopen && (m[i][d >> 6] & bit)) ++i;
        if (i == nopen) {
            if (nopen == kBinOpen) {        // close the oldest window (padded)
                for (int j = 0; j + 1 < kBinOpen; ++j) {
                    for (int t = 0; t < 4; ++t) m[j][t] = m[j + 1][t];
                    fill[j] = fill[j + 1];
                    wid[j] = wid[j + 1];
                }
                --nopen;
            }
            i = nopen++;
            for (int t = 0; t < 4; ++t) m[i][t] = 0;
            fill[i] = 0;
            wid[i] = next++;
        }
        if (FILL) {
            const int slot = base + wid[i] * MAXK_BIN_WINDOW + fill[i];
            bin_pos[order[q]] = slot;
            bin_dst[slot] = (uint8_t)d;
        }
        m[i][d >> 6] |= bit;
        if (++fill[i] == MAXK_BIN_WINDOW) {  // full: close it
            for (int j = i; j + 1 < nopen; ++j) {
                for (int t = 0; t < 4; ++t) m[j][t] = m[j + 1][t];
                fill[j] = fill[j + 1];
                wid[j] = wid[j + 1];
            }
            --nopen;
        }
    }
    if (!FILL) nwin[b] = next;
}

__global__ void bin_ptr_kernel(const int32_t *__restrict__ win_start, int nbins,
                               int32_t *__restrict__ bin_ptr)
{
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b <= nbins) bin_ptr[b] = win_start[b] * MAXK_BIN_WINDOW;
}

extern "C" {

static int bin_count(int num_cols) { return (num_cols + MAXK_BIN_DESTS - 1) / MAXK_BIN_DESTS; }

size_t maxk_bin_plan_workspace_bytes(int64_t num_edges, int num_cols)
{
    if (num_edges < 0 || num_edges > INT32_MAX || num_cols < 1) return 0;
    const int64_t nb = bin_count(num_cols);
    const size_t tb = sort_temp_bytes(num_edges, bits_for(nb * kBinXcds));
    const size_t sb = scan_temp_bytes(nb + 1);
    return align_up((size_t)num_edges * 4, 256) * 3 + align_up((size_t)num_edges, 256) +
           align_up((size_t)(nb + 1) * 4, 256) * 3 + align_up(tb > sb ? tb : sb, 256) + 256;
}

int maxk_bin_plan_build(const int32_t *sched, int64_t num_panels, const int32_t *indices,
                        int64_t num_edges, int num_cols, int32_t *bin_pos, int32_t *bin_ptr,
                        uint8_t *bin_dst, int64_t slot_capacity, int64_t *num_slots,
                        void *workspace, size_t workspace_bytes, void *stream)
{
    if (!sched || num_panels < 1 || num_edges < 1 || num_edges > INT32_MAX || num_cols < 1 ||
        !indices || !num_slots)
        return MAXK_E_ARG;
    const bool fill = bin_pos != nullptr;
    if (fill && (!bin_ptr || !bin_dst)) return MAXK_E_ARG;
    if (!workspace || workspace_bytes < maxk_bin_plan_workspace_bytes(num_edges, num_cols))
        return MAXK_E_WORKSPACE;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const int nb = bin_count(num_cols);
    const int64_t E = num_edges;
    char *p = static_cast<char *>(workspace);
    int32_t *key = carve<int32_t>(p, E);
    int32_t *keys_sorted = carve<int32_t>(p, E);
    int32_t *order = carve<int32_t>(p, E);
    uint8_t *dloc = carve<uint8_t>(p, E);
    int32_t *start = carve<int32_t>(p, nb + 1);
    int32_t *nwin = carve<int32_t>(p, nb + 1);
    int32_t *win_start = carve<int32_t>(p, nb + 1);
    const unsigned bits = bits_for((int64_t)nb * kBinXcds);
    size_t tb = sort_temp_bytes(E, bits);
    const size_t sb = scan_temp_bytes(nb + 1);
    hipLaunchKernelGGL(bin_keys_kernel, dim3((unsigned)blocks_for(E)), dim3(kThreads), 0, st,
                       reinterpret_cast<const int2 *>(sched), num_panels, indices, E, key);
    int rc = launch_status();
    if (rc) return rc;
    rocprim::counting_iterator<int32_t> iota(0);
    hipError_t e = rocprim::radix_sort_pairs(p, tb, key, keys_sorted, iota, order, (size_t)E, 0u,
                                             bits, st);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(bin_bounds_kernel, dim3((unsigned)blocks_for(nb + 1)), dim3(kThreads), 0, st,
                       keys_sorted, E, nb, start);
    hipLaunchKernelGGL(bin_dloc_kernel, dim3((unsigned)blocks_for(E)), dim3(kThreads), 0, st,
                       keys_sorted, order, indices, E, dloc);
    hipLaunchKernelGGL(bin_pack_kernel<false>, dim3((unsigned)blocks_for(nb)), dim3(kThreads), 0,
                       st, start, nb, dloc, order, nwin, (const int32_t *)nullptr,
                       (int32_t *)nullptr, (uint8_t *)nullptr);
    if ((rc = launch_status())) return rc;
    size_t sbytes = sb;
    e = rocprim::exclusive_scan(p, sbytes, nwin, win_start, 0, (size_t)nb + 1,
                                rocprim::plus<int32_t>(), st);
    if (e != hipSuccess) return (int)e;
    int32_t total_windows = 0;
    e = hipMemcpyAsync(&total_windows, win_start + nb, sizeof(int32_t), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return (int)e;
    const int64_t slots = (int64_t)total_windows * MAXK_BIN_WINDOW;
    *num_slots = slots;
    if (slots > INT32_MAX) return MAXK_E_ARG;
    if (!fill) return MAXK_OK;
    if (slot_capacity < slots) return MAXK_E_WORKSPACE;
    hipLaunchKernelGGL(bin_ptr_kernel, dim3((unsigned)blocks_for(nb + 1)), dim3(kThreads), 0, st,
                       win_start, nb, bin_ptr);
    if ((rc = launch_status())) return rc;
    e = hipMemsetAsync(bin_dst, 0xFF, (size_t)slots, st);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(bin_pack_kernel<true>, dim3((unsigned)blocks_for(nb)), dim3(kThreads), 0, st,
                       start, nb, dloc, order, nwin, bin_ptr, bin_pos, bin_dst);
    return launch_status();
}

}  // extern "C"
