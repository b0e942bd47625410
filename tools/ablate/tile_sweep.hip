// tile_sweep.hip -- floor of a source-tiled backward (development tool).
// Every workgroup (1024 threads, one per CU) sweeps the gradient rows of its
// source split into an LDS ring by LDS-DMA (global_load_lds_dwordx4, one 1 KB
// row per wave-instruction), one barrier per chunk, and touches each staged row
// with one ds_read per lane.  Measures what the staging alone costs: the floor
// of a backward that reads each G row once per CU instead of gathering per edge.
//   tile_sweep <rows> <splits> <buffers> <chunk_rows> [reps]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

__device__ __forceinline__ void glds16(const float *g, unsigned lds_byte)
{
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(__builtin_amdgcn_readfirstlane(lds_byte)) : "memory");
}

template <int NB, int PER>  // PER = rows per wave per chunk (chunk = 16 * PER rows)
__global__ __launch_bounds__(1024) void sweep(const float *__restrict__ G, int rows, int splits,
                                              float *__restrict__ sink)
{
    extern __shared__ float lds[];
    constexpr int CH = 16 * PER;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int split = blockIdx.x % splits;
    const int r0 = (int)((long long)split * rows / splits), r1 = (int)((long long)(split + 1) * rows / splits);
    const int nch = (r1 - r0) / CH;  // whole chunks only
    auto issue = [&](int c) {
        if (c >= nch) return;
        const unsigned buf = (unsigned)(c % NB) * CH * 1024u;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int rr = w * PER + i;
            glds16(G + (size_t)(r0 + c * CH + rr) * 256 + lane * 4, buf + rr * 1024u);
        }
    };
    for (int c = 0; c < NB - 1; ++c) issue(c);
    float acc = 0.f;
    for (int c = 0; c < nch; ++c) {
        // chunk c landed (this wave's pieces): at most NB-2 later chunks in flight
        if (NB == 2) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        else if (NB == 3) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" :: "i"(PER) : "memory");
        else asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" :: "i"(2 * PER) : "memory");
        issue(c + NB - 1);
        const float *b = lds + (size_t)(c % NB) * CH * 256;
#pragma unroll
        for (int i = 0; i < 4; ++i) acc += b[((lane * 37 + i * 11 + w) % CH) * 256 + lane * 4];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (acc == 12345.f) sink[threadIdx.x] = acc;
}

int main(int argc, char **argv)
{
    const int rows = argc > 1 ? atoi(argv[1]) : 232965;
    const int splits = argc > 2 ? atoi(argv[2]) : 2;
    const int nb = argc > 3 ? atoi(argv[3]) : 2;
    const int per = argc > 4 ? atoi(argv[4]) : 3;
    const int reps = argc > 5 ? atoi(argv[5]) : 10;
    const int grid = argc > 6 ? atoi(argv[6]) : 256;
    float *G, *sink;
    CK(hipMalloc(&G, (size_t)rows * 1024));
    CK(hipMemset(G, 0, (size_t)rows * 1024));
    CK(hipMalloc(&sink, 4096 * 4));
    const size_t lds = (size_t)nb * 16 * per * 1024;
    if (lds > 160 * 1024) { printf("lds %zu too big\n", lds); return 1; }
    auto launch = [&]() {
#define L(NB, P) hipLaunchKernelGGL((sweep<NB, P>), dim3(grid), dim3(1024), lds, 0, G, rows, splits, sink)
        if (nb == 2 && per == 3) L(2, 3);
        else if (nb == 2 && per == 4) L(2, 4);
        else if (nb == 3 && per == 2) L(3, 2);
        else if (nb == 3 && per == 3) L(3, 3);
        else if (nb == 4 && per == 2) L(4, 2);
        else if (nb == 4 && per == 1) L(4, 1);
        else if (nb == 2 && per == 2) L(2, 2);
        else { printf("unsupported\n"); exit(1); }
#undef L
    };
    launch();
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    const int ch = 16 * per;
    const double per_wg = (double)((rows / splits) / ch) * ch * 1024;
    printf("rows %d splits %d buffers %d chunk %d grid %d: %.3f ms, %.1f GB/s per CU, %.2f TB/s chip\n", rows,
           splits, nb, ch, grid, ms, per_wg / ms / 1e6, per_wg * grid / ms / 1e9);
    return 0;
}
