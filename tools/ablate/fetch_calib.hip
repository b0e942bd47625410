// fetch_calib.hip -- calibrate rocprofv3 FETCH_SIZE against known byte counts for
// the access shapes the hot-path kernels use (development tool; run under
// rocprofv3 --pmc FETCH_SIZE).  The table (4 GiB) is far larger than the
// Infinity Cache and every 128-B line is touched at most once per launch, so
// every line read is one fabric fetch.
//   stream16 : streaming 16 B/lane (the guide's calibrated case: FETCH_SIZE = bytes / 2)
//   line16   : random lines, 8 lanes x 16 B each (the forward's CBSR data row)
//   piece32  : random lines, 8 lanes x 4 B = 32 B of the line (the selector row)
//   dword1   : random lines, 1 lane x 4 B (LOCAL's scattered G reads)
// Each launch touches N_LINES distinct lines (a permutation of the table's lines).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)
typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned long long line_of(unsigned long long i, unsigned long long nlines)
{
    return (i * 2654435761ull + 12345ull) % nlines;  // odd multiplier: a permutation when nlines is a power of 2
}

template <int MODE>
__global__ __launch_bounds__(256) void rd(const float *__restrict__ t, unsigned long long nlines,
                                          unsigned long long nuse, float *__restrict__ sink)
{
    const unsigned long long tid = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    float acc = 0.f;
    if constexpr (MODE == 0) {  // stream16
        for (unsigned long long i = tid; i < nuse * 8; i += stride) {
            const f4 v = reinterpret_cast<const f4 *>(t)[i];
            acc += v.x + v.y + v.z + v.w;
        }
    } else if constexpr (MODE == 1 || MODE == 2) {  // 8 lanes per line
        const unsigned sub = threadIdx.x & 7;
        for (unsigned long long i = tid; i < nuse * 8; i += stride) {
            const unsigned long long ln = line_of(i >> 3, nlines);
            if constexpr (MODE == 1) {
                const f4 v = reinterpret_cast<const f4 *>(t + ln * 32)[sub];
                acc += v.x + v.y + v.z + v.w;
            } else {
                acc += t[ln * 32 + sub];
            }
        }
    } else {  // one dword per line
        for (unsigned long long i = tid; i < nuse; i += stride) acc += t[line_of(i, nlines) * 32];
    }
    if (acc == 12345.678f) sink[0] = acc;
}

int main()
{
    const unsigned long long bytes = 4ull << 30, nlines = bytes / 128, nuse = nlines / 4;
    float *t, *sink;
    CK(hipMalloc(&t, bytes));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(t, 0, bytes));
    dim3 g(256 * 32), b(256);
    hipLaunchKernelGGL(rd<0>, g, b, 0, 0, t, nlines, nuse, sink);
    hipLaunchKernelGGL(rd<1>, g, b, 0, 0, t, nlines, nuse, sink);
    hipLaunchKernelGGL(rd<2>, g, b, 0, 0, t, nlines, nuse, sink);
    hipLaunchKernelGGL(rd<3>, g, b, 0, 0, t, nlines, nuse, sink);
    CK(hipDeviceSynchronize());
    printf("lines per launch %llu = %.3f GB of whole lines; stream16 reads the same bytes\n", nuse,
           nuse * 128.0 / 1e9);
    return 0;
}
