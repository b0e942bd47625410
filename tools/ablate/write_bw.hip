// write_bw.hip -- HBM store bandwidth by store form (development tool).
// Writes N bytes (default 14.7 GB, the STAGED staging rows at Reddit k=32).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)
typedef float f4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256) void wr(float *__restrict__ p, size_t n4, unsigned rows128)
{
    const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    const f4 v = f4{1.f, 2.f, 3.f, (float)threadIdx.x};
    if constexpr (MODE <= 2) {       // sequential 16 B per lane
        for (size_t i = tid; i < n4; i += stride) {
            f4 *q = reinterpret_cast<f4 *>(p) + i;
            if constexpr (MODE == 0) *q = v;
            else if constexpr (MODE == 1) __builtin_nontemporal_store(v, q);
            else { __hip_atomic_store(reinterpret_cast<float *>(q), v.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
        }
    } else if constexpr (MODE == 3) {  // sequential 4 B per lane (dword)
        for (size_t i = tid; i < n4 * 4; i += stride) p[i] = (float)i;
    } else {                           // scattered 128-B rows, 8 lanes x 16 B per row
        const unsigned lane = threadIdx.x & 63, sub = lane & 7;
        for (size_t i = tid; i < n4; i += stride) {
            const size_t rowi = i >> 3;
            const size_t row = (rowi * 2654435761ull) % rows128;
            f4 *q = reinterpret_cast<f4 *>(p + row * 32) + sub;
            if constexpr (MODE == 4) *q = v;
            else __builtin_nontemporal_store(v, q);
        }
    }
}

template <int MODE>
float run(float *p, size_t bytes, int reps)
{
    const size_t n4 = bytes / 16;
    const unsigned rows = (unsigned)(bytes / 128);
    dim3 g(256 * 16), b(256);
    hipLaunchKernelGGL(wr<MODE>, g, b, 0, 0, p, n4, rows);
    CK(hipDeviceSynchronize());
    hipEvent_t a, e;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&e));
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(wr<MODE>, g, b, 0, 0, p, n4, rows);
    CK(hipEventRecord(e));
    CK(hipEventSynchronize(e));
    float ms;
    CK(hipEventElapsedTime(&ms, a, e));
    return ms / reps;
}

int main(int argc, char **argv)
{
    const size_t bytes = argc > 1 ? (size_t)atoll(argv[1]) : (size_t)14670000000ull;
    float *p;
    CK(hipMalloc(&p, bytes));
    const char *names[] = {"seq dwordx4 plain", "seq dwordx4 nt", "seq dword atomic-store(agent)",
                           "seq dword plain", "scattered 128B rows plain", "scattered 128B rows nt"};
    float t[6] = {run<0>(p, bytes, 3), run<1>(p, bytes, 3), run<2>(p, bytes / 4, 3),
                  run<3>(p, bytes, 3), run<4>(p, bytes, 3), run<5>(p, bytes, 3)};
    for (int i = 0; i < 6; ++i) {
        const double b = (i == 2) ? bytes / 16.0 : (double)bytes;
        printf("%-32s %8.3f ms  %7.0f GB/s\n", names[i], t[i], b / t[i] / 1e6);
    }
    return 0;
}
