// gather_rate.hip -- the ceiling of the forward's access pattern: random whole
// records of R bytes from a table of T bytes, one record per (edge) index
// streamed from HBM, every record used once per index.  Development tool, not
// product code (the forward's pattern roofline).
//
// Each wave takes 64 consecutive indices per step; R/16 lanes read one record
// (16 B per lane), so a wave-instruction covers 64*16/R records; U steps in
// flight.  The sum of everything read goes to one float per wave (so nothing is
// optimised away).  Prints the record-byte rate (records * R / time) and the
// index-inclusive rate.
//
// usage: gather_rate <record_bytes 16..256> <table_MB> <num_indices_M> [reps]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

template <int R>
__global__ __launch_bounds__(256) void gather(const f4 *__restrict__ table, const int *__restrict__ idx,
                                              long n, float *__restrict__ out)
{
    constexpr int LPR = R / 16;          // lanes per record
    constexpr int RPI = 64 / LPR;        // records per wave-instruction
    constexpr int U = 8;
    const int lane = threadIdx.x & 63;
    const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const long waves = ((long)gridDim.x * blockDim.x) >> 6;
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    for (long base = wave * RPI * U; base < n; base += waves * RPI * U) {
        f4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long i = base + (long)u * RPI + lane / LPR;
            const int r = i < n ? __builtin_nontemporal_load(idx + i) : 0;
            v[u] = table[(long)r * LPR + lane % LPR];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u];
    }
    const float s = acc.x + acc.y + acc.z + acc.w;
    if (s == 12345.678f) out[wave] = s;   // practically never: keeps the loads
}

template <int R>
double run(long rows, long n, int reps)
{
    f4 *table;
    int *idx;
    float *out;
    CK(hipMalloc(&table, rows * R));
    CK(hipMemset(table, 0, rows * R));
    CK(hipMalloc(&idx, n * sizeof(int)));
    CK(hipMalloc(&out, 1 << 24));
    std::vector<int> h(n);
    unsigned x = 12345u;
    for (long i = 0; i < n; ++i) {
        x = x * 1664525u + 1013904223u;
        h[i] = (int)(((unsigned long long)x * (unsigned long long)rows) >> 32);
    }
    CK(hipMemcpy(idx, h.data(), n * sizeof(int), hipMemcpyHostToDevice));
    const int blocks = 256 * 8;   // 8 workgroups of 4 waves per CU
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    gather<R><<<blocks, 256>>>(table, idx, n, out);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) gather<R><<<blocks, 256>>>(table, idx, n, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipFree(table));
    CK(hipFree(idx));
    CK(hipFree(out));
    return ms / reps;
}

int main(int argc, char **argv)
{
    if (argc < 4) {
        printf("usage: %s record_bytes table_MB num_indices_M [reps]\n", argv[0]);
        return 2;
    }
    const int R = atoi(argv[1]);
    const double tmb = atof(argv[2]);
    const long n = (long)(atof(argv[3]) * 1e6);
    const int reps = argc > 4 ? atoi(argv[4]) : 10;
    const long rows = (long)(tmb * 1e6 / R);
    double ms;
    switch (R) {
    case 32: ms = run<32>(rows, n, reps); break;
    case 64: ms = run<64>(rows, n, reps); break;
    case 128: ms = run<128>(rows, n, reps); break;
    case 256: ms = run<256>(rows, n, reps); break;
    default: printf("record_bytes must be 32, 64, 128 or 256\n"); return 2;
    }
    printf("R=%d B table=%.0f MB n=%ld: %.3f ms  records %.2f TB/s  (+indices %.2f TB/s)\n", R,
           rows * (double)R / 1e6, n, ms, n * (double)R / ms / 1e9, n * (R + 4.0) / ms / 1e9);
    return 0;
}
