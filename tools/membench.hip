// membench.hip -- streaming microbenchmark for the SC decode's HBM access pattern (tooling only).
// Each wave processes 64-codeword tiles of 64 fp32 words (16 KiB read, optional 8 KiB write), the
// same addressing as sc_fast_kernel<64>.  Prints GB/s for several wave/workgroup geometries.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#pragma clang diagnostic ignored "-Wunused-result"

typedef float f4 __attribute__((ext_vector_type(4)));

template <int WPG, bool STORE, int UNROLL, bool ILV = false>
__global__ __launch_bounds__(64 * WPG) void stream_kernel(const f4* __restrict__ y, f4* __restrict__ out, long ntiles,
                                                           float* sink) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    f4 acc = {0, 0, 0, 0};
    // ILV: adjacent tiles go to consecutive workgroups (round-robin over XCDs) instead of one workgroup's waves
    const long t0 = ILV ? (long)wave * gridDim.x + blockIdx.x : (long)blockIdx.x * WPG + wave;
    for (long t = t0; t < ntiles; t += (long)gridDim.x * WPG) {
        f4 v[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) v[q] = y[t * 1024 + lane + 64 * q];
#pragma unroll
        for (int q = 0; q < 16; ++q) acc += v[q];
        if (STORE) {
#pragma unroll
            for (int q = 0; q < 8; ++q) out[t * 512 + lane + 64 * q] = acc + (float)q;
        }
    }
    if (acc.x == 123.456f) sink[0] = acc.y;
}

template <int WPG, bool STORE, bool ILV = false>
static void run(f4** ys, f4** outs, long ntiles, float* sink, int cus, int per_cu, const char* name) {
    int grid = cus * per_cu / WPG;
    if (grid < 1) grid = 1;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int w = 0; w < 2; ++w) hipLaunchKernelGGL((stream_kernel<WPG, STORE, 1, ILV>), dim3(grid), dim3(64 * WPG), 0, 0, ys[w % 5], outs[w % 5], ntiles, sink);
    hipEventRecord(a);
    const int it = 10;
    for (int i = 0; i < it; ++i)
        hipLaunchKernelGGL((stream_kernel<WPG, STORE, 1, ILV>), dim3(grid), dim3(64 * WPG), 0, 0, ys[i % 5], outs[i % 5], ntiles, sink);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    ms /= it;
    double bytes = (double)ntiles * (16384 + (STORE ? 8192 : 0));
    printf("%-28s waves/CU=%2d  %8.3f ms  %7.1f GB/s\n", name, per_cu, ms, bytes / ms / 1e6);
}

int main() {
    const long ntiles = 1L << 14;  // 2^20 codewords x 64 fp32 = 256 MiB
    f4 *ys[5], *outs[5];
    float* sink;
    for (int i = 0; i < 5; ++i) {
        (void)hipMalloc(&ys[i], ntiles * 16384);
        (void)hipMalloc(&outs[i], ntiles * 8192);
        (void)hipMemset(ys[i], 0x11, ntiles * 16384);
    }
    (void)hipMalloc(&sink, 64);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    printf("CUs = %d\n", cus);
    for (int per_cu : {2, 4, 8, 16, 32}) {
        run<1, false>(ys, outs, ntiles, sink, cus, per_cu, "1-wave WG, read");
        run<4, false>(ys, outs, ntiles, sink, cus, per_cu, "4-wave WG, read");
        run<1, true>(ys, outs, ntiles, sink, cus, per_cu, "1-wave WG, read+write");
        run<4, true>(ys, outs, ntiles, sink, cus, per_cu, "4-wave WG, read+write");
        run<8, false>(ys, outs, ntiles, sink, cus, per_cu, "8-wave WG, read");
        run<8, true>(ys, outs, ntiles, sink, cus, per_cu, "8-wave WG, read+write");
        run<8, false, true>(ys, outs, ntiles, sink, cus, per_cu, "8-wave WG ilv, read");
        run<8, true, true>(ys, outs, ntiles, sink, cus, per_cu, "8-wave WG ilv, read+write");
    }
    return 0;
}
