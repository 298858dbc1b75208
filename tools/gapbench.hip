// Cost model for filling the issue gaps of v_mfma_f32_16x16x32_f16 with VALU work (the fp16x3 GRU kernel's problem:
// 216 MFMAs and ~3k cycles of gate / split VALU per 16-codeword wave-step).  Each case runs 16 MFMAs per iteration on
// 4 independent accumulators with the same filler group after every MFMA, in program order (inline asm), at one and at
// two waves per SIMD.  Prints ns per MFMA per SIMD and the equivalent cycles at the clock of the MFMA-only case
// (16 cycles per MFMA by the guide's back-to-back row).
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/gapbench tools/gapbench.hip && tools/bin/gapbench
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef _Float16 hf8 __attribute__((ext_vector_type(8)));

#define MF(acc) asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(acc) : "v"(A), "v"(Bm))
#define EXP(k) asm volatile("v_exp_f32 %0, %1" : "=v"(x[k]) : "v"(y[k]))
#define RCP(k) asm volatile("v_rcp_f32 %0, %1" : "=v"(x[k]) : "v"(y[k]))
#define ADD(k) asm volatile("v_add_f32 %0, %1, %2" : "=v"(x[k]) : "v"(y[k]), "v"(y[(k) + 1]))
#define FMA(k) asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(x[k]) : "v"(y[k]), "v"(y[(k) + 1]), "v"(y[(k) + 2]))
#define PKF(k) asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(p[k]) : "v"(q[k]), "v"(q[(k) + 1]), "v"(q[(k) + 2]))
#define PKA(k) asm volatile("v_pk_add_f32 %0, %1, %2" : "=v"(p[k]) : "v"(q[k]), "v"(q[(k) + 1]))
#define CVT(k) asm volatile("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(u[k]) : "v"(y[k]), "v"(y[(k) + 1]))
// dependent chain on one register: exp -> add -> rcp -> fma, the GRU gate's shape
#define DEXP asm volatile("v_exp_f32 %0, %0" : "+v"(d))
#define DADD asm volatile("v_add_f32 %0, 1.0, %0" : "+v"(d))
#define DRCP asm volatile("v_rcp_f32 %0, %0" : "+v"(d))

// filler group after each MFMA, by case
template <int C>
__device__ __forceinline__ void fill(float (&x)[8], const float (&y)[12], f2 (&p)[4], const f2 (&q)[8],
                                     unsigned (&u)[4], float& d, int g) {
    const int k = g & 3;
    (void)k;
    if constexpr (C == 0) {
    } else if constexpr (C == 1) { EXP(0);
    } else if constexpr (C == 2) { EXP(0); EXP(1);
    } else if constexpr (C == 3) { ADD(0);
    } else if constexpr (C == 4) { ADD(0); ADD(1);
    } else if constexpr (C == 5) { ADD(0); ADD(1); ADD(2);
    } else if constexpr (C == 6) { ADD(0); ADD(1); ADD(2); ADD(3);
    } else if constexpr (C == 7) { EXP(0); ADD(1);
    } else if constexpr (C == 8) { EXP(0); ADD(1); ADD(2);
    } else if constexpr (C == 9) { EXP(0); RCP(1); ADD(2); ADD(3);
    } else if constexpr (C == 10) { PKF(0);
    } else if constexpr (C == 11) { FMA(0); FMA(1);
    } else if constexpr (C == 12) { PKA(0);
    } else if constexpr (C == 13) { CVT(0);
    } else if constexpr (C == 14) { DEXP;
    } else if constexpr (C == 15) { DADD; DRCP;
    } else if constexpr (C == 16) { DEXP; DADD; DRCP;
    } else if constexpr (C == 17) { EXP(0); EXP(1); ADD(2); ADD(3);
    } else if constexpr (C == 18) { EXP(0); RCP(1); EXP(2); ADD(3); ADD(4); FMA(5);
    }
}

template <int C>
__global__ __launch_bounds__(512) void kern(float* out, int iters) {
    const int lane = threadIdx.x;
    const float a = out[lane] + 1.0f;
    hf8 A, Bm;
    for (int j = 0; j < 8; ++j) {
        A[j] = (_Float16)(a * 0.01f + j);
        Bm[j] = (_Float16)(a * 0.02f - j);
    }
    f4 acc[4];
    for (int t = 0; t < 4; ++t) acc[t] = f4{0.f, 0.f, 0.f, 0.f};
    float x[8], y[12];
    f2 p[4], q[8];
    unsigned u[4];
    float d = a * 1e-3f;
    for (int i = 0; i < 12; ++i) y[i] = a + i * 0.125f;
    for (int i = 0; i < 8; ++i) x[i] = 0.f;
    for (int i = 0; i < 8; ++i) q[i] = f2{a + i, a - i};
    for (int i = 0; i < 4; ++i) p[i] = f2{0.f, 0.f};
    for (int i = 0; i < 4; ++i) u[i] = 0u;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            MF(acc[g & 3]);
            fill<C>(x, y, p, q, u, d, g);
        }
    }
    float s = d;
    for (int t = 0; t < 4; ++t) s += acc[t][0] + acc[t][1] + acc[t][2] + acc[t][3];
    for (int i = 0; i < 8; ++i) s += x[i];
    for (int i = 0; i < 4; ++i) s += p[i][0] + p[i][1] + (float)u[i];
    out[blockIdx.x * blockDim.x + lane] = s;
}

static const char* NAMES[] = {"mfma only", "1 exp", "2 exp", "1 add", "2 add", "3 add", "4 add", "exp+add",
                              "exp+2add", "exp+rcp+2add", "1 pk_fma", "2 fma", "1 pk_add", "1 cvt_pk_f16",
                              "dep exp", "dep add,rcp", "dep exp,add,rcp", "2exp+2add", "exp,rcp,exp,2add,fma"};

template <int C>
static void run(float* out, int cu, float base_ns[2]) {
    const int IT = 4000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int w = 0; w < 2; ++w) {
        const int waves = 4 * (w + 1);
        hipLaunchKernelGGL(kern<C>, dim3(cu), dim3(64 * waves), 0, 0, out, IT);
        hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern<C>, dim3(cu), dim3(64 * waves), 0, 0, out, IT);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        // one block per CU: waves / 4 waves per SIMD, each 16 IT MFMAs
        const double mfma_per_simd = (waves / 4) * 16.0 * IT;
        const double ns = ms / 5 * 1e6 / mfma_per_simd;
        if (C == 0) base_ns[w] = (float)ns;
        printf("%-24s %d wave/SIMD: %7.3f ns/MFMA  %6.2f cyc (MFMA-only = 16)\n", NAMES[C], w + 1, ns,
               16.0 * ns / base_ns[w]);
    }
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

template <int C>
static void run_all(float* out, int cu, float base[2]) {
    run<C>(out, cu, base);
    if constexpr (C < 18) run_all<C + 1>(out, cu, base);
}

int main() {
    int cu = 0;
    hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, 0);
    float* out;
    hipMalloc(&out, sizeof(float) * cu * 512);
    hipMemset(out, 0, sizeof(float) * cu * 512);
    float base[2] = {1.f, 1.f};
    run_all<0>(out, cu, base);
    return 0;
}
