// Does fp32 MFMA work of one wave overlap VALU work (plain fp32 and transcendental) of another wave on the
// same SIMD, or of the same wave?  Decides the GRU kernel's layout (one wave per SIMD vs two).
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/coissue tools/coissue.hip && tools/bin/coissue
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f16v __attribute__((ext_vector_type(16)));
typedef _Float16 hf8 __attribute__((ext_vector_type(8)));

// role: 0 = MFMA chain work, 1 = VALU fma work, 2 = VALU exp/rcp work, 3 = MFMA + fma interleaved (one wave),
//       4 = fp16 MFMA work (8 x v_mfma_f32_32x32x16_f16 per iteration: the same 256 SIMD-cycles as role 0's
//       four fp32 MFMAs if the f16 rate is 8x), 5 = fp16 MFMA + fma interleaved (one wave)
template <int ITERS>
__global__ void kern(float* out, const int* roles, int nroles) {
    const int wave = threadIdx.x >> 6;
    const int role = roles[wave % nroles];
    float a = out[threadIdx.x] + 1.0f, b = a * 0.5f;
    if (role == 4 || role == 5) {
        f16v acc[4];
        for (int t = 0; t < 4; ++t)
            for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
        hf8 ha, hb;
        for (int j = 0; j < 8; ++j) {
            ha[j] = (_Float16)(a + j);
            hb[j] = (_Float16)(b - j);
        }
        float x0 = a, x1 = b, x2 = a + b, x3 = a - b;
        for (int it = 0; it < ITERS; ++it) {
#pragma unroll
            for (int r = 0; r < 2; ++r)
#pragma unroll
                for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ha, hb, acc[t], 0, 0, 0);
            if (role == 5) {
#pragma unroll
                for (int k = 0; k < 24; ++k) {
                    x0 = fmaf(x0, 1.0001f, 0.5f);
                    x1 = fmaf(x1, 0.9999f, 0.25f);
                    x2 = fmaf(x2, 1.0002f, 0.125f);
                    x3 = fmaf(x3, 0.9998f, 0.0625f);
                }
            }
        }
        float s = x0 + x1 + x2 + x3;
        for (int t = 0; t < 4; ++t)
            for (int i = 0; i < 16; ++i) s += acc[t][i];
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    } else if (role == 0 || role == 3) {
        f16v acc[4];
        for (int t = 0; t < 4; ++t)
            for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
        float x0 = a, x1 = b, x2 = a + b, x3 = a - b;
        for (int it = 0; it < ITERS; ++it) {
#pragma unroll
            for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[t], 0, 0, 0);
            if (role == 3) {
#pragma unroll
                for (int k = 0; k < 24; ++k) {
                    x0 = fmaf(x0, 1.0001f, 0.5f);
                    x1 = fmaf(x1, 0.9999f, 0.25f);
                    x2 = fmaf(x2, 1.0002f, 0.125f);
                    x3 = fmaf(x3, 0.9998f, 0.0625f);
                }
            }
        }
        float s = x0 + x1 + x2 + x3;
        for (int t = 0; t < 4; ++t)
            for (int i = 0; i < 16; ++i) s += acc[t][i];
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    } else {
        float x[8];
        for (int i = 0; i < 8; ++i) x[i] = a + i;
        for (int it = 0; it < ITERS; ++it) {
            if (role == 1) {
#pragma unroll
                for (int k = 0; k < 12; ++k)
#pragma unroll
                    for (int i = 0; i < 8; ++i) x[i] = fmaf(x[i], 1.0001f, 0.5f);
            } else {
#pragma unroll
                for (int k = 0; k < 3; ++k)
#pragma unroll
                    for (int i = 0; i < 8; ++i) x[i] = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-x[i]));
            }
        }
        float s = 0;
        for (int i = 0; i < 8; ++i) s += x[i];
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    }
}

int main() {
    const int CU = 256, IT = 20000;
    float* out;
    int* roles;
    hipMalloc(&out, sizeof(float) * CU * 512);
    hipMalloc(&roles, sizeof(int) * 8);
    hipMemset(out, 0, sizeof(float) * CU * 512);
    struct Case {
        const char* name;
        int waves;
        int r[8];
    } cases[] = {
        {"mfma x4 (1/SIMD)", 4, {0, 0, 0, 0}},
        {"fma x4 (1/SIMD)", 4, {1, 1, 1, 1}},
        {"exp/rcp x4 (1/SIMD)", 4, {2, 2, 2, 2}},
        {"mfma x4 + fma x4 (2/SIMD)", 8, {0, 0, 0, 0, 1, 1, 1, 1}},
        {"mfma x4 + exp/rcp x4 (2/SIMD)", 8, {0, 0, 0, 0, 2, 2, 2, 2}},
        {"mfma x8 (2/SIMD)", 8, {0, 0, 0, 0, 0, 0, 0, 0}},
        {"mfma+fma same wave x4", 4, {3, 3, 3, 3}},
        {"f16 mfma x8 (1/SIMD)", 4, {4, 4, 4, 4}},
        {"f16 mfma x8 + fma x4 (2/SIMD)", 8, {4, 4, 4, 4, 1, 1, 1, 1}},
        {"f16 mfma x8 + exp/rcp x4 (2/SIMD)", 8, {4, 4, 4, 4, 2, 2, 2, 2}},
        {"f16 mfma x8 (2/SIMD)", 8, {4, 4, 4, 4, 4, 4, 4, 4}},
        {"f16 mfma+fma same wave x4", 4, {5, 5, 5, 5}},
    };
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (auto& c : cases) {
        hipMemcpy(roles, c.r, sizeof(int) * 8, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(kern<IT>, dim3(CU), dim3(64 * c.waves), 0, 0, out, roles, c.waves);
        hipEventRecord(e0);
        for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(kern<IT>, dim3(CU), dim3(64 * c.waves), 0, 0, out, roles, c.waves);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        // per iteration: 4 MFMA (64 cyc each at 1/SIMD) = 256 SIMD-cycles; fma role 96 VALU; exp role 48 trans + 24 add
        printf("%-34s %8.3f ms/launch  %6.1f ns/iter\n", c.name, ms / 3, ms / 3 * 1e6 / IT);
    }
    return 0;
}
