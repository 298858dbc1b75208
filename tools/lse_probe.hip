// Diagnostic only (not part of libnpd): evaluates the device LSE check node -- the same statement as
// npd_lse.hip's lse_f -- on recorded (x, y) pairs and prints where it differs from the CPU result.
// Build: hipcc --offload-arch=gfx950 -O3 -Iinclude -Ineural_polar_decoder_amd/csrc tools/lse_probe.hip -o tools/bin/lse_probe
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

__device__ __forceinline__ float lse_avoid_nan(float x, float y) {
    const float s = x + y;
    const float dyx = y - x;
    const float t1 = logf(1.0f + expf(s));
    const float t3 = logf(1.0f + expf(dyx));
    float r = (t1 - x) - t3;
    const float ad = fabsf(x - y);
    const float mx = (x > y) ? x : y;
    const float mn = (x < y) ? x : y;
    if (s > 200.0f) r = (ad < 200.0f) ? (y - t3) : mn;
    else if (s < -200.0f) r = (ad < 200.0f) ? (-x - t3) : -mx;
    else if (ad > 200.0f && fabsf(s) < 200.0f) r = t1 - mx;
    return r;
}
__device__ __forceinline__ float lse_f(float x, float y) {
    float r = lse_avoid_nan(x, y);
    if (r == 0.0f) {
        const float s = x + y;
        const float nume = (s < 0.0f) ? 0.0f : s;
        const float denom = (x > y) ? x : y;
        const float term1 = 0.5f * (expf(-nume) + expf(s - nume));
        const float term2 = 0.5f * (expf(x - denom) + expf(y - denom));
        const float T1 = (fabsf(term1 - 1.0f) < 1e-7f) ? (term1 - 1.0f) : logf(term1);
        const float T2 = (fabsf(term2 - 1.0f) < 1e-7f) ? (term2 - 1.0f) : logf(term2);
        float c = ((nume - denom) + T1) - T2;
        if (c == 0.0f) {
            const float a = (x < y) ? x : y;
            const float b = (-x < -y) ? -x : -y;
            c = (s > 0.0f) ? a : b;
        }
        r = c;
    }
    return r;
}
__global__ void probe(const float* xyr, float* out, float* parts, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const float x = xyr[3 * i], y = xyr[3 * i + 1];
        out[i] = lse_f(x, y);
        parts[4 * i + 0] = expf(x + y);
        parts[4 * i + 1] = logf(1.0f + expf(x + y));
        parts[4 * i + 2] = expf(y - x);
        parts[4 * i + 3] = logf(1.0f + expf(y - x));
    }
}
int main(int argc, char** argv) {
    FILE* f = fopen(argc > 1 ? argv[1] : "tools/lse_probe_calls.bin", "rb");
    if (!f) { printf("no input\n"); return 1; }
    std::vector<float> h;
    float v;
    while (fread(&v, 4, 1, f) == 1) h.push_back(v);
    fclose(f);
    const int n = (int)h.size() / 3;
    float *d, *o, *p;
    hipMalloc(&d, h.size() * 4); hipMalloc(&o, n * 4); hipMalloc(&p, n * 16);
    hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    probe<<<(n + 255) / 256, 256>>>(d, o, p, n);
    std::vector<float> out(n), parts(4 * n);
    hipMemcpy(out.data(), o, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(parts.data(), p, n * 16, hipMemcpyDeviceToHost);
    int shown = 0, diff = 0;
    for (int i = 0; i < n; ++i) {
        const float c = h[3 * i + 2], g = out[i];
        const bool same = (isnan(c) && isnan(g)) || c == g;
        if (!same) {
            ++diff;
            if (shown++ < 12)
                printf("call %d x=%.9g y=%.9g cpu=%.9g gpu=%.9g | exp(s)=%.9g t1=%.9g exp(d)=%.9g t3=%.9g\n", i, h[3 * i],
                       h[3 * i + 1], c, g, parts[4 * i], parts[4 * i + 1], parts[4 * i + 2], parts[4 * i + 3]);
        }
    }
    printf("calls %d differing %d\n", n, diff);
    return 0;
}
