// npd_common.hpp -- shared host/device helpers for libnpd (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "npd.h"

namespace npd {

// ------------------------------------------------------------------------------------- errors
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what);

#define NPD_HIP(call)                                              \
    do {                                                           \
        hipError_t _e = (call);                                    \
        if (_e != hipSuccess) return ::npd::hip_fail(_e, #call);   \
    } while (0)

#define NPD_ARG(cond, msg)                                         \
    do {                                                           \
        if (!(cond)) return ::npd::fail(NPD_EINVAL, (msg));        \
    } while (0)

// launch check: a failed launch is reported through hipGetLastError
inline int launch_check(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, what);
    return NPD_OK;
}

constexpr int kWave = 64;     // CDNA wavefront
constexpr int kMaxN = 256;    // largest code length compiled in
constexpr int kMaxWords = kMaxN / 32;

// ------------------------------------------------------------------------------------- code handle
struct CodeParams {           // passed to kernels by value (lives in SGPRs / kernarg segment)
    uint32_t frozen[kMaxWords];   // bit i = 1 iff position i frozen
    uint32_t rank[kMaxN];         // rank[i] = index of position i in the sorted info set (if info)
    int32_t info[kMaxN];          // sorted info positions
    int N, n, K;
    float infty;
    uint32_t tapmask;             // PAC: state-index taps (bit t -> state[t] participates)
    uint32_t smask;               // PAC: (1 << state_len) - 1
    int pac;
    // Subtree classes for the fast Polar kernel: 2 bits per node, node id = (N >> D) + (S0 >> D) for the
    // node of 2^D leaves starting at S0 (root id 1, ids < N).  0 = mixed, 1 = rate-0 (all frozen),
    // 2 = rate-1 (all information), 3 = repetition (only the last leaf carries information).
    uint32_t ntype[kMaxN / 16];
};

enum NodeType : uint32_t { kNodeMixed = 0, kNodeRate0 = 1, kNodeRate1 = 2, kNodeRep = 3 };

}  // namespace npd

struct npd_code {
    npd::CodeParams p;
    int device;
};

namespace npd {

// ------------------------------------------------------------------------------------- Philox
constexpr uint32_t kStreamMsg = 0x6D736700u;    // must match oracle/npd_oracle.c
constexpr uint32_t kStreamNoise = 0x6E300000u;

struct u32x4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u32x4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                              uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        // one 32x32 -> 64-bit product per multiplier (v_mad_u64_u32) instead of separate lo/hi multiplies
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return {c0, c1, c2, c3};
}

__device__ __forceinline__ u32x4 philox_block(uint64_t seed, uint32_t stream, uint64_t cw, uint32_t blk) {
    return philox4x32_10(blk, stream, (uint32_t)cw, (uint32_t)(cw >> 32), (uint32_t)seed, (uint32_t)(seed >> 32));
}

// uniform in (0, 1], exact in fp32
__device__ __forceinline__ float u01(uint32_t x) { return (float)((x >> 8) + 1u) * 5.9604644775390625e-08f; }

// two Box-Muller pairs -> 4 standard normals on the transcendental units: r = sqrt(-2 ln u1) with
// v_log_f32 (log2) and v_sqrt_f32; (cos, sin)(2 pi u2) with v_cos_f32 / v_sin_f32, whose argument is in
// revolutions (u2 itself, in (0, 1]).  ~10 instructions per pair instead of the ~150 of the libm
// functions; the oracle evaluates the same formula with glibc log2f / sqrtf and double-precision
// sin / cos (agreement ~1e-6, tests/test_sc_gpu.py).
__device__ __forceinline__ void normals4(const u32x4& o, float z[4]) {
    constexpr float kM2Ln2 = -1.38629436111989061883f;  // -2 ln 2
    const float r0 = __builtin_amdgcn_sqrtf(kM2Ln2 * __builtin_amdgcn_logf(u01(o.x)));
    const float t0 = u01(o.y);
    const float r1 = __builtin_amdgcn_sqrtf(kM2Ln2 * __builtin_amdgcn_logf(u01(o.z)));
    const float t1 = u01(o.w);
    z[0] = r0 * __builtin_amdgcn_cosf(t0);
    z[1] = r0 * __builtin_amdgcn_sinf(t0);
    z[2] = r1 * __builtin_amdgcn_cosf(t1);
    z[3] = r1 * __builtin_amdgcn_sinf(t1);
}

// ------------------------------------------------------------------------------------- misc device
__device__ __forceinline__ float sgnf(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }

__device__ __forceinline__ uint32_t fbits(float x) { return __float_as_uint(x); }
__device__ __forceinline__ float bitsf(uint32_t x) { return __uint_as_float(x); }

// wave-wide sum of a 32-bit value (all 64 lanes active)
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

inline int grid_for(int64_t tiles, int per_cu_blocks, int num_cu) {
    int64_t cap = (int64_t)per_cu_blocks * num_cu;
    if (tiles < cap) return (int)(tiles > 0 ? tiles : 1);
    return (int)cap;
}

int device_cu_count();

}  // namespace npd
