// npd_lse.hip -- exact log-sum-exp successive-cancellation decoding for gfx950
// (PolarCode.sc_decode and, below, the soft-output PolarCode.sc_decode_soft).
//
// Replaces PolarCode.sc_decode / decode (polar.py:209-279): the same SC tree as sc_decode_new, but
//   * the check-node update is the exact boxplus of utils.py:348-397 (log_sum_avoid_zero_NaN), not
//     min-sum;
//   * frozen leaves are decided +1 outright (no LLR prior, polar.py:236-238, 249-251);
//   * information leaves decide sign(L) (args.hard_decision) or tanh(L/2) (the reference's argparse
//     default, "soft SC"), and the partial sums propagated up the tree are products of those values;
//   * the output is sign(decoded_bits)[:, info] (polar.py:222), optionally decoded_bits itself.
//
// This decoder is transcendental-bound (4 exp/log per check node), not HBM-bound.  One codeword per
// lane.  N <= 128 (lse_sc_reg_kernel, below): the tree is unrolled at compile time with every LLR level
// and partial sum in registers (156 VGPRs at N = 64, 3 waves/SIMD; 256 + AGPRs at N = 128, 1 wave/SIMD,
// no scratch).  N = 256 (lse_sc_kernel): the SC schedule is walked iteratively (leaf i: one g step at depth
// ctz(i)+1, f steps down to the leaf, partial-sum combines for the ctz(i+1) finished nodes), and the
// per-lane LLR levels (N-1 floats) and partial sums (N floats) in LDS, lane-interleaved
// (element e of lane l at dword e*64 + l: every access of a wave is conflict-free).  The root level is
// read from y directly (two passes: f then g), through L1/L2.
//
// Floating point: each reference tensor op is one rounded fp32 op here (no contraction: rmul makes
// every product opaque); exp/log/tanh are the device libm (<= 1 ulp, as is torch's CPU Sleef path),
// so results agree with the reference to a few ulp and decisions agree except on near-zero LLRs
// (tests/test_lse_gpu.py states the tolerance).
#include <stdlib.h>

#include "npd_common.hpp"

namespace npd {
namespace lse {

struct Args {
    const float* y;
    float* msg;     // (B,K) sign(decoded_bits)[:, info], or null
    float* ubits;   // (B,N) decoded_bits, or null
    int64_t B;
    int64_t ntiles;
    float scale;
};

__device__ __forceinline__ float rmul(float a, float b) {
    float r = a * b;
    asm("" : "+v"(r));
    return r;
}

// log_sum_avoid_NaN (utils.py:295-345) evaluated elementwise.  The reference computes the "standard"
// formula and, only if the TENSOR holds a NaN/inf, patches four index sets.  Every element of a patched
// set either has a non-finite standard value (so the patch always runs for it) or a patched value equal
// to its standard value bit for bit, so applying the patches per element unconditionally is exact.
__device__ __forceinline__ float lse_avoid_nan(float x, float y) {
    const float s = x + y;
    const float dyx = y - x;
    const float t1 = logf(1.0f + expf(s));    // torch.log(1 + (x+y).exp())
    const float t3 = logf(1.0f + expf(dyx));  // torch.log(1 + (y-x).exp())
    float r = (t1 - x) - t3;
    const float ad = fabsf(x - y);
    const float mx = (x > y) ? x : y;  // a = torch.max(x, y)  (x, y are not NaN on these branches)
    const float mn = (x < y) ? x : y;  // b = torch.min(x, y)
    if (s > 200.0f) {                         // idx_1
        r = (ad < 200.0f) ? (y - t3) : mn;    // subset_1 / idx_1 ^ subset_1
    } else if (s < -200.0f) {                 // idx_2
        r = (ad < 200.0f) ? (-x - t3) : -mx;  // subset_2 / idx_2 ^ subset_2
    } else if (ad > 200.0f && fabsf(s) < 200.0f) {
        r = t1 - mx;                          // idx_3
    }
    return r;
}

// log_sum_avoid_zero_NaN (utils.py:348-397): re-evaluate exact zeros with the shifted formula
__device__ __forceinline__ float lse_f(float x, float y) {
    float r = lse_avoid_nan(x, y);
    if (r == 0.0f) {
        const float s = x + y;
        const float nume = (s < 0.0f) ? 0.0f : s;  // torch.relu (keeps -0)
        const float denom = (x > y) ? x : y;       // torch.max
        const float term1 = 0.5f * (expf(-nume) + expf(s - nume));
        const float term2 = 0.5f * (expf(x - denom) + expf(y - denom));
        const float T1 = (fabsf(term1 - 1.0f) < 1e-7f) ? (term1 - 1.0f) : logf(term1);
        const float T2 = (fabsf(term2 - 1.0f) < 1e-7f) ? (term2 - 1.0f) : logf(term2);
        float c = ((nume - denom) + T1) - T2;
        if (c == 0.0f) {
            const float a = (x < y) ? x : y;      // torch.min(x, y)
            const float b = (-x < -y) ? -x : -y;  // torch.min(-x, -y)
            c = (s > 0.0f) ? a : b;
        }
        r = c;
    }
    return r;
}

// g = u_hat * L_left + L_right (polar.py:253, 276); u is +-1/0 (hard) or a tanh product (soft)
__device__ __forceinline__ float lse_g(float u, float a, float b) { return rmul(u, a) + b; }

template <bool SOFT>
__global__ __launch_bounds__(64) void lse_sc_kernel(const CodeParams p, const Args a) {
    extern __shared__ float lds[];
    const int lane = threadIdx.x;
    const int N = p.N, n = p.n, K = p.K;
    float* const L = lds + lane;              // LLR level d (2^d values) at elements [2^d - 1, 2^(d+1) - 1)
    float* const beta = L + (N - 1) * kWave;  // partial sums, N values
#define LV(base, j) (L[((base) + (j)) * kWave])
#define BT(j) (beta[(j) * kWave])

    for (int64_t t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
        const int64_t row = t * kWave + lane;
        const bool valid = row < a.B;
        const int64_t r = valid ? row : a.B - 1;
        const float* yr = a.y + r * N;
        float* ub = (a.ubits && valid) ? a.ubits + row * N : nullptr;
        float* mh = (a.msg && valid) ? a.msg + row * K : nullptr;

        for (int i = 0; i < N; ++i) {
            int d;
            if (i == 0) {  // left child of the root: f on the channel LLRs
                const int h = N >> 1;
                for (int j = 0; j < h; ++j) LV(h - 1, j) = lse_f(rmul(a.scale, yr[j]), rmul(a.scale, yr[j + h]));
                d = n - 1;
            } else {  // right child of the node of 2^(k+1) leaves starting at i - 2^k
                const int k = __builtin_ctz((unsigned)i);
                const int h = 1 << k;
                const int s = i - h;
                if (k + 1 == n) {
                    for (int j = 0; j < h; ++j)
                        LV(h - 1, j) = lse_g(BT(s + j), rmul(a.scale, yr[j]), rmul(a.scale, yr[j + h]));
                } else {
                    for (int j = 0; j < h; ++j) LV(h - 1, j) = lse_g(BT(s + j), LV(2 * h - 1, j), LV(2 * h - 1, j + h));
                }
                d = k;
            }
            for (int dd = d; dd >= 1; --dd) {  // left children down to the leaf
                const int h = 1 << (dd - 1);
                for (int j = 0; j < h; ++j) LV(h - 1, j) = lse_f(LV(2 * h - 1, j), LV(2 * h - 1, j + h));
            }
            // leaf (polar.py:233-262)
            const bool frozen = (p.frozen[i >> 5] >> (i & 31)) & 1u;
            float u = 1.0f;
            if (!frozen) {
                const float Lf = LV(0, 0);
                u = SOFT ? tanhf(Lf * 0.5f) : sgnf(Lf);
            }
            BT(i) = u;
            if (ub) ub[i] = u;
            if (mh && !frozen) mh[p.rank[i]] = sgnf(u);
            // combine partial sums of every node whose right child ends at leaf i (polar.py:264, 279)
            for (int l = 1; l < n && ((i + 1) & ((1 << l) - 1)) == 0; ++l) {
                const int h = 1 << (l - 1);
                const int s = i + 1 - (1 << l);
                for (int j = 0; j < h; ++j) BT(s + j) = BT(s + j) * BT(s + h + j);
            }
        }
    }
#undef LV
#undef BT
}

template <bool SOFT>
static int launch(const CodeParams& p, Args a, hipStream_t stream) {
    const size_t lds = (size_t)(2 * p.N - 1) * kWave * sizeof(float);
    auto kern = lse_sc_kernel<SOFT>;
    static bool attr_set = false;  // benign race (idempotent)
    if (!attr_set && lds > 65536) {
        NPD_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
        attr_set = true;
    }
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, kWave, lds) != hipSuccess || occ <= 0) {
        (void)hipGetLastError();
        occ = 1;
    }
    a.ntiles = (a.B + kWave - 1) / kWave;
    const int grid = grid_for(a.ntiles, occ, device_cu_count());
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kWave), lds, stream, p, a);
    return launch_check("lse_sc_kernel launch");
}

// ------------------------------------------------------------------------------ register variant
// N <= 128: the SC tree unrolled at compile time (template recursion over the nodes), every LLR level
// and partial sum in a fixed VGPR (level d at lv[2^d, 2^(d+1)), the root at lv[N, 2N)): no LDS round
// trips, and the independent check nodes of a level give the scheduler parallel exp/log chains.
template <int N>
struct RegState {
    float lv[2 * N];
    float beta[N];
    uint32_t fz[(N + 31) / 32];  // frozen words, re-read opaquely per tile
    int k;                       // information leaves decided so far (= msg_hat column; info is sorted)
};

// Per-tile opaque copies of the loop-invariant frozen words: left alone, LICM hoists every per-leaf frozen
// test (a 64-bit lane mask) out of the tile loop and parks them in VGPR lanes (hundreds of v_writelane /
// v_readlane per tile at N = 64).  Priors are read per leaf at an opaque index for the same reason (an
// escaped pointer to the by-value argument would copy it to scratch instead).
template <int N>
__device__ __forceinline__ void opaque_code(RegState<N>& st, const CodeParams& p) {
#pragma unroll
    for (int w = 0; w < (N + 31) / 32; ++w) {
        uint32_t fw = p.frozen[w];
        asm volatile("" : "+s"(fw));
        st.fz[w] = fw;
    }
    st.k = 0;
}

template <int N, bool SOFT, int D, int S0>
__device__ __forceinline__ void reg_node(RegState<N>& st, const CodeParams& p, float* ub, float* mh) {
    if constexpr (D == 0) {
        const bool frozen = (st.fz[S0 >> 5] >> (S0 & 31)) & 1u;
        float u = 1.0f;
        if (!frozen) u = SOFT ? tanhf(st.lv[1] * 0.5f) : sgnf(st.lv[1]);
        st.beta[S0] = u;
        if (ub) ub[S0] = u;
        if (!frozen) {
            if (mh) mh[st.k] = sgnf(u);
            ++st.k;
        }
    } else {
        constexpr int h = 1 << (D - 1);
#pragma unroll
        for (int j = 0; j < h; ++j) st.lv[h + j] = lse_f(st.lv[2 * h + j], st.lv[3 * h + j]);
        reg_node<N, SOFT, D - 1, S0>(st, p, ub, mh);
#pragma unroll
        for (int j = 0; j < h; ++j) st.lv[h + j] = lse_g(st.beta[S0 + j], st.lv[2 * h + j], st.lv[3 * h + j]);
        reg_node<N, SOFT, D - 1, S0 + h>(st, p, ub, mh);
        if constexpr ((1 << D) < N) {
#pragma unroll
            for (int j = 0; j < h; ++j) st.beta[S0 + j] = st.beta[S0 + j] * st.beta[S0 + h + j];
        }
    }
}

template <int N>
constexpr int ilog2() {
    int n = 0;
    while ((1 << n) < N) ++n;
    return n;
}

template <int N, bool SOFT>
__global__ __launch_bounds__(64) void lse_sc_reg_kernel(const CodeParams p, const Args a) {
    const int lane = threadIdx.x;
    for (int64_t t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
        const int64_t row = t * kWave + lane;
        const bool valid = row < a.B;
        const int64_t r = valid ? row : a.B - 1;
        float* ub = (a.ubits && valid) ? a.ubits + row * N : nullptr;
        float* mh = (a.msg && valid) ? a.msg + row * p.K : nullptr;
        RegState<N> st;
        opaque_code(st, p);
        const float4* yr = reinterpret_cast<const float4*>(a.y + r * N);
#pragma unroll
        for (int q = 0; q < N / 4; ++q) {
            const float4 v = yr[q];
            st.lv[N + 4 * q + 0] = rmul(a.scale, v.x);
            st.lv[N + 4 * q + 1] = rmul(a.scale, v.y);
            st.lv[N + 4 * q + 2] = rmul(a.scale, v.z);
            st.lv[N + 4 * q + 3] = rmul(a.scale, v.w);
        }
        reg_node<N, SOFT, ilog2<N>(), 0>(st, p, ub, mh);
    }
}

template <int N, bool SOFT>
static int launch_reg(const CodeParams& p, Args a, hipStream_t stream) {
    auto kern = lse_sc_reg_kernel<N, SOFT>;
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, kWave, 0) != hipSuccess || occ <= 0) {
        (void)hipGetLastError();
        occ = 1;
    }
    a.ntiles = (a.B + kWave - 1) / kWave;
    const int grid = grid_for(a.ntiles, occ, device_cu_count());
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kWave), 0, stream, p, a);
    return launch_check("lse_sc_reg_kernel launch");
}

template <bool SOFT>
static int dispatch(const CodeParams& p, const Args& a, hipStream_t s) {
    // the register variant reads y rows as float4: 16-byte aligned rows only
    const bool aligned = ((uintptr_t)a.y & 15u) == 0;
    if (aligned) {
        switch (p.N) {
            case 4: return launch_reg<4, SOFT>(p, a, s);
            case 8: return launch_reg<8, SOFT>(p, a, s);
            case 16: return launch_reg<16, SOFT>(p, a, s);
            case 32: return launch_reg<32, SOFT>(p, a, s);
            case 64: return launch_reg<64, SOFT>(p, a, s);
            case 128: return launch_reg<128, SOFT>(p, a, s);
            default: break;
        }
    }
    return launch<SOFT>(p, a, s);
}

// ------------------------------------------------------------------------------ soft SC (sc_decode_soft)
// PolarCode.sc_decode_soft / decode_soft (polar.py:281-358): the same tree, but every node returns LLRs
// instead of partial sums -- leaf: L^ = clamp(L + prior, -1000, 1000) (utils.py:259-263 with the 1e-10
// margins vanishing in fp32), decided sign/tanh; right child input LSE(L^_left, L_a) + L_b; node return
// [LSE(L^_u, L^_v), L^_v].  No frozen handling (priors carry it).
// PolarCode.sc_decode_soft_new (polar.py:485-607) is the same decoder spelled differently: per leaf it
// re-walks the root-to-leaf path (updateLLR_soft / partial_decode_soft) and rebuilds the "soft partial
// sums" from the leaf LLRs decided so far (updatePartialSums_soft: stage s replaces [a, b] by
// [LSE(a, b), b] at stride 2^s), which for every completed block equals the returned-LLR vector above
// (same operands, same order).  Differences: its leaf stores clamp(L + prior) + prior, and its output is
// u_hat = sign(stored leaf)[:, info] -- SoftArgs::twice with hard decisions.  N <= 64: register-resident;
// N = 128, 256: LDS-resident iterative walk (lse_soft_lds_kernel, the layout of lse_sc_kernel).
struct SoftArgs {
    const float* y;
    float* msg;
    float* ubits;
    int64_t B;
    int64_t ntiles;
    float scale;
    int twice;  // sc_decode_soft_new: the stored leaf LLR is clamp(L + prior) + prior (polar.py:520-546)
    float prior[kMaxN];
};

__device__ __forceinline__ float clamp1000(float x) { return x < -1000.0f ? -1000.0f : (x > 1000.0f ? 1000.0f : x); }

template <int N, bool SOFT, int D, int S0>
__device__ __forceinline__ void soft_node(RegState<N>& st, const CodeParams& p, const SoftArgs& a, float* ub, float* mh) {
    if constexpr (D == 0) {
        int ix = S0;
        asm volatile("" : "+s"(ix));
        const float pr = a.prior[ix];
        float L = clamp1000(st.lv[1] + pr);
        if (a.twice) L = L + pr;
        const float u = SOFT ? tanhf(L * 0.5f) : sgnf(L);
        st.beta[S0] = L;
        if (ub) ub[S0] = u;
        const bool frozen = (st.fz[S0 >> 5] >> (S0 & 31)) & 1u;
        if (!frozen) {
            if (mh) mh[st.k] = sgnf(u);
            ++st.k;
        }
    } else {
        constexpr int h = 1 << (D - 1);
#pragma unroll
        for (int j = 0; j < h; ++j) st.lv[h + j] = lse_f(st.lv[2 * h + j], st.lv[3 * h + j]);
        soft_node<N, SOFT, D - 1, S0>(st, p, a, ub, mh);
#pragma unroll
        for (int j = 0; j < h; ++j) st.lv[h + j] = lse_f(st.beta[S0 + j], st.lv[2 * h + j]) + st.lv[3 * h + j];
        soft_node<N, SOFT, D - 1, S0 + h>(st, p, a, ub, mh);
        if constexpr ((1 << D) < N) {  // the root's returned LLRs are never used
#pragma unroll
            for (int j = 0; j < h; ++j) st.beta[S0 + j] = lse_f(st.beta[S0 + j], st.beta[S0 + h + j]);
        }
    }
}

template <int N, bool SOFT>
__global__ __launch_bounds__(64) void lse_soft_sc_kernel(const CodeParams p, const SoftArgs a) {
    const int lane = threadIdx.x;
    for (int64_t t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
        const int64_t row = t * kWave + lane;
        const bool valid = row < a.B;
        const int64_t r = valid ? row : a.B - 1;
        float* ub = (a.ubits && valid) ? a.ubits + row * N : nullptr;
        float* mh = (a.msg && valid) ? a.msg + row * p.K : nullptr;
        RegState<N> st;
        opaque_code(st, p);
        const float4* yr = reinterpret_cast<const float4*>(a.y + r * N);
#pragma unroll
        for (int q = 0; q < N / 4; ++q) {
            const float4 v = yr[q];
            st.lv[N + 4 * q + 0] = rmul(a.scale, v.x);
            st.lv[N + 4 * q + 1] = rmul(a.scale, v.y);
            st.lv[N + 4 * q + 2] = rmul(a.scale, v.z);
            st.lv[N + 4 * q + 3] = rmul(a.scale, v.w);
        }
        soft_node<N, SOFT, ilog2<N>(), 0>(st, p, a, ub, mh);
    }
}

template <int N, bool SOFT>
static int launch_soft(const CodeParams& p, SoftArgs a, hipStream_t stream) {
    auto kern = lse_soft_sc_kernel<N, SOFT>;
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, kWave, 0) != hipSuccess || occ <= 0) {
        (void)hipGetLastError();
        occ = 1;
    }
    a.ntiles = (a.B + kWave - 1) / kWave;
    const int grid = grid_for(a.ntiles, occ, device_cu_count());
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kWave), 0, stream, p, a);
    return launch_check("lse_soft_sc_kernel launch");
}

// N >= 128: per-lane LLR levels (N-1 floats) and returned LLRs (N floats) in LDS, lane-interleaved; the
// schedule of lse_sc_kernel with decode_soft's node rules: right-child input LSE(L^_left, L_a) + L_b,
// node return [LSE(L^_u, L^_v), L^_v] combined in place when a node's right child finishes.
template <bool SOFT>
__global__ __launch_bounds__(64) void lse_soft_lds_kernel(const CodeParams p, const SoftArgs a) {
    extern __shared__ float lds[];
    const int lane = threadIdx.x;
    const int N = p.N, n = p.n, K = p.K;
    float* const L = lds + lane;              // LLR level with 2^d values at elements [2^d - 1, 2^(d+1) - 1)
    float* const beta = L + (N - 1) * kWave;  // returned LLRs L^, N values
#define LV(base, j) (L[((base) + (j)) * kWave])
#define BT(j) (beta[(j) * kWave])
    for (int64_t t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
        const int64_t row = t * kWave + lane;
        const bool valid = row < a.B;
        const int64_t r = valid ? row : a.B - 1;
        const float* yr = a.y + r * N;
        float* ub = (a.ubits && valid) ? a.ubits + row * N : nullptr;
        float* mh = (a.msg && valid) ? a.msg + row * K : nullptr;
        for (int i = 0; i < N; ++i) {
            int d;
            if (i == 0) {
                const int h = N >> 1;
                for (int j = 0; j < h; ++j) LV(h - 1, j) = lse_f(rmul(a.scale, yr[j]), rmul(a.scale, yr[j + h]));
                d = n - 1;
            } else {
                const int k = __builtin_ctz((unsigned)i);
                const int h = 1 << k;
                const int s = i - h;
                if (k + 1 == n) {
                    for (int j = 0; j < h; ++j)
                        LV(h - 1, j) = lse_f(BT(s + j), rmul(a.scale, yr[j])) + rmul(a.scale, yr[j + h]);
                } else {
                    for (int j = 0; j < h; ++j) LV(h - 1, j) = lse_f(BT(s + j), LV(2 * h - 1, j)) + LV(2 * h - 1, j + h);
                }
                d = k;
            }
            for (int dd = d; dd >= 1; --dd) {
                const int h = 1 << (dd - 1);
                for (int j = 0; j < h; ++j) LV(h - 1, j) = lse_f(LV(2 * h - 1, j), LV(2 * h - 1, j + h));
            }
            float Lf = clamp1000(LV(0, 0) + a.prior[i]);
            if (a.twice) Lf = Lf + a.prior[i];
            const float u = SOFT ? tanhf(Lf * 0.5f) : sgnf(Lf);
            BT(i) = Lf;
            if (ub) ub[i] = u;
            const bool frozen = (p.frozen[i >> 5] >> (i & 31)) & 1u;
            if (mh && !frozen) mh[p.rank[i]] = sgnf(u);
            for (int l = 1; l < n && ((i + 1) & ((1 << l) - 1)) == 0; ++l) {
                const int h = 1 << (l - 1);
                const int s = i + 1 - (1 << l);
                for (int j = 0; j < h; ++j) BT(s + j) = lse_f(BT(s + j), BT(s + h + j));
            }
        }
    }
#undef LV
#undef BT
}

template <bool SOFT>
static int launch_soft_lds(const CodeParams& p, SoftArgs a, hipStream_t stream) {
    const size_t lds = (size_t)(2 * p.N - 1) * kWave * sizeof(float);
    auto kern = lse_soft_lds_kernel<SOFT>;
    static bool attr_set = false;  // benign race (idempotent)
    if (!attr_set && lds > 65536) {
        NPD_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
        attr_set = true;
    }
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, kWave, lds) != hipSuccess || occ <= 0) {
        (void)hipGetLastError();
        occ = 1;
    }
    a.ntiles = (a.B + kWave - 1) / kWave;
    const int grid = grid_for(a.ntiles, occ, device_cu_count());
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kWave), lds, stream, p, a);
    return launch_check("lse_soft_lds_kernel launch");
}

template <bool SOFT>
static int dispatch_soft(const CodeParams& p, const SoftArgs& a, hipStream_t s) {
    switch (p.N) {
        case 4: return launch_soft<4, SOFT>(p, a, s);
        case 8: return launch_soft<8, SOFT>(p, a, s);
        case 16: return launch_soft<16, SOFT>(p, a, s);
        case 32: return launch_soft<32, SOFT>(p, a, s);
        case 64: return launch_soft<64, SOFT>(p, a, s);
        default: return launch_soft_lds<SOFT>(p, a, s);
    }
}

}  // namespace lse
}  // namespace npd

using namespace npd;

extern "C" int npd_sc_decode_lse(const npd_code* code, const float* y, float llr_scale, int hard_decision,
                                 float* msg_hat, float* u_bits, int64_t B, void* stream) {
    NPD_ARG(code != nullptr, "npd_sc_decode_lse: code is NULL");
    NPD_ARG(!code->p.pac, "npd_sc_decode_lse: Polar codes only (PolarCode.sc_decode)");
    NPD_ARG(code->p.N >= 2 && code->p.N <= kMaxN, "npd_sc_decode_lse: 2 <= N <= 256");
    NPD_ARG(B >= 0, "npd_sc_decode_lse: B < 0");
    NPD_ARG(B == 0 || y != nullptr, "npd_sc_decode_lse: y is NULL");
    if (B == 0) return NPD_OK;
    lse::Args a{};
    a.y = y;
    a.msg = msg_hat;
    a.ubits = u_bits;
    a.B = B;
    a.scale = llr_scale;
    if (getenv("NPD_LSE_LDS")) {  // force the LDS-resident variant (testing / A-B)
        return hard_decision ? lse::launch<false>(code->p, a, (hipStream_t)stream)
                             : lse::launch<true>(code->p, a, (hipStream_t)stream);
    }
    return hard_decision ? lse::dispatch<false>(code->p, a, (hipStream_t)stream)
                         : lse::dispatch<true>(code->p, a, (hipStream_t)stream);
}

static int soft_entry(const npd_code* code, const float* y, float llr_scale, int hard_decision, int twice,
                      const float* priors, float* msg_hat, float* u_bits, int64_t B, void* stream) {
    lse::SoftArgs a{};
    a.y = y;
    a.msg = msg_hat;
    a.ubits = u_bits;
    a.B = B;
    a.scale = llr_scale;
    a.twice = twice;
    for (int i = 0; i < kMaxN; ++i) a.prior[i] = (priors && i < code->p.N) ? priors[i] : 0.0f;
    if (getenv("NPD_SOFT_LDS")) {  // force the LDS-resident variant (testing / A-B)
        return hard_decision ? lse::launch_soft_lds<false>(code->p, a, (hipStream_t)stream)
                             : lse::launch_soft_lds<true>(code->p, a, (hipStream_t)stream);
    }
    return hard_decision ? lse::dispatch_soft<false>(code->p, a, (hipStream_t)stream)
                         : lse::dispatch_soft<true>(code->p, a, (hipStream_t)stream);
}

extern "C" int npd_sc_decode_soft(const npd_code* code, const float* y, float llr_scale, int hard_decision,
                                  const float* priors, float* msg_hat, float* u_bits, int64_t B, void* stream) {
    NPD_ARG(code != nullptr, "npd_sc_decode_soft: code is NULL");
    NPD_ARG(!code->p.pac, "npd_sc_decode_soft: Polar codes only (PolarCode.sc_decode_soft)");
    NPD_ARG(code->p.N >= 4 && code->p.N <= kMaxN, "npd_sc_decode_soft: 4 <= N <= 256");
    NPD_ARG(B >= 0, "npd_sc_decode_soft: B < 0");
    NPD_ARG(B == 0 || y != nullptr, "npd_sc_decode_soft: y is NULL");
    NPD_ARG(((uintptr_t)y & 15u) == 0, "npd_sc_decode_soft: y must be 16-byte aligned");
    if (B == 0) return NPD_OK;
    return soft_entry(code, y, llr_scale, hard_decision, 0, priors, msg_hat, u_bits, B, stream);
}

extern "C" int npd_sc_decode_soft_new(const npd_code* code, const float* y, float llr_scale, const float* priors,
                                      float* msg_hat, float* u_hat, int64_t B, void* stream) {
    NPD_ARG(code != nullptr, "npd_sc_decode_soft_new: code is NULL");
    NPD_ARG(!code->p.pac, "npd_sc_decode_soft_new: Polar codes only (PolarCode.sc_decode_soft_new)");
    NPD_ARG(code->p.N >= 4 && code->p.N <= kMaxN, "npd_sc_decode_soft_new: 4 <= N <= 256");
    NPD_ARG(B >= 0, "npd_sc_decode_soft_new: B < 0");
    NPD_ARG(B == 0 || y != nullptr, "npd_sc_decode_soft_new: y is NULL");
    NPD_ARG(((uintptr_t)y & 15u) == 0, "npd_sc_decode_soft_new: y must be 16-byte aligned");
    if (B == 0) return NPD_OK;
    return soft_entry(code, y, llr_scale, 1, 1, priors, msg_hat, u_hat, B, stream);
}
