// npd_gen.hip -- encoder, AWGN channel, fused Monte-Carlo data generation and error counters.
//
//   npd_encode       <- PolarCode.encode_plotkin (polar.py:128-148), PAC.pac_encode (pac_code.py:220-224)
//   npd_awgn         <- PolarCode.channel (polar.py:201-207) / PAC.channel (pac_code.py:226-231)
//   npd_mc_generate  <- msg = 1-2*randint; x = encode(msg); y = channel(x) (run_models.py:318-323)
//   npd_count_errors <- errors_ber / errors_bler counting (utils.py:17-51)
#include "npd_common.hpp"

namespace npd {
namespace gen {

__device__ __forceinline__ void lds_wr(char* lds, uint32_t byte, float v) { *reinterpret_cast<float*>(lds + byte) = v; }
__device__ __forceinline__ float lds_rd(const char* lds, uint32_t byte) { return *reinterpret_cast<const float*>(lds + byte); }

// ---------------------------------------------------------------------------------- encode (float, exact)
// One lane per codeword; the codeword row lives in LDS (stride N+1 floats: conflict-free per-lane rows).
// msg tile and x tile move between HBM and LDS with coalesced dword accesses.
__global__ __launch_bounds__(64) void encode_kernel(const CodeParams p, const float* __restrict__ msg,
                                                    float* __restrict__ x, int64_t B) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int lane = threadIdx.x;
    const int N = p.N, K = p.K, NP = N + 1;
    const int KP = K | 1;
    char* rowbuf = lds;                                   // 64 x NP floats
    char* msgbuf = lds + kWave * NP * 4;                  // 64 x KP floats
    int32_t* info = reinterpret_cast<int32_t*>(msgbuf + kWave * KP * 4);
    for (int k = lane; k < K; k += kWave) info[k] = p.info[k];
    const int64_t ntiles = (B + kWave - 1) / kWave;
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int64_t row0 = t * kWave;
        const int rows = (int)((B - row0) < kWave ? (B - row0) : kWave);
        // coalesced msg tile -> LDS rows
        for (int e = lane; e < rows * K; e += kWave) {
            const int r = e / K, k = e % K;
            lds_wr(msgbuf, (uint32_t)((r * KP + k) * 4), msg[row0 * K + e]);
        }
        char* u = rowbuf + lane * NP * 4;
        for (int i = 0; i < N; ++i) lds_wr(u, 4 * i, 1.0f);
        for (int k = 0; k < K; ++k) lds_wr(u, 4 * info[k], lds_rd(msgbuf, (uint32_t)((lane * KP + k) * 4)));
        if (p.pac) {
            // conv pre-transform (pac_code.py:181-208): u_i = v_i * prod_{taps} state, state <- v
            uint32_t st = 0;
            for (int i = 0; i < N; ++i) {
                const float v = lds_rd(u, 4 * i);
                const float ui = (__builtin_popcount(st & p.tapmask) & 1) ? -v : v;
                st = ((st << 1) | (v < 0.0f ? 1u : 0u)) & p.smask;
                lds_wr(u, 4 * i, ui);
            }
        }
        // Plotkin butterfly, stage order d = 0..n-1 (products in the reference's order)
        for (int h = 1; h < N; h <<= 1)
            for (int i = 0; i < N; i += 2 * h)
                for (int j = 0; j < h; ++j) lds_wr(u, 4 * (i + j), lds_rd(u, 4 * (i + j)) * lds_rd(u, 4 * (i + h + j)));
        // coalesced x tile store
        for (int e = lane; e < rows * N; e += kWave) {
            const int r = e / N, i = e % N;
            x[row0 * N + e] = lds_rd(rowbuf, (uint32_t)((r * NP + i) * 4));
        }
    }
}

// ---------------------------------------------------------------------------------- AWGN
// one thread per 4 consecutive elements of one codeword: 16-B loads/stores, one Philox call
__global__ __launch_bounds__(256) void awgn_kernel(const float4* __restrict__ x, float4* __restrict__ y, int64_t B,
                                                   int C, float sigma, uint64_t seed, uint32_t snr_index,
                                                   uint64_t cw_offset) {
    const int64_t total = B * (int64_t)C;
    for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = idx / C;
        const uint32_t j = (uint32_t)(idx - b * C);
        const u32x4 o = philox_block(seed, kStreamNoise + snr_index, cw_offset + (uint64_t)b, j);
        float z[4];
        normals4(o, z);
        const float4 xv = x[idx];
        float4 yv;
        // y = x + fl32(sigma * z): two roundings, no contraction (torch: sigma*randn, then add)
        yv.x = __fadd_rn(xv.x, __fmul_rn(sigma, z[0]));
        yv.y = __fadd_rn(xv.y, __fmul_rn(sigma, z[1]));
        yv.z = __fadd_rn(xv.z, __fmul_rn(sigma, z[2]));
        yv.w = __fadd_rn(xv.w, __fmul_rn(sigma, z[3]));
        y[idx] = yv;
    }
}

// ---------------------------------------------------------------------------------- fused MC generation
// Phase 1, one lane per codeword: Philox message bits -> positions (bit domain) -> PAC conv (bit domain) ->
// Plotkin butterfly as XOR on 32-bit words; the codeword's bits go to LDS.  Phase 2, one lane per 16-B
// chunk of the wave's 64 x N output tile: BPSK + sigma * N(0,1) (Philox counter = (chunk, codeword), so
// the mapping of work to lanes does not change any value), stored coalesced.
template <int N>
__global__ __launch_bounds__(256) void mc_generate_kernel(const CodeParams p, float* __restrict__ msg,
                                                          float* __restrict__ x, float* __restrict__ y, int64_t B,
                                                          float sigma, uint64_t seed, uint32_t snr_index,
                                                          uint64_t cw_offset) {
    constexpr int NW = (N + 31) / 32;
    constexpr int MB = (N + 127) / 128;  // Philox blocks for up to N message bits
    constexpr int C = N / 4;             // 16-B chunks per row
    __shared__ uint32_t sU[4][kWave][NW];
    __shared__ uint32_t sM[4][kWave][4 * MB + 1];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t b0 = ((int64_t)blockIdx.x * 4 + wave) * kWave;
    const int64_t b = b0 + lane;
    if (b < B) {
        const uint64_t cw = cw_offset + (uint64_t)b;
        uint32_t m[4 * MB];
#pragma unroll
        for (int blk = 0; blk < MB; ++blk) {
            const u32x4 o = philox_block(seed, kStreamMsg, cw, (uint32_t)blk);
            m[4 * blk + 0] = o.x; m[4 * blk + 1] = o.y; m[4 * blk + 2] = o.z; m[4 * blk + 3] = o.w;
        }
        if (msg) {
#pragma unroll
            for (int q = 0; q < 4 * MB; ++q) sM[wave][lane][q] = m[q];
        }
        // scatter message bits to positions: info positions are sorted, so slot k advances with i
        uint32_t U[NW];
#pragma unroll
        for (int w = 0; w < NW; ++w) U[w] = 0;
        uint32_t cur = m[0];
        int kk = 0;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            if (!((p.frozen[i >> 5] >> (i & 31)) & 1u)) {
                U[i >> 5] |= (cur & 1u) << (i & 31);
                cur >>= 1;
                ++kk;
                if ((kk & 31) == 0) {
                    uint32_t w = 0;
#pragma unroll
                    for (int q = 1; q < 4 * MB; ++q) w = ((kk >> 5) == q) ? m[q] : w;
                    cur = w;
                }
            }
        }
        if (p.pac) {
            // u_i = v_i xor parity(state & taps); state <- v (pac_code.py:181-208), bit domain (1 == -1)
            uint32_t st = 0;
#pragma unroll
            for (int i = 0; i < N; ++i) {
                const uint32_t v = (U[i >> 5] >> (i & 31)) & 1u;
                const uint32_t par = (uint32_t)__builtin_popcount(st & p.tapmask) & 1u;
                U[i >> 5] ^= par << (i & 31);
                st = ((st << 1) | v) & p.smask;
            }
        }
        // Plotkin butterfly: left ^= right, stage order irrelevant in GF(2)
#pragma unroll
        for (int h = 1; h < 32 && h < N; h <<= 1) {
            uint32_t msk = 0;
            for (int i = 0; i < 32; ++i)
                if (((i / h) & 1) == 0) msk |= 1u << i;
#pragma unroll
            for (int w = 0; w < NW; ++w) U[w] ^= (U[w] >> h) & msk;
        }
#pragma unroll
        for (int hw = 1; hw < NW; hw <<= 1)
#pragma unroll
            for (int w = 0; w < NW; ++w)
                if (((w / hw) & 1) == 0) U[w] ^= U[w + hw];
#pragma unroll
        for (int w = 0; w < NW; ++w) sU[wave][lane][w] = U[w];
    }
    __syncthreads();
    if (msg) {  // message rows of the tile, coalesced: float f = codeword f / K, bit f % K
        const int64_t nf = (B - b0 < kWave ? B - b0 : kWave) * (int64_t)p.K;
        float* mt = msg + b0 * p.K;
        for (int f = lane; f < nf; f += kWave) {
            const int r = f / p.K, k = f % p.K;
            mt[f] = ((sM[wave][r][k >> 5] >> (k & 31)) & 1u) ? -1.0f : 1.0f;
        }
    }
    // BPSK + noise, coalesced: chunk g of the tile = codeword g / C, float4 g % C of its row
    float4* yt = reinterpret_cast<float4*>(y) + b0 * C;
    float4* xt = x ? reinterpret_cast<float4*>(x) + b0 * C : nullptr;
    const int64_t nchunks = (B - b0 < kWave ? B - b0 : kWave) * C;
#pragma unroll 4
    for (int q = 0; q < C; ++q) {
        const int g = lane + kWave * q;
        if (g < nchunks) {
            const int r = g / C, j = g % C;
            const uint64_t cw = cw_offset + (uint64_t)(b0 + r);
            const u32x4 o = philox_block(seed, kStreamNoise + snr_index, cw, (uint32_t)j);
            float z[4];
            normals4(o, z);
            const uint32_t bits = (sU[wave][r][(4 * j) >> 5] >> ((4 * j) & 31)) & 0xFu;
            float xv[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) xv[e] = ((bits >> e) & 1u) ? -1.0f : 1.0f;
            float4 yv;
            yv.x = __fadd_rn(xv[0], __fmul_rn(sigma, z[0]));
            yv.y = __fadd_rn(xv[1], __fmul_rn(sigma, z[1]));
            yv.z = __fadd_rn(xv[2], __fmul_rn(sigma, z[2]));
            yv.w = __fadd_rn(xv[3], __fmul_rn(sigma, z[3]));
            yt[g] = yv;
            if (xt) xt[g] = make_float4(xv[0], xv[1], xv[2], xv[3]);
        }
    }
}

// ---------------------------------------------------------------------------------- error counters
// One wave per row at a time, lanes over the K compared positions: the reference row and the decision
// row are read with consecutive-lane (coalesced) loads, a ballot + popcount counts the row's bit errors,
// and a nonzero count is a block error.  Four rows are in flight per wave iteration.  Decisions may be
// full (B, W) rows read at columns cols[k] (e.g. decoded (B, N) at the information positions) so no
// gathered (B, K) copy is made.  One counter atomic pair per workgroup.
struct CountArgs {
    const float* ref;
    const float* hat;
    unsigned long long* counters;
    int64_t B;
    int K, W, use_cols;
    int32_t cols[kMaxN];
};

__global__ __launch_bounds__(256) void count_errors_kernel(const CountArgs a) {
    __shared__ uint32_t red[2];
    const int lane = threadIdx.x & 63;
    if (threadIdx.x < 2) red[threadIdx.x] = 0u;
    __syncthreads();
    const int64_t nw = (int64_t)gridDim.x * 4;
    uint32_t eb = 0, bl = 0;
    for (int64_t r0 = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r0 < a.B; r0 += 4 * nw) {
        uint32_t ne[4] = {0u, 0u, 0u, 0u};
        for (int k0 = 0; k0 < a.K; k0 += 64) {
            const int k = k0 + lane;
            const int c = k < a.K ? (a.use_cols ? a.cols[k] : k) : 0;
            float rv[4], hv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int64_t r = r0 + u * nw;
                const bool ok = k < a.K && r < a.B;
                rv[u] = ok ? a.ref[r * a.K + k] : 0.0f;
                hv[u] = ok ? a.hat[r * a.W + c] : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) ne[u] += (uint32_t)__builtin_popcountll(__ballot(rintf(rv[u]) != rintf(hv[u])));
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            eb += ne[u];
            bl += ne[u] ? 1u : 0u;
        }
    }
    if (lane == 0 && (eb | bl)) {
        atomicAdd(&red[0], eb);
        atomicAdd(&red[1], bl);
    }
    __syncthreads();
    if (threadIdx.x < 2 && red[threadIdx.x]) atomicAdd(a.counters + threadIdx.x, (unsigned long long)red[threadIdx.x]);
}

// Masked count (errors_ber's mask argument, utils.py:17-25): counters[0] += sum(mask * [round(ref) !=
// round(hat)]), counters[1] += sum(mask), over (B, K) with an integer mask (the reference's loops pass
// torch.ones(...).long(), run_models.py:325-326).  Both sums are exact (uint64); grid-stride over elements,
// one atomic pair per workgroup.
__global__ __launch_bounds__(256) void count_errors_masked_kernel(const float* __restrict__ ref,
                                                                  const float* __restrict__ hat,
                                                                  const int64_t* __restrict__ mask, int64_t n,
                                                                  unsigned long long* counters) {
    __shared__ unsigned long long red[2][4];
    unsigned long long se = 0, sm = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const unsigned long long m = (unsigned long long)mask[i];
        sm += m;
        se += (rintf(ref[i]) != rintf(hat[i])) ? m : 0ull;
    }
    for (int o = 32; o > 0; o >>= 1) {
        se += __shfl_xor(se, o, 64);
        sm += __shfl_xor(sm, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = se;
        red[1][threadIdx.x >> 6] = sm;
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        const unsigned long long v = red[threadIdx.x][0] + red[threadIdx.x][1] + red[threadIdx.x][2] + red[threadIdx.x][3];
        if (v) atomicAdd(counters + threadIdx.x, v);
    }
}

}  // namespace gen
}  // namespace npd

using namespace npd;

extern "C" int npd_encode(const npd_code* code, const float* msg, float* x, int64_t B, void* stream) {
    NPD_ARG(code != nullptr, "npd_encode: code is NULL");
    NPD_ARG(B >= 0, "npd_encode: B < 0");
    if (B == 0) return NPD_OK;
    NPD_ARG(x != nullptr && (msg != nullptr || code->p.K == 0), "npd_encode: null pointer");
    const int N = code->p.N, K = code->p.K;
    const size_t lds = (size_t)kWave * (N + 1) * 4 + (size_t)kWave * (K | 1) * 4 + (size_t)N * 4;
    static bool attr = false;
    if (!attr) {
        NPD_HIP(hipFuncSetAttribute((const void*)gen::encode_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
        attr = true;
    }
    const int64_t tiles = (B + kWave - 1) / kWave;
    const int grid = grid_for(tiles, 4, device_cu_count());
    hipLaunchKernelGGL(gen::encode_kernel, dim3(grid), dim3(kWave), lds, (hipStream_t)stream, code->p, msg, x, B);
    return launch_check("encode_kernel launch");
}

extern "C" int npd_awgn(const float* x, float* y, int64_t B, int N, float sigma, uint64_t seed, uint32_t snr_index,
                        uint64_t cw_offset, void* stream) {
    NPD_ARG(B >= 0, "npd_awgn: B < 0");
    NPD_ARG(N > 0 && N % 4 == 0, "npd_awgn: N must be a positive multiple of 4");
    if (B == 0) return NPD_OK;
    NPD_ARG(x != nullptr && y != nullptr, "npd_awgn: null pointer");
    NPD_ARG(((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0, "npd_awgn: x and y must be 16-byte aligned");
    const int C = N / 4;
    const int64_t total = B * C;
    const int grid = grid_for((total + 255) / 256, 8, device_cu_count());
    hipLaunchKernelGGL(gen::awgn_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const float4*)x, (float4*)y, B, C,
                       sigma, seed, snr_index, cw_offset);
    return launch_check("awgn_kernel launch");
}

template <int N>
static int mc_gen_launch(const npd_code* code, float* msg, float* x, float* y, int64_t B, float sigma, uint64_t seed,
                         uint32_t snr_index, uint64_t cw_offset, hipStream_t s) {
    const int64_t blocks = (B + 4 * kWave - 1) / (4 * kWave);
    hipLaunchKernelGGL(gen::mc_generate_kernel<N>, dim3((unsigned)blocks), dim3(256), 0, s, code->p, msg, x, y, B, sigma,
                       seed, snr_index, cw_offset);
    return launch_check("mc_generate_kernel launch");
}

extern "C" int npd_mc_generate(const npd_code* code, float* msg, float* x, float* y, int64_t B, float sigma,
                               uint64_t seed, uint32_t snr_index, uint64_t cw_offset, void* stream) {
    NPD_ARG(code != nullptr, "npd_mc_generate: code is NULL");
    NPD_ARG(B >= 0, "npd_mc_generate: B < 0");
    if (B == 0) return NPD_OK;
    NPD_ARG(y != nullptr, "npd_mc_generate: y is NULL");
    NPD_ARG(((uintptr_t)y & 15) == 0 && ((uintptr_t)x & 15) == 0, "npd_mc_generate: x and y must be 16-byte aligned");
    NPD_ARG(B <= (int64_t)0x7fffffff * 256, "npd_mc_generate: B too large for one call");
    hipStream_t s = (hipStream_t)stream;
    switch (code->p.N) {
        case 4: return mc_gen_launch<4>(code, msg, x, y, B, sigma, seed, snr_index, cw_offset, s);
        case 8: return mc_gen_launch<8>(code, msg, x, y, B, sigma, seed, snr_index, cw_offset, s);
        case 16: return mc_gen_launch<16>(code, msg, x, y, B, sigma, seed, snr_index, cw_offset, s);
        case 32: return mc_gen_launch<32>(code, msg, x, y, B, sigma, seed, snr_index, cw_offset, s);
        case 64: return mc_gen_launch<64>(code, msg, x, y, B, sigma, seed, snr_index, cw_offset, s);
        case 128: return mc_gen_launch<128>(code, msg, x, y, B, sigma, seed, snr_index, cw_offset, s);
        case 256: return mc_gen_launch<256>(code, msg, x, y, B, sigma, seed, snr_index, cw_offset, s);
        default: return fail(NPD_EINVAL, "npd_mc_generate: unsupported N");
    }
}

static int count_launch(gen::CountArgs& a, hipStream_t s) {
    const int64_t groups = (a.B + 15) / 16;  // 4 waves x 4 rows in flight
    const int grid = grid_for(groups, 8, device_cu_count());
    hipLaunchKernelGGL(gen::count_errors_kernel, dim3(grid), dim3(256), 0, s, a);
    return launch_check("count_errors_kernel launch");
}

extern "C" int npd_count_errors(const float* ref, const float* hat, int64_t B, int K, unsigned long long* counters,
                                void* stream) {
    NPD_ARG(B >= 0 && K >= 0, "npd_count_errors: negative size");
    NPD_ARG(counters != nullptr, "npd_count_errors: counters is NULL");
    if (B == 0 || K == 0) return NPD_OK;
    NPD_ARG(ref != nullptr && hat != nullptr, "npd_count_errors: null pointer");
    gen::CountArgs a{};
    a.ref = ref;
    a.hat = hat;
    a.counters = counters;
    a.B = B;
    a.K = K;
    a.W = K;
    a.use_cols = 0;
    return count_launch(a, (hipStream_t)stream);
}

extern "C" int npd_count_errors_cols(const float* ref, const float* hat, int64_t B, int K, int W, const int32_t* cols,
                                     unsigned long long* counters, void* stream) {
    NPD_ARG(B >= 0 && K >= 0 && W >= 0, "npd_count_errors_cols: negative size");
    NPD_ARG(counters != nullptr && cols != nullptr, "npd_count_errors_cols: NULL counters / cols");
    NPD_ARG(K <= kMaxN, "npd_count_errors_cols: K <= 256");
    if (B == 0 || K == 0) return NPD_OK;
    NPD_ARG(ref != nullptr && hat != nullptr, "npd_count_errors_cols: null pointer");
    gen::CountArgs a{};
    for (int k = 0; k < K; ++k) {
        NPD_ARG(cols[k] >= 0 && cols[k] < W, "npd_count_errors_cols: column out of range");
        a.cols[k] = cols[k];
    }
    a.ref = ref;
    a.hat = hat;
    a.counters = counters;
    a.B = B;
    a.K = K;
    a.W = W;
    a.use_cols = 1;
    return count_launch(a, (hipStream_t)stream);
}

extern "C" int npd_count_errors_masked(const float* ref, const float* hat, const int64_t* mask, int64_t B, int K,
                                       unsigned long long* counters, void* stream) {
    NPD_ARG(B >= 0 && K >= 0, "npd_count_errors_masked: negative size");
    NPD_ARG(counters != nullptr, "npd_count_errors_masked: counters is NULL");
    if (B == 0 || K == 0) return NPD_OK;
    NPD_ARG(ref != nullptr && hat != nullptr && mask != nullptr, "npd_count_errors_masked: null pointer");
    const int64_t n = B * (int64_t)K;
    const int grid = grid_for((n + 255) / 256, 4, device_cu_count());
    hipLaunchKernelGGL(gen::count_errors_masked_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, ref, hat, mask, n,
                       counters);
    return launch_check("count_errors_masked_kernel launch");
}
