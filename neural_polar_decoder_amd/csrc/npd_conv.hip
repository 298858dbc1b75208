// npd_conv.hip -- convNet decoder (models.py:691-772) on MFMA.
//
// Reference forward (models.py:742-767): 10 dilated Conv1d(k=7) + GELU with three residual blocks,
// flatten (c*N + l), Linear(E*N -> 4N) + GELU, Linear(4N -> N) + GELU, Linear(N -> N), Dropout (eval:
// identity), LayerNorm(N, eps 1e-6), decisions = sign(logits).
//
// MI355X mapping (fp32 path, v_mfma_f32_32x32x2_f32, exact fp32 FMA chains):
//   * conv layer = implicit GEMM  out[co][l] = sum_{t,ci} W[co][ci][t] * in[ci][l + d(t-3)]:
//     MFMA rows = output channels (A = weights, pre-permuted on the host into A-operand order,
//     k = t*Cin + ci), columns = positions (B = the input slab staged in LDS with its zero halo);
//     the epilogue fuses bias + GELU (+ residual) and writes 32 consecutive positions per register.
//   * FC layers = LDS-tiled GEMM with MFMA rows = codewords, columns = output features (so the
//     epilogue writes contiguous feature runs), bias + GELU fused.
//   * LayerNorm + sign: one wave per codeword.
// Activations of a chunk of codewords live in a caller-provided workspace, (B, N, C) (channels
// contiguous); FC0's weights are permuted on the host to that flatten order.
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <type_traits>
#include <vector>

#include "npd_common.hpp"

namespace npd {
namespace conv {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

constexpr int kLayers = 10;
constexpr int kChunk = 8192;  // codewords per pass through the layer pipeline (FC0: 256-row tiles fill 256 CUs)

struct LayerDesc {
    int cin, cout, dil;
    int res;        // 1: add the block input (residual) after GELU
    int64_t woff;   // offset (floats) of the permuted weights in the device image
    int64_t boff;   // offset of the bias
    int ksteps;     // ceil(7*cin / 2)
    // fp16x3 split (precision 3, cin > 1): weight image offset (floats) and the weight scale exponent SW (the kernels
    // descale the accumulators by 2^-(SW + SA), SA from the input activations' range)
    int64_t soff;
    int sw;
    int64_t soff16;  // cin 32 / 64: the same split weights as 16x16x32 A fragments (conv_ws16_kernel), else -1
};

// fp16x3: activations are split as fp16(a 2^SA) + fp16(a 2^SA - hi) when staged: SA = 4 (lo normal for |a| >= 2^-7,
// below that lo's absolute resolution is 2^-28) while max |a| < 2^11, lower where a layer's inputs reach further
// (split_sa: max |a| 2^SA < 2^15, so hi cannot overflow fp16); the weights of each layer are scaled by 2^SW on the host
// so that max |w| 2^SW is in [2^12, 2^13) (hi and lo normal for |w| >= max |w| 2^-11)
constexpr int kSplitSA = 4;



__device__ __forceinline__ float gelu(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f)); }

// The max |a| of one activation is kept in kAmaxSpread words kAmaxStride words apart (4 KB): each producing wave
// atomicMax-es one of them (by block and wave), so tens of thousands of small blocks (layer 0) do not serialise on one
// address; a consumer reads all of them with one load per lane and reduces over the wave.
constexpr int kAmaxSpread = 64;
constexpr int kAmaxStride = 16;
constexpr int kAmaxWords = kAmaxSpread * kAmaxStride;  // per activation

// max over a full wave, returned wave-uniform: DPP within rows of 16 lanes, then the 4 row results by readlane
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false));  // row_half_mirror
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false));  // row_mirror
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 0), r1 = (uint32_t)__builtin_amdgcn_readlane((int)v, 16);
    const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)v, 32), r3 = (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
    return max(max(r0, r1), max(r2, r3));
}

__device__ __forceinline__ int split_sa(const uint32_t* amax) {
    if (amax == nullptr) return kSplitSA;
    const uint32_t m = wave_max_u32(__builtin_nontemporal_load(amax + (threadIdx.x & 63) * kAmaxStride));
    const int e = (int)((m >> 23) & 0xFFu) - 126;  // max |a| < 2^e
    return min(kSplitSA, 15 - e);
}

__device__ __forceinline__ float amax4(const f4& v) {
    return fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
}

// max over the wave of m (m >= 0, not NaN), then one atomicMax of its bits (non-negative floats order as unsigned
// integers)
__device__ __forceinline__ void publish_amax(uint32_t* amax, float m) {
    const uint32_t w = wave_max_u32(__float_as_uint(m));
    if ((threadIdx.x & 63) == 0) {
        const uint32_t blk = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
        atomicMax(amax + ((blk * 8 + (threadIdx.x >> 6)) % kAmaxSpread) * kAmaxStride, w);
    }
}

__device__ __forceinline__ f16v mfma(float a, float b, const f16v& c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// ------------------------------------------------------------------------------ conv layer
// Activations are (B, N, C) -- channels contiguous per position -- so a block's input slab (64 positions
// plus the dilation halo, all channels) is one contiguous run in HBM (16-B loads) and lands in LDS as
// [position][channel] rows of stride CS = cin + 4 (16-B aligned, conflict-free ds_read_b128 across the
// 32 position columns of a wave).  MFMA k-steps run tap by tap; within tap t, k-step s pairs channel s
// (lane half 0) with channel s + cin/2 (half 1), so the B operands of 4 consecutive k-steps are one
// ds_read_b128 and the A operands (weights, permuted on the host in the same order) one 16-B load.
// The accumulator's registers 4q..4q+3 hold 4 consecutive output channels of one position: bias, GELU,
// residual and the store are 16-B vectors.  Layer 0 (cin = 1): the 7 taps are the k-steps (padded to 8).
// grid: (N/64 position tiles, cout_pad/64 channel tiles, codewords); block 256 = 2 (co) x 2 (pos) waves.
template <bool CIN1>
__global__ __launch_bounds__(256) void conv_layer_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                         const float* __restrict__ res, const float* __restrict__ wimg,
                                                         const float* __restrict__ bias, int cin, int cout, int N,
                                                         int dil, int do_res, uint32_t* __restrict__ amax_out) {
    extern __shared__ __attribute__((aligned(16))) float slab[];
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, col = lane & 31;
    const int l0 = blockIdx.x * 64;
    const int64_t b = blockIdx.z;
    const int halo = 3 * dil;
    const int W = 64 + 2 * halo;
    const int CS = CIN1 ? 4 : cin + 4;
    if constexpr (CIN1) {
        const float* inb = in + b * (int64_t)N;
        for (int p = tid; p < W; p += 256) {
            const int l = l0 - halo + p;
            slab[p * CS] = (l >= 0 && l < N) ? inb[l] : 0.0f;
        }
    } else {
        const int c4n = cin >> 2;
        const f4* inb = reinterpret_cast<const f4*>(in + b * (int64_t)N * cin);
        for (int e = tid; e < W * c4n; e += 256) {
            const int p = e / c4n, c4 = e - p * c4n;
            const int l = l0 - halo + p;
            const f4 v = (l >= 0 && l < N) ? inb[(int64_t)l * c4n + c4] : f4{0.f, 0.f, 0.f, 0.f};
            *reinterpret_cast<f4*>(slab + p * CS + 4 * c4) = v;
        }
    }
    __syncthreads();
    const int co_sub = wave & 1, pos_sub = wave >> 1;
    const int co_t32 = blockIdx.y * 2 + co_sub;  // 32-channel tile index
    const int pcol = pos_sub * 32 + col;
    f16v acc = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if constexpr (CIN1) {
        const f4 w = reinterpret_cast<const f4*>(wimg)[co_t32 * 64 + lane];
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
            const int t = 2 * s2 + h;
            const float bv = t < 7 ? slab[(pcol + dil * t) * CS] : 0.0f;
            acc = mfma(w[s2], bv, acc);
        }
    } else {
        const int ng = cin >> 3;  // groups of 4 k-steps per tap
        const f4* wq = reinterpret_cast<const f4*>(wimg) + (int64_t)co_t32 * 7 * ng * 64 + lane;
        f4 wn = wq[0];
#pragma unroll
        for (int t = 0; t < 7; ++t) {
            const f4* brow = reinterpret_cast<const f4*>(slab + (pcol + dil * t) * CS + h * (cin >> 1));
            for (int g = 0; g < ng; ++g) {
                const f4 w = wn;
                const int nxt = t * ng + g + 1;
                if (nxt < 7 * ng) wn = wq[nxt * 64];
                const f4 bv = brow[g];
                acc = mfma(w.x, bv.x, acc);
                acc = mfma(w.y, bv.y, acc);
                acc = mfma(w.z, bv.z, acc);
                acc = mfma(w.w, bv.w, acc);
            }
        }
    }
    // epilogue: registers 4q..4q+3 = channels co_t32*32 + 8q + 4h + 0..3 at position l0 + pcol
    const int l = l0 + pcol;
    float amx = 0.0f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int co = co_t32 * 32 + 8 * q + 4 * h;
        if (co < cout) {
            const int64_t o = (b * N + l) * (int64_t)cout + co;
            const f4 bb = *reinterpret_cast<const f4*>(bias + co);
            f4 v;
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = gelu(acc[4 * q + e] + bb[e]);
            if (do_res) {
                const f4 rv = *reinterpret_cast<const f4*>(res + o);
                v += rv;
            }
            *reinterpret_cast<f4*>(out + o) = v;
            amx = fmaxf(amx, amax4(v));
        }
    }
    if (amax_out != nullptr) publish_amax(amax_out, amx);
}

// ------------------------------------------------------------------------------ conv layer, fp16x3
// precision 3 (cin > 1): the same implicit GEMM on v_mfma_f32_32x32x16_f16 with hi + lo fp16 operands, three
// products per multiply (hi.hi + hi.lo + lo.hi), fp32 accumulation -- 16 channels of one tap per MFMA triple instead
// of 8 fp32 MFMAs of 2 channels: 96 against 512 MFMA cycles per tap-group.  32x32x16 operand map (lane l, r = l&31,
// h = l>>5): A[row r][k = 8h + j], B[k = 8h + j][col r], j = 0..7; k-step s of tap t covers channels 16s + k.
// The slab is split once when staged: LDS holds a hi plane and a lo plane of fp16 rows [position][channel] of stride
// CSH = cin16 + 8 (cin16 = cin rounded up to 16, the pad channels zero), so a B fragment (8 channels) is one
// ds_read_b128 per plane.  Each wave owns 32 output channels x P position tiles: an A fragment pair (global, 2 x 16 B)
// feeds P MFMA triples, which divides the weight stream by P.  Block: 2 (co) x 2 (position) waves, 64 P positions.
// Epilogue (registers 4q..4q+3 = 4 consecutive channels, as conv_layer_kernel) after the exact descale 2^-(SW+SA).
typedef _Float16 hf8 __attribute__((ext_vector_type(8)));
typedef _Float16 hf4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f16v mfma16(const hf8& a, const hf8& b, const f16v& c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

template <int P>
__global__ __launch_bounds__(256) void conv_layer_split_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                               const float* __restrict__ res, const f4* __restrict__ wimg,
                                                               const float* __restrict__ bias, int cin, int cout, int N,
                                                               int dil, int do_res, int sw,
                                                               const uint32_t* __restrict__ amax_in,
                                                               uint32_t* __restrict__ amax_out) {
    extern __shared__ __attribute__((aligned(16))) _Float16 slab16[];
    const int sa = split_sa(amax_in);
    const float sa_scale = __builtin_ldexpf(1.0f, sa), descale = __builtin_ldexpf(1.0f, -(sw + sa));
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, col = lane & 31;
    constexpr int PT = 64 * P;  // positions per block
    const int l0 = blockIdx.x * PT;
    const int64_t b = blockIdx.z;
    const int halo = 3 * dil;
    const int W = PT + 2 * halo;
    const int cin16 = (cin + 15) & ~15;
    const int CSH = cin16 + 8;
    _Float16* const hiP = slab16;
    _Float16* const loP = slab16 + (size_t)W * CSH;
    {
        // stage + split: 4 channels per element (cin is a multiple of 8), pad channels of each row zeroed
        const int c4n = cin >> 2, c4p = cin16 >> 2;
        const f4* inb = reinterpret_cast<const f4*>(in + b * (int64_t)N * cin);
        for (int e = tid; e < W * c4p; e += 256) {
            const int p = e / c4p, c4 = e - p * c4p;
            const int l = l0 - halo + p;
            f4 v = f4{0.f, 0.f, 0.f, 0.f};
            if (c4 < c4n && l >= 0 && l < N) v = inb[(int64_t)l * c4n + c4];
            hf4 hi, lo;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float x = v[j] * sa_scale;
                hi[j] = (_Float16)x;
                lo[j] = (_Float16)(x - (float)hi[j]);
            }
            *reinterpret_cast<hf4*>(hiP + p * CSH + 4 * c4) = hi;
            *reinterpret_cast<hf4*>(loP + p * CSH + 4 * c4) = lo;
        }
    }
    __syncthreads();
    const int co_sub = wave & 1, pos_sub = wave >> 1;
    const int co_t32 = blockIdx.y * 2 + co_sub;  // 32-channel tile index
    const int ng = cin16 >> 4;                   // 16-channel k-steps per tap
    f16v acc[P];
#pragma unroll
    for (int p = 0; p < P; ++p) acc[p] = f16v{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // A fragments: [t32][tap][s][part][lane] 16 B
    const f4* wq = wimg + (int64_t)co_t32 * 7 * ng * 128 + lane;
    f4 whn = wq[0], wln = wq[64];
    const int pbase = pos_sub * 32 * P + col;  // this lane's position column within the block, tile 0
    float amx = 0.0f;
    for (int t = 0; t < 7; ++t) {
        for (int g = 0; g < ng; ++g) {
            const hf8 ah = __builtin_bit_cast(hf8, whn), al = __builtin_bit_cast(hf8, wln);
            const int nxt = t * ng + g + 1;
            if (nxt < 7 * ng) {
                whn = wq[(int64_t)nxt * 128];
                wln = wq[(int64_t)nxt * 128 + 64];
            }
#pragma unroll
            for (int p = 0; p < P; ++p) {
                const int off = (pbase + 32 * p + dil * t) * CSH + 16 * g + 8 * h;
                const hf8 bh = *reinterpret_cast<const hf8*>(hiP + off);
                const hf8 bl = *reinterpret_cast<const hf8*>(loP + off);
                acc[p] = mfma16(ah, bh, acc[p]);
                acc[p] = mfma16(ah, bl, acc[p]);
                acc[p] = mfma16(al, bh, acc[p]);
            }
        }
    }
#pragma unroll
    for (int p = 0; p < P; ++p) {
        const int l = l0 + pos_sub * 32 * P + 32 * p + col;
        if (l >= N) continue;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int co = co_t32 * 32 + 8 * q + 4 * h;
            if (co < cout) {
                const int64_t o = (b * N + l) * (int64_t)cout + co;
                const f4 bb = *reinterpret_cast<const f4*>(bias + co);
                f4 v;
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = gelu(fmaf(acc[p][4 * q + e], descale, bb[e]));
                if (do_res) {
                    const f4 rv = *reinterpret_cast<const f4*>(res + o);
                    v += rv;
                }
                *reinterpret_cast<f4*>(out + o) = v;
                amx = fmaxf(amx, amax4(v));
            }
        }
    }
    if (amax_out != nullptr) publish_amax(amax_out, amx);
}

// ------------------------------------------------------------------------------ conv layer, fp16x3, weight-stationary
// The same products as conv_layer_split_kernel, reorganised so that nothing but activations streams: a persistent
// block (one per CU) keeps its waves' weight slices in registers for the whole layer and walks (codeword, 64 Q-position
// chunk) items.  NW waves = 2 (32 output channels each) x KS channel parts x NW / 2 / KS position parts; a wave holds
// 32 channels x 7 taps x NG / KS 16-channel groups, hi and lo (56 NG / KS VGPRs).  NW = 8 (cin 64 / 96 / 128, KS 2 or
// 4) keeps every wave under 256 registers, so two waves share each SIMD and one's MFMAs cover the other's LDS reads;
// the KS channel parts of a tile hand each other their partial sums through LDS and the tile's finishing wave adds
// them.  NW = 4, KS = 1 for cin <= 48.  The next item's slab (positions plus the dilation halo, all channels, fp32) is
// fetched into registers before the current item's MFMAs and split into the other half of a double-buffered fp16
// hi / lo LDS slab after them, so HBM reads overlap the matrix work and no weight fragment is re-read.  Dilation <= 4
// (conv_spec) bounds the halo at 12.
template <int NG, int Q, int KS, int NW>
__global__ __launch_bounds__(64 * NW, (NW == 4 && KS == 2) ? 2 : 1) void conv_split_ws_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                                const float* __restrict__ res,
                                                                const f4* __restrict__ wimg,
                                                                const float* __restrict__ bias, int cin, int cout,
                                                                int N, int dil, int do_res, int sw,
                                                                const uint32_t* __restrict__ amax_in,
                                                                uint32_t* __restrict__ amax_out, int64_t nb, int nslices) {
    extern __shared__ __attribute__((aligned(16))) _Float16 slab16[];
    const int sa = split_sa(amax_in);
    const float sa_scale = __builtin_ldexpf(1.0f, sa), descale = __builtin_ldexpf(1.0f, -(sw + sa));
    float amx = 0.0f;
    constexpr int NT = 64 * NW;
    constexpr int PT = 64 * Q;        // positions per item (2 Q tiles of 32)
    constexpr int C4P = 4 * NG;       // float4 channel groups per staged row (pad channels zero)
    constexpr int CSH = 16 * NG + 8;  // fp16 row stride of the LDS slab
    constexpr int MAXE = ((PT + 24) * C4P + NT - 1) / NT;
    constexpr int NGW = NG / KS;      // channel groups per wave
    constexpr int PS = NW / 2 / KS;   // position parts
    constexpr int TPW = 2 * Q / PS;   // 32-position tiles per wave
    static_assert(NG % KS == 0 && (NW / 2) % KS == 0 && (2 * Q) % PS == 0, "wave decomposition");
    // partial-sum slots per wave: KS = 2 with 2 tiles hands over exactly one (slot 0), else slot = tile
    constexpr int RS = (KS == 2 && TPW == 2) ? 1 : TPW;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, col = lane & 31;
    const int co_sub = wave & 1, rest = wave >> 1;
    const int kp = rest % KS, pp = rest / KS;
    const int g0 = kp * NGW;
    const int halo = 3 * dil;
    const int W = PT + 2 * halo;
    const int plane = W * CSH;
    const int c4n = cin >> 2;
    const int slice = blockIdx.x % nslices;
    const int co_t32 = slice * 2 + co_sub;
    hf8 ah[7][NGW], al[7][NGW];
    {
        const f4* wq = wimg + (int64_t)co_t32 * 7 * NG * 128 + lane;
#pragma unroll
        for (int t = 0; t < 7; ++t)
#pragma unroll
            for (int g = 0; g < NGW; ++g) {
                ah[t][g] = __builtin_bit_cast(hf8, wq[(t * NG + g0 + g) * 128]);
                al[t][g] = __builtin_bit_cast(hf8, wq[(t * NG + g0 + g) * 128 + 64]);
            }
    }
    // KS > 1: partial sums of the channel parts, [wave][tile][register][lane]
    float* const red = reinterpret_cast<float*>(slab16 + (size_t)4 * plane);
    const int chunks = N / PT;
    const int64_t items = nb * chunks;
    const int64_t stride = gridDim.x / nslices;
    int64_t item = blockIdx.x / nslices;
    f4 pre[MAXE];
    auto fetch = [&](int64_t it) {
        const int64_t b = it / chunks;
        const int l0 = (int)(it - b * chunks) * PT;
        const f4* inb = reinterpret_cast<const f4*>(in + b * (int64_t)N * cin);
#pragma unroll
        for (int e = 0; e < MAXE; ++e) {
            const int idx = tid + NT * e;
            const int p = idx / C4P, c4 = idx - p * C4P;
            const int l = l0 - halo + p;
            f4 v = f4{0.f, 0.f, 0.f, 0.f};
            if (p < W && c4 < c4n && l >= 0 && l < N) v = inb[(int64_t)l * c4n + c4];
            pre[e] = v;
        }
    };
    auto stash = [&](int buf) {
        _Float16* const hiP = slab16 + (size_t)buf * 2 * plane;
#pragma unroll
        for (int e = 0; e < MAXE; ++e) {
            const int idx = tid + NT * e;
            const int p = idx / C4P, c4 = idx - p * C4P;
            if (p < W) {
                hf4 hi, lo;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float x = pre[e][j] * sa_scale;
                    hi[j] = (_Float16)x;
                    lo[j] = (_Float16)(x - (float)hi[j]);
                }
                *reinterpret_cast<hf4*>(hiP + p * CSH + 4 * c4) = hi;
                *reinterpret_cast<hf4*>(hiP + plane + p * CSH + 4 * c4) = lo;
            }
        }
    };
    if (item < items) {
        fetch(item);
        stash(0);
    }
    __syncthreads();
    int buf = 0;
    const int tbase = pp * 32 * TPW + col;  // this lane's position column of its first tile within the item
    // KS = 2, two tiles per wave (the 64-channel layers): each wave finishes tile kp; its residual quads are loaded
    // before the MFMAs (one item of HBM latency hidden) instead of in the epilogue (measured +18 % on residual layers)
    constexpr bool PRE_RES = KS == 2 && TPW == 2;
    for (; item < items; item += stride) {
        const int64_t nxt = item + stride;
        if (nxt < items) fetch(nxt);
        f4 resq[4];
        if constexpr (PRE_RES) {
            if (do_res) {
                const int64_t b = item / chunks;
                const int l = (int)(item - b * chunks) * PT + tbase + 32 * kp;
#pragma unroll
                for (int r4 = 0; r4 < 4; ++r4) {
                    const int co = co_t32 * 32 + 8 * r4 + 4 * h;
                    if (co < cout) resq[r4] = *reinterpret_cast<const f4*>(res + (b * N + l) * (int64_t)cout + co);
                }
            }
        }
        const _Float16* const hiP = slab16 + (size_t)buf * 2 * plane;
        const _Float16* const loP = hiP + plane;
        f16v acc[TPW];
#pragma unroll
        for (int q = 0; q < TPW; ++q)
            acc[q] = f16v{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 7; ++t)
#pragma unroll
            for (int g = 0; g < NGW; ++g)
#pragma unroll
                for (int q = 0; q < TPW; ++q) {
                    const int off = (tbase + 32 * q + dil * t) * CSH + 16 * (g0 + g) + 8 * h;
                    const hf8 bh = *reinterpret_cast<const hf8*>(hiP + off);
                    const hf8 bl = *reinterpret_cast<const hf8*>(loP + off);
                    acc[q] = mfma16(ah[t][g], bh, acc[q]);
                    acc[q] = mfma16(ah[t][g], bl, acc[q]);
                    acc[q] = mfma16(al[t][g], bh, acc[q]);
                }
        // tile q of the (co_sub, pp) group is finished by channel part q % KS
        if constexpr (KS > 1) {
#pragma unroll
            for (int q = 0; q < TPW; ++q)
                if (q % KS != kp)
#pragma unroll
                    for (int r = 0; r < 16; ++r) red[((wave * RS + (RS == 1 ? 0 : q)) * 16 + r) * 64 + lane] = acc[q][r];
            __syncthreads();
#pragma unroll
            for (int q = 0; q < TPW; ++q)
                if (q % KS == kp)
#pragma unroll
                    for (int k = 1; k < KS; ++k) {
                        const int other = co_sub + 2 * ((kp + k) % KS + KS * pp);
#pragma unroll
                        for (int r = 0; r < 16; ++r)
                            acc[q][r] += red[((other * RS + (RS == 1 ? 0 : q)) * 16 + r) * 64 + lane];
                    }
        }
        const int64_t b = item / chunks;
        const int l0 = (int)(item - b * chunks) * PT;
#pragma unroll
        for (int q = 0; q < TPW; ++q) {
            if (q % KS != kp) continue;
            const int l = l0 + tbase + 32 * q;
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4) {
                const int co = co_t32 * 32 + 8 * r4 + 4 * h;
                if (co < cout) {
                    const int64_t o = (b * N + l) * (int64_t)cout + co;
                    const f4 bb = *reinterpret_cast<const f4*>(bias + co);
                    f4 v;
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = gelu(fmaf(acc[q][4 * r4 + e], descale, bb[e]));
                    if (do_res) {
                        if constexpr (PRE_RES) v += resq[r4];
                        else v += *reinterpret_cast<const f4*>(res + o);
                    }
                    *reinterpret_cast<f4*>(out + o) = v;
                    amx = fmaxf(amx, amax4(v));
                }
            }
        }
        if (nxt < items) stash(buf ^ 1);
        __syncthreads();
        buf ^= 1;
    }
    if (amax_out != nullptr) publish_amax(amax_out, amx);
}

// LDS bytes of conv_split_ws_kernel: two slab buffers (hi + lo planes) and, for KS > 1, the partial-sum exchange
static size_t ws_lds_bytes(int ng, int Q, int ks, int nw, int dil) {
    const size_t slabs = (size_t)2 * 2 * (64 * Q + 6 * dil) * (16 * ng + 8) * 2;
    const int tpw = 2 * Q / (nw / 2 / ks);
    const int rs = (ks == 2 && tpw == 2) ? 1 : tpw;
    return slabs + (ks > 1 ? (size_t)nw * rs * 16 * 64 * 4 : 0);
}

// ------------------------------------------------------------------------------ conv layer, fp16x3, 16-row tiles
// cin = 32 KB (KB = 1, 2, 4): the weight-stationary kernel on v_mfma_f32_16x16x32_f16.  A 16-row tile of output
// channels needs 7 taps x KB K blocks x (hi, lo) A fragments = 56 KB registers per wave (112 at cin 64), so at cin <= 64
// each wave holds ALL input channels of its 16 output channels -- no channel parts, no partial-sum exchange through LDS
// and no second barrier, which is what held conv_split_ws_kernel's 64-channel layers at ~0.4 of the MFMA rate (its
// 32-row tiles need 224 registers for all 64 channels, hence the 2 parts).  8 waves = 4 x 16 output channels (a
// 64-channel slice) x 2 position halves of a 64 Q-position item (TPW = 2 Q 16-position tiles per wave); at cin 128
// (KP = 2) the two halves are channel parts instead, each finishing half of the item's tiles with the other's 16-B
// partial sums from LDS.  16x16x32 operand map (lane l = 16 g + c): A[row c][k 8g + j], B[k 8g + j][col c],
// D[row 4g + i][col c]; k of K block kb = channel 32 kb + k, so a B fragment is 8 channels of one slab row: one
// ds_read_b128 per plane from the double-buffered hi / lo slab, and the accumulator's 4 registers are 4 consecutive
// channels of one position (16-B epilogue stores).  The next item's slab is fetched into registers before the MFMAs
// and split into the other buffer after them, the residual of this item before them; one barrier per item (two with
// channel parts).
__device__ __forceinline__ f4 mfma16x32(const hf8& a, const hf8& b, const f4& c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// A/B switches: waves per block (8: one block per CU; 4: two) and 128-position items where N allows (1) -- measured
// 234 us (8, 1) / 245 us (4, 0) / 253 us (8, 1, CIN + 8 rows) per 64-channel layer per 4096 codewords
#ifndef NPD_WS16_NW
#define NPD_WS16_NW 8
#endif
#ifndef NPD_WS16_Q2
#define NPD_WS16_Q2 1
#endif
#ifndef NPD_WS16_PAD
#define NPD_WS16_PAD 16
#endif
#ifndef NPD_WS16_128
#define NPD_WS16_128 1  // the 128-channel layer on conv_ws16_kernel<4, 1, 8, 2> (0: conv_split_ws_kernel<8, 1, 4, 8>)
#endif
template <int KB, int Q, int NW, int KP>
__global__ __launch_bounds__(64 * NW, 8 / NW) void conv_ws16_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                           const float* __restrict__ res, const f4* __restrict__ wimg,
                                                           const float* __restrict__ bias, int cout, int N, int dil,
                                                           int do_res, int sw, const uint32_t* __restrict__ amax_in,
                                                           uint32_t* __restrict__ amax_out, int64_t nb, int nslices) {
    extern __shared__ __attribute__((aligned(16))) _Float16 slab16[];
    constexpr int NT = 64 * NW;
    constexpr int CIN = 32 * KB;
    constexpr int PT = 64 * Q;        // positions per item
    constexpr int C4P = CIN / 4;      // float4 channel groups per staged row
    // fp16 row stride of the LDS slab: CIN + 16 halfs.  A B fragment read (lane 16 g + c: row c, channels 8 g ..) puts
    // rows c at c * CSH / 8 16-B units and g at +g units; with CIN + 8 (36 / 20 dwords) ds_read_b128's lane groups
    // {0-3, 12-15, 20-27}, ... collided 2-way (PMC: SQ_LDS_BANK_CONFLICT 0.48 of SQ_LDS_IDX_ACTIVE), with CIN + 16
    // (40 / 24 dwords) every group hits 16 distinct units
    constexpr int CSH = CIN + NPD_WS16_PAD;
    constexpr int MAXE = ((PT + 24) * C4P + NT - 1) / NT;
    constexpr int PP = NW / 4 / KP;   // position parts
    constexpr int TPW = 4 * Q / PP;   // 16-position tiles per wave
    constexpr int KBW = KB / KP;      // K blocks (32 input channels) per wave
    static_assert((NW == 4 || NW == 8) && PP >= 1 && KB % KP == 0 && TPW % KP == 0, "wave decomposition");
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, col = lane & 15;
    const int co16 = wave & 3, kp = (wave >> 2) % KP, pp = (wave >> 2) / KP;
    const int halo = 3 * dil;
    const int W = PT + 2 * halo;
    const int plane = W * CSH;
    const int slice = blockIdx.x % nslices;
    const int t16 = slice * 4 + co16;  // 16-channel output tile
    const int sa = split_sa(amax_in);
    const float sa_scale = __builtin_ldexpf(1.0f, sa), descale = __builtin_ldexpf(1.0f, -(sw + sa));
    hf8 ah[7][KBW], al[7][KBW];
    {
        const f4* wq = wimg + (int64_t)t16 * 7 * KB * 128 + lane;
#pragma unroll
        for (int t = 0; t < 7; ++t)
#pragma unroll
            for (int kb = 0; kb < KBW; ++kb) {
                ah[t][kb] = __builtin_bit_cast(hf8, wq[(t * KB + kp * KBW + kb) * 128]);
                al[t][kb] = __builtin_bit_cast(hf8, wq[(t * KB + kp * KBW + kb) * 128 + 64]);
            }
    }
    // KP = 2: the two channel parts of a 16-channel tile each finish half of its TPW position tiles, taking the other
    // part's partial sums (one 16-B accumulator per lane and tile) from LDS behind the slab
    f4* const red = reinterpret_cast<f4*>(slab16 + (size_t)4 * (PT + 24) * CSH);
    auto fin = [&](int q) { return q * KP / TPW == kp; };
    const int chunks = N / PT;
    const int items = (int)nb * chunks;
    const int stride = gridDim.x / nslices;
    int item = blockIdx.x / nslices;
    f4 pre[MAXE];
    auto fetch = [&](int it) {
        const int b = it / chunks;
        const int l0 = (it - b * chunks) * PT;
        const f4* inb = reinterpret_cast<const f4*>(in + (int64_t)b * N * CIN);
#pragma unroll
        for (int e = 0; e < MAXE; ++e) {
            const int idx = tid + NT * e;
            const int p = idx / C4P, c4 = idx - p * C4P;
            const int l = l0 - halo + p;
            f4 v = f4{0.f, 0.f, 0.f, 0.f};
            if (p < W && l >= 0 && l < N) v = inb[(int64_t)l * C4P + c4];
            pre[e] = v;
        }
    };
    auto stash = [&](int buf) {
        _Float16* const hiP = slab16 + (size_t)buf * 2 * plane;
#pragma unroll
        for (int e = 0; e < MAXE; ++e) {
            const int idx = tid + NT * e;
            const int p = idx / C4P, c4 = idx - p * C4P;
            if (p < W) {
                hf4 hi, lo;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float x = pre[e][j] * sa_scale;
                    hi[j] = (_Float16)x;
                    lo[j] = (_Float16)(x - (float)hi[j]);
                }
                *reinterpret_cast<hf4*>(hiP + p * CSH + 4 * c4) = hi;
                *reinterpret_cast<hf4*>(hiP + plane + p * CSH + 4 * c4) = lo;
            }
        }
    };
    if (item < items) {
        fetch(item);
        stash(0);
    }
    __syncthreads();
    int buf = 0;
    const int tbase = pp * 16 * TPW + col;  // this lane's position column of its first tile within the item
    const int co = t16 * 16 + 4 * g;        // the lane's 4 output channels
    const bool co_ok = co < cout;
    const f4 bb = co_ok ? *reinterpret_cast<const f4*>(bias + co) : f4{0.f, 0.f, 0.f, 0.f};
    float amx = 0.0f;
    for (; item < items; item += stride) {
        const int nxt = item + stride;
        if (nxt < items) fetch(nxt);
        const int b = item / chunks;
        const int64_t row0 = (int64_t)b * N + (item - b * chunks) * PT + tbase;  // output row of tile 0
        f4 resv[TPW];
        if (do_res && co_ok) {
#pragma unroll
            for (int q = 0; q < TPW; ++q)
                if (fin(q)) resv[q] = *reinterpret_cast<const f4*>(res + (row0 + 16 * q) * cout + co);
        }
        const _Float16* const hiP = slab16 + (size_t)buf * 2 * plane;
        const _Float16* const loP = hiP + plane;
        f4 acc[TPW];
#pragma unroll
        for (int q = 0; q < TPW; ++q) acc[q] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 7; ++t)
#pragma unroll
            for (int kb = 0; kb < KBW; ++kb)
#pragma unroll
                for (int q = 0; q < TPW; ++q) {
                    const int off = (tbase + 16 * q + dil * t) * CSH + 32 * (kp * KBW + kb) + 8 * g;
                    const hf8 bh = *reinterpret_cast<const hf8*>(hiP + off);
                    const hf8 bl = *reinterpret_cast<const hf8*>(loP + off);
                    acc[q] = mfma16x32(ah[t][kb], bh, acc[q]);
                    acc[q] = mfma16x32(ah[t][kb], bl, acc[q]);
                    acc[q] = mfma16x32(al[t][kb], bh, acc[q]);
                }
        if constexpr (KP > 1) {
            const int slot = (co16 * PP + pp) * KP;
#pragma unroll
            for (int q = 0; q < TPW; ++q)
                if (!fin(q)) red[((slot + kp) * TPW + q) * 64 + lane] = acc[q];
            __syncthreads();
#pragma unroll
            for (int q = 0; q < TPW; ++q)
                if (fin(q))
#pragma unroll
                    for (int o = 1; o < KP; ++o) acc[q] += red[((slot + (kp + o) % KP) * TPW + q) * 64 + lane];
        }
        if (co_ok) {
#pragma unroll
            for (int q = 0; q < TPW; ++q) {
                if (!fin(q)) continue;
                f4 v;
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = gelu(fmaf(acc[q][e], descale, bb[e]));
                if (do_res) v += resv[q];
                *reinterpret_cast<f4*>(out + (row0 + 16 * q) * cout + co) = v;
                amx = fmaxf(amx, amax4(v));
            }
        }
        if (nxt < items) stash(buf ^ 1);
        __syncthreads();
        buf ^= 1;
    }
    if (amax_out != nullptr) publish_amax(amax_out, amx);
}

// slab: 2 buffers x (hi, lo) x (64 Q + 6 dil) rows; KP = 2: + the partial sums, 8 waves x TPW tiles x 64 lanes x 16 B
// (the kernel places them after the dil = 4 slab)
static size_t ws16_lds_bytes(int kb, int Q, int dil, int kp) {
    const size_t slab = (size_t)2 * 2 * (64 * Q + 6 * (kp > 1 ? 4 : dil)) * (32 * kb + NPD_WS16_PAD) * 2;
    return slab + (kp > 1 ? (size_t)8 * (2 * Q * kp) * 64 * 16 : 0);
}

// ------------------------------------------------------------------------------ FC GEMM
// out[m][j] = act(sum_k X[m][k] * Wt[j][k] + bias[j]);  block tile 64 (m) x 64 (j), K step 32.
// LDS rows of stride GK + 4 (16-B aligned; 32 rows read with ds_read_b128 at one k offset hit every bank
// once per 16 lanes).  Within a K block, k-step s pairs k = s (lane half 0) with k = s + GK/2 (half 1),
// so the A and B operands of 4 consecutive k-steps are one ds_read_b128 each (round 1: two ds_read_b32
// per MFMA) and the tile lands in LDS with 16-B stores.
constexpr int GK = 32;
constexpr int GS = GK + 4;

__global__ __launch_bounds__(256) void fc_kernel(const float* __restrict__ X, const float* __restrict__ Wt,
                                                 const float* __restrict__ bias, float* __restrict__ out, int M, int K,
                                                 int Nout, int act) {
    __shared__ __attribute__((aligned(16))) float As[2][64 * GS];
    __shared__ __attribute__((aligned(16))) float Bs[2][64 * GS];
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, col = lane & 31;
    const int m0 = blockIdx.y * 64, j0 = blockIdx.x * 64;
    const int msub = wave & 1, jsub = wave >> 1;
    // loader mapping: 64 rows x 32 k = 512 float4 per operand; thread loads 2 float4 of A and of B
    f4 ra[2], rb[2];
    auto fetch = [&](int k0) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int idx = tid + 256 * u;  // 0..511
            const int r = idx >> 3, c4 = (idx & 7) * 4;
            int mr = m0 + r;
            if (mr >= M) mr = M - 1;
            ra[u] = *reinterpret_cast<const f4*>(X + (int64_t)mr * K + k0 + c4);
            rb[u] = *reinterpret_cast<const f4*>(Wt + (int64_t)(j0 + r) * K + k0 + c4);
        }
    };
    auto stash = [&](int buf) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int idx = tid + 256 * u;
            const int r = idx >> 3, c4 = (idx & 7) * 4;
            *reinterpret_cast<f4*>(&As[buf][r * GS + c4]) = ra[u];
            *reinterpret_cast<f4*>(&Bs[buf][r * GS + c4]) = rb[u];
        }
    };
    f16v acc = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const int nk = K / GK;
    fetch(0);
    stash(0);
    __syncthreads();
    for (int kb = 0; kb < nk; ++kb) {
        const int cur = kb & 1;
        if (kb + 1 < nk) fetch((kb + 1) * GK);
        const f4* as = reinterpret_cast<const f4*>(&As[cur][(msub * 32 + col) * GS + h * (GK / 2)]);
        const f4* bs = reinterpret_cast<const f4*>(&Bs[cur][(jsub * 32 + col) * GS + h * (GK / 2)]);
#pragma unroll
        for (int g = 0; g < GK / 8; ++g) {
            const f4 a = as[g], b = bs[g];
            acc = mfma(a.x, b.x, acc);
            acc = mfma(a.y, b.y, acc);
            acc = mfma(a.z, b.z, acc);
            acc = mfma(a.w, b.w, acc);
        }
        if (kb + 1 < nk) stash(cur ^ 1);
        __syncthreads();
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int m = m0 + msub * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int j = j0 + jsub * 32 + col;
        if (m < M) {
            float v = acc[r] + bias[j];
            if (act) v = gelu(v);
            out[(int64_t)m * Nout + j] = v;
        }
    }
}

// ------------------------------------------------------------------------------ FC GEMM, fp16x3
// precision 3: the same 64 x 64 block tile on v_mfma_f32_32x32x16_f16, hi + lo fp16 operands, three products per
// multiply, fp32 accumulation.  X (activations, fp32) is split as it is staged (x 2^SA); W arrives pre-split on the
// host (hi and lo planes of fp16(w 2^SW), same row-major (Nout, K) layout).  LDS: per buffer four fp16 planes (A hi,
// A lo, B hi, B lo) of 64 rows x 32 k, row stride 40 (16-B aligned, conflict-free row reads); k-step s of a 32-wide K
// block reads k = 16 s + 8 h .. + 7 (one ds_read_b128 per plane).  6 MFMAs of 32 cycles per K block per wave against
// 16 fp32 MFMAs of 64.  Epilogue: descale 2^-(SW+SA) (exact), bias, GELU.
constexpr int GS16 = GK + 8;

__global__ __launch_bounds__(256) void fc_split_kernel(const float* __restrict__ X, const uint16_t* __restrict__ Whi,
                                                       const uint16_t* __restrict__ Wlo, const float* __restrict__ bias,
                                                       float* __restrict__ out, int M, int K, int Nout, int act,
                                                       int sw, const uint32_t* __restrict__ amax_in,
                                                       uint32_t* __restrict__ amax_out) {
    __shared__ __attribute__((aligned(16))) _Float16 sm[2][4][64 * GS16];
    const int sa = split_sa(amax_in);
    const float sa_scale = __builtin_ldexpf(1.0f, sa), descale = __builtin_ldexpf(1.0f, -(sw + sa));
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, col = lane & 31;
    const int m0 = blockIdx.y * 64, j0 = blockIdx.x * 64;
    const int msub = wave & 1, jsub = wave >> 1;
    // loader: A 64 rows x 32 k fp32 = 512 f4 (2 per thread); B planes 64 x 32 fp16 = 256 x 16 B (1 per thread each)
    f4 ra[2];
    f4 rbh, rbl;
    auto fetch = [&](int k0) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int idx = tid + 256 * u;
            const int r = idx >> 3, c4 = (idx & 7) * 4;
            int mr = m0 + r;
            if (mr >= M) mr = M - 1;
            ra[u] = *reinterpret_cast<const f4*>(X + (int64_t)mr * K + k0 + c4);
        }
        const int r = tid >> 2, c8 = (tid & 3) * 8;
        rbh = *reinterpret_cast<const f4*>(Whi + (int64_t)(j0 + r) * K + k0 + c8);
        rbl = *reinterpret_cast<const f4*>(Wlo + (int64_t)(j0 + r) * K + k0 + c8);
    };
    auto stash = [&](int buf) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int idx = tid + 256 * u;
            const int r = idx >> 3, c4 = (idx & 7) * 4;
            hf4 hi, lo;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float x = ra[u][e] * sa_scale;
                hi[e] = (_Float16)x;
                lo[e] = (_Float16)(x - (float)hi[e]);
            }
            *reinterpret_cast<hf4*>(&sm[buf][0][r * GS16 + c4]) = hi;
            *reinterpret_cast<hf4*>(&sm[buf][1][r * GS16 + c4]) = lo;
        }
        const int r = tid >> 2, c8 = (tid & 3) * 8;
        *reinterpret_cast<f4*>(&sm[buf][2][r * GS16 + c8]) = rbh;
        *reinterpret_cast<f4*>(&sm[buf][3][r * GS16 + c8]) = rbl;
    };
    f16v acc = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const int nk = K / GK;
    fetch(0);
    stash(0);
    __syncthreads();
    const int ar = (msub * 32 + col) * GS16 + 8 * h, br = (jsub * 32 + col) * GS16 + 8 * h;
    for (int kb = 0; kb < nk; ++kb) {
        const int cur = kb & 1;
        if (kb + 1 < nk) fetch((kb + 1) * GK);
#pragma unroll
        for (int st = 0; st < GK / 16; ++st) {
            const hf8 ah = *reinterpret_cast<const hf8*>(&sm[cur][0][ar + 16 * st]);
            const hf8 al = *reinterpret_cast<const hf8*>(&sm[cur][1][ar + 16 * st]);
            const hf8 bh = *reinterpret_cast<const hf8*>(&sm[cur][2][br + 16 * st]);
            const hf8 bl = *reinterpret_cast<const hf8*>(&sm[cur][3][br + 16 * st]);
            acc = mfma16(ah, bh, acc);
            acc = mfma16(ah, bl, acc);
            acc = mfma16(al, bh, acc);
        }
        if (kb + 1 < nk) stash(cur ^ 1);
        __syncthreads();
    }
    float amx = 0.0f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int m = m0 + msub * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int j = j0 + jsub * 32 + col;
        if (m < M) {
            float v = fmaf(acc[r], descale, bias[j]);
            if (act) v = gelu(v);
            out[(int64_t)m * Nout + j] = v;
            amx = fmaxf(amx, fabsf(v));
        }
    }
    if (amax_out != nullptr) publish_amax(amax_out, amx);
}

// fp16x3 FC GEMM with a BM x 128 block tile, BM = 128 or 256 (Nout a multiple of 128: FC0 at every N, FC1 / FC2 from
// N = 128; K is E N, 4 N or N, always a multiple of 32).  Tiles are dealt XCD by XCD (blocks b, b + 8, ... share an XCD
// and its L2): the column tiles of one row block run on one XCD, so X -- FC0 streams 537 MB of it per 4096 codewords at
// configs[4] -- comes from HBM about once (PMC of this kernel: 1.79 GB fetched per 4096-codeword FC0 against the 1.61 GB
// floor of X once + W once per XCD, profiles/round6/pmc_fc_final.txt).  What bounds it is not settled by any single
// resource: with the loads replaced by constants it ran 0.62 ms per 4096 codewords, with the MFMAs removed 0.8 ms, both
// together ~1.0 ms; deeper register rings, padded or panel-major operands (round 5), conflict-free LDS stores, a
// 256-row tile (25 % fewer operand bytes per MFMA) and fragment reads pinned a k-step ahead (round 6,
// profiles/round6/fc_tile_ab.txt) all measured within +-5 %.  The loader waves' split VALU shares each SIMD's issue
// port with the MFMA wave beside it (copy-only loaders on pre-split X: -12 %, fc0_presplit_ab.txt).
constexpr int FB = 128;

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

// The waves are specialised (512 threads, two waves per SIMD): waves 0-3 only read fragments and issue MFMAs (64 x 64
// each, v_mfma_f32_32x32x16_f16, three per product); waves 4-7 only load, split (x 2^SA) and store.  The loaders keep
// FDL K blocks in flight in their registers and fill a 3-slot LDS ring two blocks ahead of the MFMA waves, which read
// the next block's first fragments during the current block's MFMAs; one LDS-only barrier per K block.  Against the
// round-4 kernel (4 waves each loading and computing, one per SIMD): 355-365 vs 386-412 us average over FC0-FC2.
#ifndef NPD_FC_FDL
#define NPD_FC_FDL 3
#endif
// workgroup barrier that orders LDS only: a __syncthreads() also waits for every global load in flight (vmcnt(0)),
// which would drain the loaders' register ring at each K block
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}
constexpr int kWspSlots = 3;
// LDS image of one K block: 64-B rows (32 halfs) with the 16-B chunk q of row r stored at chunk q ^ ((r >> 2) & 3).
// The MFMA waves' ds_read_b128 (lane -> row col, chunk 2 st + h) then hit all 64 banks in each of its 16-lane groups
// (rows r and r + 4 of a 256-B bank line differ in the swizzle), and the loaders' stores -- ds_write_b64 of 2 rows x
// 8 x 8 B per 16 lanes, ds_write_b128 of 2 rows x 4 x 16 B per 8 lanes -- cover the 32 write banks once (bank
// (a/4) mod 32: two 64-B rows).  Round 5's padded 80-B rows were conflict-free for the reads only (a third of FC0's
// LDS cycles were store conflicts, profiles/round6/pmc_fc_final.txt) and do not fit three 256-row slots in 160 KB.
__device__ __forceinline__ int wsp_off(int r, int c) { return r * 32 + ((((c >> 3) ^ (r >> 2)) & 3) << 3) + (c & 7); }
__host__ __device__ constexpr size_t fc_wsp_lds(int bm) { return (size_t)kWspSlots * (2 * bm + 2 * FB) * 32 * 2; }
// PRE: X arrives already split (fp16 hi / lo planes of X 2^SA, row-major like X, written by split_planes_kernel), so the
// loaders only copy: 16-B loads of both planes into 16-B LDS stores, no split VALU.
// BM: rows (codewords) per block tile, 128 or 256, x 128 output features.  BM = 256 moves X 32 KB + W 16 KB per K block
// for twice the 128-row tile's MFMAs (each MFMA wave owns 128 x 64, TM = 4: 128 accumulator registers, 248 VGPRs); it
// runs where the chunk gives >= one 256-row tile per CU (npd_conv_forward_ex) at the same speed as BM = 128.
template <int FDL, bool PRE, int BM>
__global__ __launch_bounds__(512, 1) void fc_split_wsp_kernel(const float* __restrict__ X, const uint16_t* __restrict__ Xhi,
                                                              const uint16_t* __restrict__ Xlo,
                                                              const uint16_t* __restrict__ Whi,
                                                              const uint16_t* __restrict__ Wlo,
                                                              const float* __restrict__ bias, float* __restrict__ out,
                                                              int M, int K, int Nout, int act, int sw,
                                                              const uint32_t* __restrict__ amax_in,
                                                              uint32_t* __restrict__ amax_out) {
    constexpr int GKT = 32, NS = kWspSlots;
    static_assert(FDL >= 2 && FDL % NS == 0, "the prologue stashes two K blocks; LDS slots repeat with the ring");
    static_assert(BM == 128 || BM == 256, "block tile rows");
    constexpr int NL = 256;                            // loader threads
    constexpr int A4 = PRE ? GKT / 8 : GKT / 4, B8 = GKT / 8;  // 16-B pieces per A row (per plane), per B row
    constexpr int UA = BM * A4 / NL, UB = FB * B8 / NL;
    constexpr int TM = BM / 64, TN = 2;
    constexpr int PA = BM * 32, PB = FB * 32;  // halfs per A plane, per B plane
    constexpr int SLOT = 2 * PA + 2 * PB;
    const uint32_t am_raw = amax_in != nullptr ? __builtin_nontemporal_load(amax_in + (threadIdx.x & 63) * kAmaxStride) : 0u;
    extern __shared__ __attribute__((aligned(16))) _Float16 smb[];  // [slot][A hi, A lo (BM rows), B hi, B lo (128)][32]
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const bool loader = wave >= 4;
    const int gx = Nout / FB;
    const int total = gridDim.x;
    int lin = blockIdx.x;
    if ((total & 7) == 0) lin = (blockIdx.x & 7) * (total >> 3) + (blockIdx.x >> 3);
    const int m0 = (lin / gx) * BM, j0 = (lin % gx) * FB;
    const int nk = K / GKT;
    const int sa = amax_in != nullptr ? min(kSplitSA, 15 - ((int)((wave_max_u32(am_raw) >> 23) & 0xFFu) - 126)) : kSplitSA;
    const float sa_scale = __builtin_ldexpf(1.0f, sa), descale = __builtin_ldexpf(1.0f, -(sw + sa));
    float amx = 0.0f;
    if (loader) {
        const int lt = tid - 256;
        // per-lane byte offsets (fixed for the launch) against wave-uniform K-block bases: one 32-bit address register
        // per load, no 64-bit address arithmetic per K block.  The offsets are relative to the block's first row of X
        // and of W (64-bit bases), so they stay below 256 K 4 B < 2^29 at the largest accepted K = 512 x 1024.
        // Piece idx -> row idx / A4: 16 (8) consecutive lanes store 2 whole rows, conflict-free (wsp_off)
        const char* const xblk = reinterpret_cast<const char*>(X) + (size_t)m0 * K * 4;
        const char* const xhblk = reinterpret_cast<const char*>(Xhi) + (size_t)m0 * K * 2;
        const char* const xlblk = reinterpret_cast<const char*>(Xlo) + (size_t)m0 * K * 2;
        const char* const hblk = reinterpret_cast<const char*>(Whi) + (size_t)j0 * K * 2;
        const char* const lblk = reinterpret_cast<const char*>(Wlo) + (size_t)j0 * K * 2;
        uint32_t offA[UA], offB[UB], ldsA[UA], ldsB[UB];
#pragma unroll
        for (int u = 0; u < UA; ++u) {
            const int idx = lt + NL * u;
            const int r = idx / A4, c4 = (idx % A4) * (PRE ? 8 : 4);
            const int mr = min(m0 + r, M - 1) - m0;  // row within the block: < BM
            offA[u] = (uint32_t)(((int64_t)mr * K + c4) * (PRE ? 2 : 4));
            ldsA[u] = (uint32_t)wsp_off(r, c4);
        }
#pragma unroll
        for (int u = 0; u < UB; ++u) {
            const int idx = lt + NL * u;
            const int r = idx / B8, c8 = (idx % B8) * 8;
            offB[u] = (uint32_t)(((int64_t)r * K + c8) * 2);
            ldsB[u] = (uint32_t)wsp_off(r, c8);
        }
        f4 ra[FDL][UA], ral[FDL][PRE ? UA : 1], rbh[FDL][UB], rbl[FDL][UB];
        auto fetch = [&](int slot, int kb) {
            const int k0 = min(kb, nk - 1) * GKT;
            const char* const xk = xblk + (size_t)k0 * 4;
            const char* const hk = hblk + (size_t)k0 * 2;
            const char* const lk = lblk + (size_t)k0 * 2;
            if constexpr (PRE) {
#pragma unroll
                for (int u = 0; u < UA; ++u) {
                    ra[slot][u] = *reinterpret_cast<const f4*>(xhblk + (size_t)k0 * 2 + offA[u]);
                    ral[slot][u] = *reinterpret_cast<const f4*>(xlblk + (size_t)k0 * 2 + offA[u]);
                }
            } else {
#pragma unroll
                for (int u = 0; u < UA; ++u) ra[slot][u] = *reinterpret_cast<const f4*>(xk + offA[u]);
            }
#pragma unroll
            for (int u = 0; u < UB; ++u) {
                rbh[slot][u] = *reinterpret_cast<const f4*>(hk + offB[u]);
                rbl[slot][u] = *reinterpret_cast<const f4*>(lk + offB[u]);
            }
        };
        auto stash = [&](int slot, auto lds_slot) {
            _Float16* const base = smb + (size_t)decltype(lds_slot)::value * SLOT;
            if constexpr (PRE) {
#pragma unroll
                for (int u = 0; u < UA; ++u) {
                    *reinterpret_cast<f4*>(base + ldsA[u]) = ra[slot][u];
                    *reinterpret_cast<f4*>(base + PA + ldsA[u]) = ral[slot][u];
                }
            } else
#pragma unroll
            for (int u = 0; u < UA; ++u) {
                hf4 hi, lo;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float x = ra[slot][u][e] * sa_scale;
                    hi[e] = (_Float16)x;
                    lo[e] = (_Float16)(x - (float)hi[e]);
                }
                *reinterpret_cast<hf4*>(base + ldsA[u]) = hi;
                *reinterpret_cast<hf4*>(base + PA + ldsA[u]) = lo;
            }
#pragma unroll
            for (int u = 0; u < UB; ++u) {
                *reinterpret_cast<f4*>(base + 2 * PA + ldsB[u]) = rbh[slot][u];
                *reinterpret_cast<f4*>(base + 2 * PA + PB + ldsB[u]) = rbl[slot][u];
            }
        };
        // block b lives in register slot b % FDL from its fetch to its stash into LDS slot b % NS
        static_for<0, FDL>([&](auto i) { fetch(i.value, i.value); });
        stash(0, std::integral_constant<int, 0>{});
        stash(1, std::integral_constant<int, 1>{});
        fetch(0, FDL);
        fetch(1, FDL + 1);
        lds_barrier();
        // step k: the MFMA waves read slot k % NS; the loaders stash block k + 2 and fetch block k + 2 + FDL
        int kb = 0;
        for (; kb + FDL <= nk; kb += FDL)
            static_for<0, FDL>([&](auto i) {
                constexpr int RS = (i.value + 2) % FDL;
                stash(RS, std::integral_constant<int, (i.value + 2) % NS>{});
                fetch(RS, kb + i.value + 2 + FDL);
                lds_barrier();
            });
        static_for<0, FDL>([&](auto i) {
            if (kb + i.value < nk) {
                constexpr int RS = (i.value + 2) % FDL;
                stash(RS, std::integral_constant<int, (i.value + 2) % NS>{});
                lds_barrier();
            }
        });
    } else {
        __builtin_amdgcn_s_setprio(1);
        const int h = lane >> 5, col = lane & 31;
        const int wm = wave & 1, wn = wave >> 1;
        f16v acc[TM][TN];
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int b = 0; b < TN; ++b)
                acc[a][b] = f16v{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        // fragment rows wm 32 TM + 32 t + col (A) and wn 64 + 32 t + col (B): every tile base is a multiple of 32, so
        // the swizzle of chunk 2 st + h depends on col only
        const int xr = (col >> 2) & 3;
        const int cq0 = ((0 + h) ^ xr) << 3, cq1 = ((2 + h) ^ xr) << 3;
        const int ar = (wm * 32 * TM + col) * 32, br = (wn * 32 * TN + col) * 32;
        struct Frags {
            hf8 ah[TM], al[TM], bh[TN], bl[TN];
        };
        auto read = [&](int slot, int st, Frags& f) {
            const _Float16* const cb = smb + (size_t)slot * SLOT + (st ? cq1 : cq0);
#pragma unroll
            for (int t = 0; t < TM; ++t) {
                f.ah[t] = *reinterpret_cast<const hf8*>(cb + ar + t * 32 * 32);
                f.al[t] = *reinterpret_cast<const hf8*>(cb + PA + ar + t * 32 * 32);
            }
#pragma unroll
            for (int t = 0; t < TN; ++t) {
                f.bh[t] = *reinterpret_cast<const hf8*>(cb + 2 * PA + br + t * 32 * 32);
                f.bl[t] = *reinterpret_cast<const hf8*>(cb + 2 * PA + PB + br + t * 32 * 32);
            }
        };
        Frags f[2];
        lds_barrier();
        read(0, 0, f[0]);
        // slot (kb + 1) % NS was complete at the barrier that ended step kb - 1, so its first k-step's fragments are
        // read during step kb's MFMAs (the loaders write slot (kb + 2) % NS meanwhile)
        auto step = [&](auto slot_c) {
            constexpr int SL = decltype(slot_c)::value;  // kb % NS
#pragma unroll
            for (int st = 0; st < GKT / 16; ++st) {
                if (st + 1 < GKT / 16)
                    read(SL, st + 1, f[(st + 1) & 1]);
                else
                    read((SL + 1) % NS, 0, f[(st + 1) & 1]);
                const Frags& c = f[st & 1];
#pragma unroll
                for (int a = 0; a < TM; ++a)
#pragma unroll
                    for (int b = 0; b < TN; ++b) {
                        acc[a][b] = mfma16(c.ah[a], c.bh[b], acc[a][b]);
                        acc[a][b] = mfma16(c.ah[a], c.bl[b], acc[a][b]);
                        acc[a][b] = mfma16(c.al[a], c.bh[b], acc[a][b]);
                    }
            }
            lds_barrier();
        };
        int kb = 0;
        for (; kb + NS <= nk; kb += NS) static_for<0, NS>([&](auto i) { step(i); });
        static_for<0, NS>([&](auto i) {
            if (kb + i.value < nk) step(i);
        });
        __builtin_amdgcn_s_setprio(0);
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int b = 0; b < TN; ++b) {
                const int j = j0 + wn * 32 * TN + 32 * b + col;
                const float bj = bias[j];
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = m0 + wm * 32 * TM + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * h;
                    if (m < M) {
                        float v = fmaf(acc[a][b][r], descale, bj);
                        if (act) v = gelu(v);
                        out[(int64_t)m * Nout + j] = v;
                        amx = fmaxf(amx, fabsf(v));
                    }
                }
            }
    }
    if (amax_out != nullptr) publish_amax(amax_out, amx);
}
#define FC_WSP(BMV) fc_split_wsp_kernel<NPD_FC_FDL, false, BMV>
#define FC_WSP_PRE fc_split_wsp_kernel<NPD_FC_FDL, true, 128>

// X (n floats, n % 4 == 0) -> fp16 planes hi = fp16(x 2^SA), lo = fp16(x 2^SA - hi), SA from the producer's max |x| as
// in every split consumer (split_sa): the operands fc_split_wsp_kernel<.., true> copies instead of splitting
__global__ __launch_bounds__(256) void split_planes_kernel(const float* __restrict__ X, int64_t n4,
                                                           const uint32_t* __restrict__ amax_in,
                                                           uint16_t* __restrict__ hi, uint16_t* __restrict__ lo) {
    const float sc = __builtin_ldexpf(1.0f, split_sa(amax_in));
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        const f4 v = __builtin_nontemporal_load(reinterpret_cast<const f4*>(X) + i);
        hf4 h, l;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float x = v[e] * sc;
            h[e] = (_Float16)x;
            l[e] = (_Float16)(x - (float)h[e]);
        }
        reinterpret_cast<hf4*>(hi)[i] = h;
        reinterpret_cast<hf4*>(lo)[i] = l;
    }
}

// ------------------------------------------------------------------------------ LayerNorm + sign
__global__ __launch_bounds__(256) void layernorm_sign_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                             const float* __restrict__ be, float* __restrict__ logits,
                                                             float* __restrict__ dec, int M, int N) {
    const int lane = threadIdx.x & 63;
    const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (m >= M) return;
    const float* r = x + m * N;
    float s = 0.0f;
    for (int i = lane; i < N; i += 64) s += r[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    const float mean = s / (float)N;
    float v = 0.0f;
    for (int i = lane; i < N; i += 64) {
        const float d = r[i] - mean;
        v += d * d;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const float rstd = 1.0f / sqrtf(v / (float)N + 1e-6f);
    for (int i = lane; i < N; i += 64) {
        const float y = (r[i] - mean) * rstd * g[i] + be[i];
        if (logits) logits[m * N + i] = y;
        if (dec) dec[m * N + i] = y > 0.0f ? 1.0f : (y < 0.0f ? -1.0f : 0.0f);
    }
}

}  // namespace conv
}  // namespace npd

using namespace npd;
using namespace npd::conv;

struct npd_conv {
    int N, E, precision, device;
    LayerDesc layers[kLayers];
    float* img;         // device: permuted conv weights + biases + FC weights/biases + LN params
    int64_t off_fc[3][2];  // (weight, bias) offsets of the three Linear layers
    int64_t off_ln[2];
    int64_t off_fc16[3][2];  // precision 3: (hi, lo) fp16 weight planes of the Linear layers (offsets in floats)
    int fc_sw[3];
};

static void conv_spec(int E, int idx, int& cin, int& cout, int& dil, int& res) {
    const int H = E / 2;
    // (cin, cout, dilation, residual-after) for layers1.0, layers1.2, layers2.0, ..., layers5.2
    static const int dils[kLayers] = {1, 2, 4, 1, 2, 4, 1, 2, 4, 1};
    dil = dils[idx];
    cin = idx == 0 ? 1 : (idx == 9 ? E : H);
    cout = idx >= 8 ? E : H;
    res = (idx == 3 || idx == 5 || idx == 7) ? 1 : 0;
}

extern "C" int npd_conv_create(int N, int embed, const float* weights, int64_t n_weights, int precision,
                               npd_conv** out) {
    NPD_ARG(out != nullptr, "npd_conv_create: out is NULL");
    *out = nullptr;
    NPD_ARG(weights != nullptr, "npd_conv_create: weights is NULL");
    NPD_ARG(N >= 64 && N <= 1024 && N % 64 == 0, "npd_conv_create: N must be a multiple of 64 in [64, 1024]");
    NPD_ARG(embed >= 16 && embed <= 512 && embed % 16 == 0, "npd_conv_create: embed must be a multiple of 16 in [16, 512]");
    NPD_ARG(precision == 0 || precision == 3, "npd_conv_create: precision must be 0 (fp32) or 3 (fp16x3 conv layers)");
    const int E = embed;
    // host weights in state_dict order: (w, b) per conv layer, then 3 x (w, b) Linear, then LN (g, b)
    int64_t expect = 0;
    for (int i = 0; i < kLayers; ++i) {
        int ci, co, d, r;
        conv_spec(E, i, ci, co, d, r);
        expect += (int64_t)co * ci * 7 + co;
    }
    expect += (int64_t)4 * N * E * N + 4 * N + (int64_t)N * 4 * N + N + (int64_t)N * N + N + 2 * N;
    NPD_ARG(n_weights == expect, "npd_conv_create: weight count does not match (N, embed)");
    npd_conv* c = new (std::nothrow) npd_conv;
    if (!c) return fail(NPD_ENOMEM, "npd_conv_create: out of memory");
    memset(c, 0, sizeof(*c));
    c->N = N;
    c->E = E;
    c->precision = precision;
    std::vector<float> img;
    const float* p = weights;
    for (int i = 0; i < kLayers; ++i) {
        int ci, co, d, r;
        conv_spec(E, i, ci, co, d, r);
        LayerDesc& L = c->layers[i];
        L.cin = ci; L.cout = co; L.dil = d; L.res = r;
        L.soff16 = -1;
        L.ksteps = (7 * ci + 1) / 2;
        // pad channel tiles to 64 so every (64-channel) block has two 32-row MFMA tiles
        const int co_pad = ((co + 63) / 64) * 64;
        while (img.size() % 4) img.push_back(0.0f);
        L.woff = (int64_t)img.size();
        const float* w = p;  // (co, ci, 7)
        if (ci == 1) {
            // [t32][lane][4]: k-step s of lane half hh is tap 2s + hh (tap 7 = 0)
            img.resize(img.size() + (size_t)(co_pad / 32) * 64 * 4, 0.0f);
            for (int t32 = 0; t32 < co_pad / 32; ++t32)
                for (int l = 0; l < 64; ++l)
                    for (int s2 = 0; s2 < 4; ++s2) {
                        const int row = 32 * t32 + (l & 31), t = 2 * s2 + (l >> 5);
                        img[L.woff + ((int64_t)t32 * 64 + l) * 4 + s2] = (row < co && t < 7) ? w[(int64_t)row * 7 + t] : 0.0f;
                    }
        } else {
            // [t32][tap][group][lane][4]: k-step 4g+e of tap t pairs channel 4g+e (half 0) with cin/2 + 4g+e
            const int ng = ci / 8;
            img.resize(img.size() + (size_t)(co_pad / 32) * 7 * ng * 64 * 4, 0.0f);
            for (int t32 = 0; t32 < co_pad / 32; ++t32)
                for (int t = 0; t < 7; ++t)
                    for (int g = 0; g < ng; ++g)
                        for (int l = 0; l < 64; ++l)
                            for (int e = 0; e < 4; ++e) {
                                const int row = 32 * t32 + (l & 31);
                                const int cc = (l >> 5) * (ci / 2) + 4 * g + e;
                                img[L.woff + ((((int64_t)t32 * 7 + t) * ng + g) * 64 + l) * 4 + e] =
                                    row < co ? w[((int64_t)row * ci + cc) * 7 + t] : 0.0f;
                            }
        }
        if (precision == 3 && ci > 1) {
            // fp16x3 A fragments [t32][tap][s][part hi/lo][lane][8 x fp16]: lane (r, hh), element j = W[row][16s + 8hh + j][t]
            // x 2^SW, split hi = fp16(v), lo = fp16(v - hi)
            float m = 0.0f;
            for (int64_t i = 0; i < (int64_t)co * ci * 7; ++i) m = fmaxf(m, fabsf(w[i]));
            const int sw = m > 0.0f ? 12 - (int)floorf(log2f(m)) : 0;
            const float sc = ldexpf(1.0f, sw);
            L.sw = sw;
            const int ng = (ci + 15) / 16;
            while (img.size() % 4) img.push_back(0.0f);
            L.soff = (int64_t)img.size();
            const size_t n16 = (size_t)(co_pad / 32) * 7 * ng * 2 * 64 * 8;
            img.resize(img.size() + n16 / 2, 0.0f);
            uint16_t* u16 = reinterpret_cast<uint16_t*>(img.data() + L.soff);
            for (int t32 = 0; t32 < co_pad / 32; ++t32)
                for (int t = 0; t < 7; ++t)
                    for (int g = 0; g < ng; ++g)
                        for (int l = 0; l < 64; ++l)
                            for (int j = 0; j < 8; ++j) {
                                const int row = 32 * t32 + (l & 31), cc = 16 * g + 8 * (l >> 5) + j;
                                const float v = (row < co && cc < ci) ? w[((int64_t)row * ci + cc) * 7 + t] * sc : 0.0f;
                                const _Float16 hi = (_Float16)v;
                                const _Float16 lo = (_Float16)(v - (float)hi);
                                const size_t e = ((((size_t)(t32 * 7 + t) * ng + g) * 2) * 64 + l) * 8 + j;
                                memcpy(&u16[e], &hi, 2);
                                memcpy(&u16[e + 64 * 8], &lo, 2);
                            }
            L.soff16 = -1;
            if (ci == 32 || ci == 64 || (ci == 128 && NPD_WS16_128)) {
                // conv_ws16_kernel A fragments [t16][tap][kb][part hi/lo][lane][8 x fp16]: 16x16x32 map, lane l = 16 g + r,
                // element j = W[row 16 t16 + r][32 kb + 8 g + j][t] x 2^SW
                const int kbn = ci / 32;
                while (img.size() % 4) img.push_back(0.0f);
                L.soff16 = (int64_t)img.size();
                const size_t m16 = (size_t)(co_pad / 16) * 7 * kbn * 2 * 64 * 8;
                img.resize(img.size() + m16 / 2, 0.0f);
                uint16_t* v16 = reinterpret_cast<uint16_t*>(img.data() + L.soff16);
                for (int t16 = 0; t16 < co_pad / 16; ++t16)
                    for (int t = 0; t < 7; ++t)
                        for (int kb = 0; kb < kbn; ++kb)
                            for (int l = 0; l < 64; ++l)
                                for (int j = 0; j < 8; ++j) {
                                    const int row = 16 * t16 + (l & 15), cc = 32 * kb + 8 * (l >> 4) + j;
                                    const float v = row < co ? w[((int64_t)row * ci + cc) * 7 + t] * sc : 0.0f;
                                    const _Float16 hi = (_Float16)v;
                                    const _Float16 lo = (_Float16)(v - (float)hi);
                                    const size_t e = ((((size_t)(t16 * 7 + t) * kbn + kb) * 2) * 64 + l) * 8 + j;
                                    memcpy(&v16[e], &hi, 2);
                                    memcpy(&v16[e + 64 * 8], &lo, 2);
                                }
            }
        }
        p += (int64_t)co * ci * 7;
        L.boff = (int64_t)img.size();
        img.insert(img.end(), p, p + co);
        img.resize(L.boff + co_pad, 0.0f);
        while (img.size() % 4) img.push_back(0.0f);
        p += co;
    }
    const int64_t fcin[3] = {(int64_t)E * N, 4 * N, N}, fcout[3] = {4 * N, N, N};
    for (int f = 0; f < 3; ++f) {
        while (img.size() % 4) img.push_back(0.0f);  // 16-B alignment for f4 loads
        c->off_fc[f][0] = (int64_t)img.size();
        if (f == 0) {
            // the activations are (B, N, E): flatten index l*E + c instead of torch's c*N + l
            const size_t base = img.size();
            img.resize(base + (size_t)fcin[0] * fcout[0]);
            for (int64_t j = 0; j < fcout[0]; ++j)
                for (int cc = 0; cc < E; ++cc)
                    for (int l = 0; l < N; ++l) img[base + j * fcin[0] + (int64_t)l * E + cc] = p[j * fcin[0] + (int64_t)cc * N + l];
        } else {
            img.insert(img.end(), p, p + fcin[f] * fcout[f]);
        }
        if (precision == 3) {
            // hi / lo fp16 planes of the (permuted) weights x 2^SW, max |w| 2^SW in [2^12, 2^13)
            const int64_t nwf = fcin[f] * fcout[f];
            const int64_t wsrc = c->off_fc[f][0];
            float m = 0.0f;
            for (int64_t i = 0; i < nwf; ++i) m = fmaxf(m, fabsf(img[wsrc + i]));
            const int sw = m > 0.0f ? 12 - (int)floorf(log2f(m)) : 0;
            const float sc = ldexpf(1.0f, sw);
            c->fc_sw[f] = sw;
            while (img.size() % 4) img.push_back(0.0f);
            c->off_fc16[f][0] = (int64_t)img.size();
            c->off_fc16[f][1] = c->off_fc16[f][0] + (nwf + 7) / 8 * 4;  // 16-B aligned lo plane
            img.resize(c->off_fc16[f][1] + (nwf + 7) / 8 * 4, 0.0f);
            uint16_t* hp = reinterpret_cast<uint16_t*>(img.data() + c->off_fc16[f][0]);
            uint16_t* lp = reinterpret_cast<uint16_t*>(img.data() + c->off_fc16[f][1]);
            for (int64_t i = 0; i < nwf; ++i) {
                const float v = img[wsrc + i] * sc;
                const _Float16 hi = (_Float16)v;
                const _Float16 lo = (_Float16)(v - (float)hi);
                memcpy(hp + i, &hi, 2);
                memcpy(lp + i, &lo, 2);
            }
        }
        p += fcin[f] * fcout[f];
        c->off_fc[f][1] = (int64_t)img.size();
        img.insert(img.end(), p, p + fcout[f]);
        p += fcout[f];
    }
    c->off_ln[0] = (int64_t)img.size();
    img.insert(img.end(), p, p + N);
    p += N;
    c->off_ln[1] = (int64_t)img.size();
    img.insert(img.end(), p, p + N);
    hipError_t e = hipGetDevice(&c->device);
    if (e == hipSuccess) e = hipMalloc(&c->img, img.size() * 4);
    if (e == hipSuccess) e = hipMemcpy(c->img, img.data(), img.size() * 4, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        if (c->img) (void)hipFree(c->img);
        delete c;
        return hip_fail(e, "npd_conv_create");
    }
    *out = c;
    return NPD_OK;
}

extern "C" int npd_conv_destroy(npd_conv* c) {
    if (!c) return NPD_OK;
    if (c->img) (void)hipFree(c->img);
    delete c;
    return NPD_OK;
}

// codewords per pass: kChunk, halved (to >= 512) while the three (chunk, E, N) fp32 activation buffers would pass
// 4 GiB -- configs[4] (E N = 32768) keeps 8192 (3.2 GB); the widest accepted net (E 512, N 1024) runs 512
static int64_t chunk_of(const npd_conv* c, int64_t B) {
    int64_t ch = kChunk;
    while (ch > 512 && 3 * ch * (int64_t)c->E * c->N * 4 > ((int64_t)4 << 30)) ch >>= 1;
    return B < ch ? B : ch;
}
// A/B switch NPD_FC0_PRESPLIT=0/1 (default 0): FC0 on pre-split X planes (split_planes_kernel + fc_split_wsp_kernel<..,
// true>).  Round 6 (profiles/round6/fc0_presplit_ab.txt): with copy-only loaders FC0 takes 935-938 us
// per 4096 codewords against 1,061 us splitting in its loaders (-12 %), but the separate split pass costs 197 us, so the
// default keeps the in-loader split; a split fused into the producing conv layer's epilogue would bound the gain at
// those 12 % of FC0 (~3 % of the forward) -- the FC0 GEMM is not bound by its loaders' split work
static bool fc0_presplit() {
    const char* e = getenv("NPD_FC0_PRESPLIT");
    return e != nullptr && atoi(e) != 0;
}
// A/B switch NPD_FC_BM = 128 / 256 (default 0: automatic): FC block-tile rows, see fc_split_wsp_kernel
static int fc_bm_env() {
    const char* e = getenv("NPD_FC_BM");
    const int v = e == nullptr ? 0 : atoi(e);
    return v == 128 || v == 256 ? v : 0;  // anything else: automatic (the grid is sized for the tile actually launched)
}// max |activation| records of one chunk (fp16x3; kAmaxWords words each): conv layer i's output at record i, FC f's at
// record kLayers + f
constexpr int kAmaxSlots = kLayers + 3;

// input4 (models.py:750, returned by convNet.forward): the (nb, N, C) activation after layers3 (+ residual) as
// the reference's channels-first (nb, C, N).  A 64 x 64 (position x channel) tile per workgroup through LDS,
// so both the reads (channels contiguous) and the writes (positions contiguous) are coalesced.
__global__ __launch_bounds__(256) void act_to_channels_first_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                                    int N, int C) {
    __shared__ float t[64][65];
    const int64_t b = blockIdx.z;
    const int l0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
    const float* src = in + b * (int64_t)N * C;
    float* dst = out + b * (int64_t)N * C;
    for (int e = threadIdx.x; e < 64 * 64; e += 256) {
        const int l = e >> 6, cc = e & 63;
        if (l0 + l < N && c0 + cc < C) t[l][cc] = src[(int64_t)(l0 + l) * C + c0 + cc];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < 64 * 64; e += 256) {
        const int cc = e >> 6, l = e & 63;
        if (l0 + l < N && c0 + cc < C) dst[(int64_t)(c0 + cc) * N + l0 + l] = t[l][cc];
    }
}

extern "C" int64_t npd_conv_workspace_bytes(const npd_conv* c, int64_t B) {
    if (!c || B <= 0) return 0;
    const int64_t Bc = chunk_of(c, B);
    // three activation buffers of (Bc, E, N) + FC1/FC2/FC3 outputs + the activation-range words (kAmaxSlots)
    return (3 * Bc * (int64_t)c->E * c->N + Bc * 4 * (int64_t)c->N + 2 * Bc * (int64_t)c->N) * 4 + 256 + (int64_t)kAmaxSlots * kAmaxWords * 4;
}

extern "C" int npd_conv_forward_ex(const npd_conv* c, const float* y, float* logits, float* decoded, float* input4,
                                   void* workspace, int64_t B, void* stream);

extern "C" int npd_conv_forward(const npd_conv* c, const float* y, float* logits, float* decoded, void* workspace,
                                int64_t B, void* stream) {
    return npd_conv_forward_ex(c, y, logits, decoded, nullptr, workspace, B, stream);
}

extern "C" int npd_conv_forward_ex(const npd_conv* c, const float* y, float* logits, float* decoded, float* input4,
                                   void* workspace, int64_t B, void* stream) {
    NPD_ARG(c != nullptr, "npd_conv_forward: conv is NULL");
    NPD_ARG(B >= 0, "npd_conv_forward: B < 0");
    if (B == 0) return NPD_OK;
    NPD_ARG(y != nullptr && workspace != nullptr, "npd_conv_forward: null pointer");
    NPD_ARG(logits != nullptr || decoded != nullptr, "npd_conv_forward: nothing to write");
    hipStream_t s = (hipStream_t)stream;
    const int N = c->N, E = c->E;
    const int64_t Bc = chunk_of(c, B);
    float* ws = reinterpret_cast<float*>(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
    float* A0 = ws;
    float* A1 = A0 + Bc * (int64_t)E * N;
    float* A2 = A1 + Bc * (int64_t)E * N;
    float* H1 = A2 + Bc * (int64_t)E * N;
    float* H2 = H1 + Bc * 4 * (int64_t)N;
    float* H3 = H2 + Bc * (int64_t)N;
    uint32_t* amax = reinterpret_cast<uint32_t*>(H3 + Bc * (int64_t)N);
    const bool split = c->precision == 3;
    static bool attr = false;
    if (!attr) {
        NPD_HIP(hipFuncSetAttribute((const void*)conv_layer_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    163840));
        NPD_HIP(hipFuncSetAttribute((const void*)conv_layer_split_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    163840));
        NPD_HIP(hipFuncSetAttribute((const void*)conv_layer_split_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    163840));
        NPD_HIP(hipFuncSetAttribute((const void*)FC_WSP(128), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)fc_wsp_lds(128)));
        NPD_HIP(hipFuncSetAttribute((const void*)FC_WSP(256), hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)fc_wsp_lds(256)));
        NPD_HIP(hipFuncSetAttribute((const void*)FC_WSP_PRE, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)fc_wsp_lds(128)));
        const void* ws[8] = {(const void*)conv_split_ws_kernel<1, 1, 1, 4>, (const void*)conv_split_ws_kernel<1, 2, 1, 4>,
                             (const void*)conv_split_ws_kernel<2, 1, 1, 4>, (const void*)conv_split_ws_kernel<2, 2, 1, 4>,
                             (const void*)conv_split_ws_kernel<3, 1, 1, 4>, (const void*)conv_split_ws_kernel<3, 2, 1, 4>,
                             (const void*)conv_split_ws_kernel<4, 1, 2, 4>, (const void*)conv_split_ws_kernel<8, 1, 4, 8>};
        for (const void* k : ws) NPD_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
        const void* w16[5] = {(const void*)conv_ws16_kernel<1, 1, NPD_WS16_NW, 1>,
                              (const void*)conv_ws16_kernel<1, 2, NPD_WS16_NW, 1>,
                              (const void*)conv_ws16_kernel<2, 1, NPD_WS16_NW, 1>,
                              (const void*)conv_ws16_kernel<2, 2, NPD_WS16_NW, 1>, (const void*)conv_ws16_kernel<4, 1, 8, 2>};
        for (const void* k : w16) NPD_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
        attr = true;
    }
    for (int64_t b0 = 0; b0 < B; b0 += Bc) {
        const int64_t nb = (B - b0) < Bc ? (B - b0) : Bc;
        if (split) NPD_HIP(hipMemsetAsync(amax, 0, (size_t)kAmaxSlots * kAmaxWords * 4, s));
        // layer inputs/outputs: x (N floats per cw) -> A0 -> A1 -> ... ; block inputs kept for the residual
        const float* src = y + b0 * N;
        // buffers: cur input, output, residual source
        float* bufs[3] = {A0, A1, A2};
        int in_idx = -1;   // -1: y
        int res_idx = -1;  // buffer holding the current block input
        int out_idx = 0;
        for (int i = 0; i < kLayers; ++i) {
            const LayerDesc& L = c->layers[i];
            const float* in = in_idx < 0 ? src : bufs[in_idx];
            // choose an output buffer that is neither the input nor the pending residual
            out_idx = 0;
            while (out_idx == in_idx || out_idx == res_idx) ++out_idx;
            float* o = bufs[out_idx];
            const float* rsrc = L.res ? bufs[res_idx] : nullptr;
            const int halo = 3 * L.dil;
            const size_t lds = (size_t)(L.cin == 1 ? 4 : L.cin + 4) * (64 + 2 * halo) * 4;
            dim3 grid(N / 64, (L.cout + 63) / 64, (unsigned)nb);
            uint32_t* const am_out = split ? amax + i * kAmaxWords : nullptr;
            const uint32_t* const am_in = i > 0 ? amax + (i - 1) * kAmaxWords : nullptr;
            if (L.cin == 1)
                hipLaunchKernelGGL(conv_layer_kernel<true>, grid, dim3(256), lds, s, in, o, rsrc, c->img + L.woff,
                                   c->img + L.boff, L.cin, L.cout, N, L.dil, L.res, am_out);
            else if (split && L.dil <= 4 && L.soff16 >= 0) {
                // cin 32 / 64: 16x16x32 weight-stationary kernel, no channel parts; one 8-wave block per CU, a multiple of
                // the 64-channel slice count; 128-position items where N allows.  cin 128: two channel parts of 64,
                // 64-position items
                const int kbn = L.cin / 32;
                const int kp = kbn == 4 ? 2 : 1;
                const int nw = kp == 2 ? 8 : NPD_WS16_NW;
                const int Q = kp == 1 && N % 128 == 0 && NPD_WS16_Q2 ? 2 : 1;
                const int nslices = (L.cout + 63) / 64;
                const int64_t items = nb * (N / (64 * Q)) * nslices;
                int64_t nblk = (int64_t)device_cu_count() * (8 / nw);
                nblk -= nblk % nslices;
                if (nblk > items) nblk = items;
                if (nblk < nslices) nblk = nslices;
                const size_t ls = ws16_lds_bytes(kbn, Q, L.dil, kp);
                const f4* wi = reinterpret_cast<const f4*>(c->img + L.soff16);
#define NPD_WS16(KBV, QV, NWV, KPV)                                                                                \
    hipLaunchKernelGGL((conv_ws16_kernel<KBV, QV, NWV, KPV>), dim3((unsigned)nblk), dim3(64 * NWV), ls, s, in, o,    \
                       rsrc, wi, c->img + L.boff, L.cout, N, L.dil, L.res, L.sw, am_in, am_out, nb, nslices)
                if (kbn == 4) NPD_WS16(4, 1, 8, 2);
                else if (kbn == 2) { if (Q == 2) NPD_WS16(2, 2, NPD_WS16_NW, 1); else NPD_WS16(2, 1, NPD_WS16_NW, 1); }
                else { if (Q == 2) NPD_WS16(1, 2, NPD_WS16_NW, 1); else NPD_WS16(1, 1, NPD_WS16_NW, 1); }
#undef NPD_WS16
            } else if (split && L.dil <= 4 && (L.cin <= 64 || L.cin == 128)) {
                // weight-stationary persistent blocks: one per CU, a multiple of the 64-channel slice count.
                // cin <= 48: 4 waves (KS 1); 64: 4 waves, 2 channel parts, two blocks per CU; 128: 8 waves, 4 channel
                // parts, 64-position items (the 128-position slab would not fit).  Other widths (e.g. 80, 96: a 2-part
                // split of 96 channels spills) run the slab kernel below.
                const int ng = (L.cin + 15) / 16;
                const int ks = ng <= 3 ? 1 : (ng == 8 ? 4 : 2);  // ng in {1, 2, 3, 4, 8}
                const int nw = ng == 8 ? 8 : 4;
                const int Q = (ng <= 3 && N % 128 == 0) ? 2 : 1;
                const int nslices = (L.cout + 63) / 64;
                const int64_t items = nb * (N / (64 * Q)) * nslices;
                // cin 64: two independent 4-wave blocks per CU (67 KB of LDS each), so one block's barrier and
                // latency waits are filled by the other's work; the others one 8- or 4-wave block per CU
                int64_t nblk = (int64_t)device_cu_count() * (ng == 4 ? 2 : 1);
                nblk -= nblk % nslices;
                if (nblk > items) nblk = items;
                if (nblk < nslices) nblk = nslices;
                const size_t ls = ws_lds_bytes(ng, Q, ks, nw, L.dil);
                const f4* wi = reinterpret_cast<const f4*>(c->img + L.soff);
#define NPD_WS(NGV, QV, KSV, NWV)                                                                                   \
    hipLaunchKernelGGL((conv_split_ws_kernel<NGV, QV, KSV, NWV>), dim3((unsigned)nblk), dim3(64 * NWV), ls, s, in, o, \
                       rsrc, wi, c->img + L.boff, L.cin, L.cout, N, L.dil, L.res, L.sw, am_in, am_out, nb, nslices)
                if (ng == 8) NPD_WS(8, 1, 4, 8);
                else if (ng == 4) NPD_WS(4, 1, 2, 4);
                else if (ng == 1) { if (Q == 2) NPD_WS(1, 2, 1, 4); else NPD_WS(1, 1, 1, 4); }
                else if (ng == 2) { if (Q == 2) NPD_WS(2, 2, 1, 4); else NPD_WS(2, 1, 1, 4); }
                else { if (Q == 2) NPD_WS(3, 2, 1, 4); else NPD_WS(3, 1, 1, 4); }
#undef NPD_WS
            } else if (split) {
                // positions per block 64 P: P = 2 where 128 <= N and the two fp16 slab planes fit, else 1.  (P = 4 reuses
                // each weight fragment over 4 position tiles but its 80 KB slab leaves one block per CU, no overlap of
                // one block's staging with another's MFMAs: configs[4] forward 11.6-12.1 ms at P = 4, 10.3-10.6 at
                // P = 2, 10.6-10.7 at P = 1 per 8192 codewords, profiles/round4/conv_p_ab.txt)
                const int cs = ((L.cin + 15) & ~15) + 8;
                int P = 2;
                while (P > 1 && (64 * P > N || (size_t)2 * (64 * P + 2 * halo) * cs * 2 > 160 * 1024)) P >>= 1;
                const size_t ls = (size_t)2 * (64 * P + 2 * halo) * cs * 2;
                dim3 gs((N + 64 * P - 1) / (64 * P), (L.cout + 63) / 64, (unsigned)nb);
                const f4* wi = reinterpret_cast<const f4*>(c->img + L.soff);
                if (P == 2)
                    hipLaunchKernelGGL(conv_layer_split_kernel<2>, gs, dim3(256), ls, s, in, o, rsrc, wi, c->img + L.boff,
                                       L.cin, L.cout, N, L.dil, L.res, L.sw, am_in, am_out);
                else
                    hipLaunchKernelGGL(conv_layer_split_kernel<1>, gs, dim3(256), ls, s, in, o, rsrc, wi, c->img + L.boff,
                                       L.cin, L.cout, N, L.dil, L.res, L.sw, am_in, am_out);
            } else
                hipLaunchKernelGGL(conv_layer_kernel<false>, grid, dim3(256), lds, s, in, o, rsrc, c->img + L.woff,
                                   c->img + L.boff, L.cin, L.cout, N, L.dil, L.res, nullptr);
            int rc = launch_check("conv_layer_kernel launch");
            if (rc) return rc;
            // block structure (models.py:742-766): the output of layers1 (i == 1) and of each residual
            // block (i == 3, 5, 7) is the next block's input and residual
            if (i == 1 || i == 3 || i == 5 || i == 7) res_idx = out_idx;
            in_idx = out_idx;
            if (i == 5 && input4) {  // input4 = layers3(input3) + residual3 (models.py:750)
                dim3 gt((N + 63) / 64, (L.cout + 63) / 64, (unsigned)nb);
                hipLaunchKernelGGL(act_to_channels_first_kernel, gt, dim3(256), 0, s, o, input4 + b0 * (int64_t)L.cout * N,
                                   N, L.cout);
                rc = launch_check("input4 transpose launch");
                if (rc) return rc;
            }
        }
        const float* flat = bufs[in_idx];  // (nb, N*E): l*E + c (FC0's weights are permuted to match)
        int free_idx = 0;                   // an activation buffer no longer read: room for FC0's split planes
        while (free_idx == in_idx) ++free_idx;
        const int64_t K1 = (int64_t)E * N;
        dim3 g1(4 * N / 64, (unsigned)((nb + 63) / 64));
        dim3 g2(N / 64, (unsigned)((nb + 63) / 64));
        const float* fin[3] = {flat, H1, H2};
        float* fout[3] = {H1, H2, H3};
        const int fk[3] = {(int)K1, 4 * N, N}, fo[3] = {4 * N, N, N}, fa[3] = {1, 1, 0};
        for (int f = 0; f < 3; ++f) {
            if (c->precision == 3) {
                const uint16_t* wh = reinterpret_cast<const uint16_t*>(c->img + c->off_fc16[f][0]);
                const uint16_t* wl = reinterpret_cast<const uint16_t*>(c->img + c->off_fc16[f][1]);
                const uint32_t* am_in = amax + (f == 0 ? kLayers - 1 : kLayers + f - 1) * kAmaxWords;
                uint32_t* am_out = f < 2 ? amax + (kLayers + f) * kAmaxWords : nullptr;  // FC2 feeds the fp32 LayerNorm
                if (fo[f] % FB == 0 && f == 0 && fc0_presplit()) {
                    // FC0's X split once into fp16 planes in a free activation buffer (layer 9's input: 4 B per
                    // element, as X), then copied by the GEMM's loaders
                    uint16_t* xh = reinterpret_cast<uint16_t*>(bufs[free_idx]);
                    uint16_t* xl = xh + nb * K1;
                    const int64_t n4 = nb * K1 / 4;
                    const int gs = (int)std::min<int64_t>((n4 + 255) / 256, (int64_t)device_cu_count() * 8);
                    hipLaunchKernelGGL(split_planes_kernel, dim3(gs), dim3(256), 0, s, flat, n4, am_in, xh, xl);
                    dim3 gb((unsigned)((fo[f] / FB) * ((nb + FB - 1) / FB)));
                    hipLaunchKernelGGL(FC_WSP_PRE, gb, dim3(512), fc_wsp_lds(128), s, fin[f], xh, xl, wh, wl,
                                       c->img + c->off_fc[f][1], fout[f], (int)nb, fk[f], fo[f], fa[f], c->fc_sw[f],
                                       am_in, am_out);
                } else if (fo[f] % FB == 0) {
                    // 256-row tiles where they alone give every CU a tile (FC0 of an 8192-codeword chunk at N >= 256),
                    // else 128 x 128
                    const int64_t t256 = (fo[f] / FB) * ((nb + 255) / 256);
                    const int bm_env = fc_bm_env();
                    const int bm = bm_env ? bm_env : (t256 >= device_cu_count() ? 256 : 128);
                    dim3 gb((unsigned)((fo[f] / FB) * ((nb + bm - 1) / bm)));
                    auto kern = bm == 256 ? FC_WSP(256) : FC_WSP(128);
                    hipLaunchKernelGGL(kern, gb, dim3(512), fc_wsp_lds(bm), s, fin[f], nullptr, nullptr, wh, wl,
                                       c->img + c->off_fc[f][1], fout[f], (int)nb, fk[f], fo[f], fa[f], c->fc_sw[f],
                                       am_in, am_out);
                } else {
                    hipLaunchKernelGGL(fc_split_kernel, f == 0 ? g1 : g2, dim3(256), 0, s, fin[f], wh, wl,
                                       c->img + c->off_fc[f][1], fout[f], (int)nb, fk[f], fo[f], fa[f], c->fc_sw[f],
                                       am_in, am_out);
                }
            } else {
                hipLaunchKernelGGL(fc_kernel, f == 0 ? g1 : g2, dim3(256), 0, s, fin[f], c->img + c->off_fc[f][0],
                                   c->img + c->off_fc[f][1], fout[f], (int)nb, fk[f], fo[f], fa[f]);
            }
        }
        int rc = launch_check("fc launch");
        if (rc) return rc;
        hipLaunchKernelGGL(layernorm_sign_kernel, dim3((unsigned)((nb + 3) / 4)), dim3(256), 0, s, H3,
                           c->img + c->off_ln[0], c->img + c->off_ln[1], logits ? logits + b0 * N : nullptr,
                           decoded ? decoded + b0 * N : nullptr, (int)nb, N);
        rc = launch_check("fc/layernorm launch");
        if (rc) return rc;
    }
    return NPD_OK;
}
