// npd_gru.hip -- CRISP GRU autoregressive decoder (RNN_decoder.decode, y_input, test branch).
//
// Reference: rnn_all.py:294-398 (RNN_Model: nn.GRU(N+2, F, layers) + Linear(F, 1)), rnn_all.py:532-547
// (per-bit loop: x_i = [y, onehot(prev)], one GRU step, d_i = sign(out) on information positions),
// get_onehot rnn_all.py:258-260, PyTorch GRUCell (r, z, n gate order; h' = (h - n) * z + n).
//
// MI355X design: the per-step matvecs of all codewords of a wave form GEMMs
//   gates^T (3F x 32 codewords) = W (3F x F) . h^T (F x 32)
// computed with v_mfma_f32_32x32x2_f32 (exact fp32 FMA chains).  Gate rows are the MFMA rows and
// codewords the columns, so a 32x32 accumulator tile of h' is, register for register, the B operand
// of the next step's MFMAs (no transpose, no LDS round trip for the state); the weight matrices are
// permuted once on the host into the matching A-operand order and live in LDS for the whole launch
// (one 256-thread workgroup per CU, four waves, 32 codewords per wave).  The y part of the input
// projection, W_ih0[:, :N] y, is constant over the N steps and computed once per codeword (P); the
// one-hot / previous-decision column and all biases are folded into one extra MFMA k-step whose B
// operand is [1, x_i].
#include <stdlib.h>
#include <string.h>

#include <new>
#include <type_traits>
#include <vector>

#include "npd_common.hpp"

struct npd_gru {
    int N, F, layers, onehot, precision, device;
    float b_lin;
    float* img;   // LDS image (device)
    float* wy;    // y-projection A operands (device)
    int64_t img_floats;
    int64_t wy_lo;
    float* img16;  // 16-codeword split kernel's image (F = 64, 2 layers, split precisions), or NULL
    float* wy16;
    int64_t wy16_lo;
    int split16;   // its SplitT variant
    int cell;      // 0 GRU, 1 LSTM (fp32)
    int ln;        // use_layernorm head (rnn_all.py:317-320, :387-398): linear weights hold w * gamma, b_lin b + w . beta
    float ln_eps;
    float* hd;     // out_linear_depth > 1 head image (device; head_image below), or NULL
    int hd_depth, hd_tiles;
    float hd_bout;
};

namespace npd {
namespace gru {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

template <int N>
struct IC {
    static constexpr int value = N;
};
// compile-time loop: f(IC<i>{}) for i in [B, E)
template <int B, int E, typename Fn>
__device__ __forceinline__ void static_for(Fn&& f) {
    if constexpr (B < E) {
        f(IC<B>{});
        static_for<B + 1, E>(f);
    }
}

template <int F, int L>
struct Geo {
    static constexpr int TT = 3 * F / 32;  // 32-row tiles of the 3F gate rows
    static constexpr int HT = F / 32;      // 32-row tiles of the hidden state
    static constexpr int KS = F / 2;       // k-steps (2 hidden units each) per matvec
    static constexpr int KG = KS / 4;      // groups of 4 k-steps (one ds_read_b128)
    static constexpr int NG = (L == 2) ? 3 : 1;     // weight images: L0 hh, L1 ih, L1 hh
    static constexpr int G_SIZE = TT * KG * 64 * 4;  // floats per image
    static constexpr int OFF_X = NG * G_SIZE;        // extra k-step A operands [g][t][64]
    static constexpr int OFF_IN = OFF_X + NG * TT * 64;  // layer-0 n-gate input extra [HT][64]
    static constexpr int OFF_WL = OFF_IN + HT * 64;      // linear weights [half][HT][16]
    // bias vectors in accumulator-register order (tile, lane half, register i = row (i&3) + 8(i>>2) + 4 half) for the
    // folded kernel's accumulator initialisation: [b_hh0 n: HT tiles][layer-1 c0: TT tiles][b_hh1 n: HT tiles]
    static constexpr int OFF_CV = OFF_WL + 2 * HT * 16;
    static constexpr int TOTAL = OFF_CV + (2 * HT + TT) * 32;
};

// hidden unit fed by lane half `kk` at k-step s (accumulator row map of the 32x32 MFMA tile)
__host__ __device__ inline int hid_of(int s, int kk) {
    const int i = s & 15;
    return 32 * (s >> 4) + (i & 3) + 8 * (i >> 2) + 4 * kk;
}

struct Args {
    const float* img;
    const f4* wy;
    const float* y;   // NULL: no y input (decoding_type 'y_h0': the RNN input is the previous bit alone)
    const float* h0;  // NULL: zero initial state; else (B, F L), element f L + l = layer l, unit f (get_h0's x)
    const float* gt;
    float* decoded;
    float* logits;
    int64_t B;
    int N;
    int rev;
    int onehot;
    float b_lin;
    uint32_t info[kMaxWords];
    int ln;                // LayerNorm head (gru_decode_kernel only)
    float ln_eps;
    const f4* hd;          // out_linear_depth > 1 head (gru_decode_kernel<.., HDT > 0>): image, depth, last bias
    int hd_depth;
    float hd_bout;
};

__device__ __forceinline__ f16v mfma(float a, float b, const f16v& c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// acc[0..NT) += W_g[tiles t0..t0+NT) . h  over all KS k-steps.  Weight groups (4 k-steps, one
// ds_read_b128 per tile) are read one group ahead of the MFMAs that consume them; the empty asm with a
// memory clobber bounds that look-ahead so the weights of a whole matvec are never hoisted into VGPRs.
template <int TT, int KG, int NT, int HT>
__device__ __forceinline__ void gemm_chain(const f4* __restrict__ smem4, int g, int t0, int lane, f16v (&acc)[NT],
                                           const f16v (&h)[HT]) {
    f4 wc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) wc[t] = smem4[((g * TT + t0 + t) * KG + 0) * 64 + lane];
#pragma unroll
    for (int s4 = 0; s4 < KG; ++s4) {
        f4 wn[NT];
        if (s4 + 1 < KG) {
#pragma unroll
            for (int t = 0; t < NT; ++t) wn[t] = smem4[((g * TT + t0 + t) * KG + s4 + 1) * 64 + lane];
        }
        asm volatile("" ::: "memory");
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int s = 4 * s4 + e;
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[t] = mfma(wc[t][e], h[s >> 4][s & 15], acc[t]);
        }
        if (s4 + 1 < KG) {
#pragma unroll
            for (int t = 0; t < NT; ++t) wc[t] = wn[t];
        }
    }
}

// Gate nonlinearities on the hardware transcendentals (gru_update below): sigmoid(x) = rcp(1 + exp2(-x log2 e)),
// tanh(x) = 2 sigmoid(2x) - 1 (v_exp_f32 / v_rcp_f32, ~1 ulp each; absolute error of tanh ~1e-7 near 0).
// PyTorch's CPU kernels are not bit-reproducible either; the logit tolerance (tests) covers both.

// PyTorch GRUCell update on one 32x32 tile pair: h = (h - n) * z + n,
// r = sigmoid(a_r), z = sigmoid(a_z), n = tanh(a_in + r * a_hn)
// The fp32 MFMAs and this VALU work do not co-issue (PMC: MFMA-busy + VALU-active ~ 1), so the update's
// instruction count is on the critical path: element pairs go through v_pk_mul/add/fma_f32 (two lanes'
// worth of fp32 per instruction); only exp2 / rcp stay scalar.  Same operations and rounding per element.
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v exp2_2(f2v x) { return f2v{__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)}; }
__device__ __forceinline__ f2v rcp_2(f2v x) { return f2v{__builtin_amdgcn_rcpf(x.x), __builtin_amdgcn_rcpf(x.y)}; }

// FOLD: the image's gate rows were pre-multiplied by their exp2 constants (build_image(..., fold)): the accumulators
// already hold -log2(e) a (r, z) and -2 log2(e) a (n), so no scaling multiply per gate
// gemm_chain with the A operands in global memory (the out_linear_depth > 1 head's image: a few KB, the same for every
// wave, so they come from L1 / L2), one group of 4 k-steps ahead of the MFMAs
template <int KG, int NT, int HT>
__device__ __forceinline__ void gemm_chain_g(const f4* __restrict__ W, int lane, f16v (&acc)[NT], const f16v (&h)[HT]) {
    f4 wc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) wc[t] = W[(t * KG) * 64 + lane];
#pragma unroll
    for (int s4 = 0; s4 < KG; ++s4) {
        f4 wn[NT];
        if (s4 + 1 < KG) {
#pragma unroll
            for (int t = 0; t < NT; ++t) wn[t] = W[(t * KG + s4 + 1) * 64 + lane];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int s = 4 * s4 + e;
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[t] = mfma(wc[t][e], h[s >> 4][s & 15], acc[t]);
        }
        if (s4 + 1 < KG) {
#pragma unroll
            for (int t = 0; t < NT; ++t) wc[t] = wn[t];
        }
    }
}

// nn.SELU (the out_linear_depth > 1 head's activation, rnn_all.py:336-343)
__device__ __forceinline__ float selu(float x) {
    return 1.0507009873554805f * (x > 0.0f ? x : 1.6732632423543772f * expm1f(x));
}

// head image (floats): per hidden layer l = 0 .. depth - 2: A operands [HDT tiles][K_l / 8 groups][64 lanes][4] (K_0 = F,
// else 32 HDT), then its bias in accumulator order [HDT][2 halves][16]; then the last Linear's weights [2][HDT][16]
__host__ __device__ inline int head_layer_off(int l, int F, int hdt) {
    return l == 0 ? 0 : hdt * (F / 8) * 256 + hdt * 32 + (l - 1) * (hdt * (4 * hdt) * 256 + hdt * 32);
}

template <bool FOLD = false>
__device__ __forceinline__ void gru_update(f16v& h, const f16v& ar, const f16v& az, const f16v& ain, const f16v& ahn) {
    const f2v one = {1.0f, 1.0f};
    const f2v two = {2.0f, 2.0f};
    // (2x)(-log2 e) == x(-2 log2 e), both exact scalings
    constexpr float k1 = FOLD ? 1.0f : -1.44269504088896340736f, k2 = FOLD ? 1.0f : -2.88539008177792681472f;
#pragma unroll
    for (int i = 0; i < 16; i += 2) {
        f2v er = f2v{ar[i], ar[i + 1]}, ez = f2v{az[i], az[i + 1]};
        if constexpr (!FOLD) {
            er = f2v{k1, k1} * er;
            ez = f2v{k1, k1} * ez;
        }
        const f2v r = rcp_2(one + exp2_2(er));
        const f2v z = rcp_2(one + exp2_2(ez));
        f2v x = f2v{ain[i], ain[i + 1]} + f2v{ahn[i], ahn[i + 1]} * r;
        if constexpr (!FOLD) x = f2v{k2, k2} * x;
        const f2v s2 = rcp_2(one + exp2_2(x));
        const f2v nn = __builtin_elementwise_fma(two, s2, -one);
        const f2v hv = f2v{h[i], h[i + 1]};
        const f2v hn = (hv - nn) * z + nn;
        h[i] = hn.x;
        h[i + 1] = hn.y;
    }
}

// Waves per workgroup of the F <= 64 kernels: all share the workgroup's LDS copy of the weights.  8 waves
// would put two on every SIMD (one wave's gate VALU work overlapping the other's MFMAs), but at <= 256
// registers per wave the F = 64, 2-layer kernel spills (P, both states, the gate accumulators and the
// weight look-ahead need ~300): measured 0.63 of the fp32 MFMA peak vs 0.77 with 4 waves.
#define NPD_GRU_WPB 4  // measured: 8 waves spill 716 B/lane and run 0.63 vs 0.77 of peak
#ifndef NPD_GRU_BF_WPB
#define NPD_GRU_BF_WPB 4
#endif

// The image's gate rows carry their exp2 constants (build_image(..., fold = true)) and the biases initialise the
// accumulators (Geo::OFF_CV): only layer 0's r, z tiles keep the [1, x_i] k-step.  Measured in round 3 (same box,
// alternating, 2^20 Polar(64,32) words): folding 41.0 -> 40.3 ms, bias initialisation 40.07 -> 39.70 ms.
template <int F, int L, int WPB = NPD_GRU_WPB, int HDT = 0>
__global__ __launch_bounds__(64 * WPB) void gru_decode_kernel(const Args a) {
    constexpr bool FOLD = true, BINIT = true;
    using G = Geo<F, L>;
    constexpr int TT = G::TT, HT = G::HT, KG = G::KG;
    extern __shared__ __attribute__((aligned(16))) f4 smem4[];
    const float* smem = reinterpret_cast<const float*>(smem4);
    {
        const f4* src = reinterpret_cast<const f4*>(a.img);
        for (int i = threadIdx.x; i < G::TOTAL / 4; i += blockDim.x) smem4[i] = src[i];
        __syncthreads();
    }
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int half = lane >> 5;
    const int col = lane & 31;
    const int N = a.N;
    const int64_t ntiles = (a.B + 31) / 32;
    const f16v zero = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // this lane's 16 accumulator-row values of a bias vector tile at float offset `off` (Geo::OFF_CV region)
    auto cvec = [&](int off) -> f16v {
        const f4* p = reinterpret_cast<const f4*>(smem + off + half * 16);
        const f4 x0 = p[0], x1 = p[1], x2 = p[2], x3 = p[3];
        return f16v{x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3],
                    x2[0], x2[1], x2[2], x2[3], x3[0], x3[1], x3[2], x3[3]};
    };

    for (int64_t tile = (int64_t)blockIdx.x * WPB + wave; tile < ntiles; tile += (int64_t)gridDim.x * WPB) {
        const int64_t cw = tile * 32 + col;
        const bool valid = cw < a.B;
        const int64_t cwc = valid ? cw : a.B - 1;

        // ---- P = W_ih0[:, :N] . y  (k-step s pairs y[s] (half 0) with y[s + N/2] (half 1))
        f16v P[TT];
#pragma unroll
        for (int t = 0; t < TT; ++t) P[t] = zero;
        if (a.y) {
            const f4* yr = reinterpret_cast<const f4*>(a.y + cwc * N + half * (N / 2));
            const int ng = N / 8;
            for (int s4 = 0; s4 < ng; ++s4) {
                const f4 yv = yr[s4];
#pragma unroll
                for (int t = 0; t < TT; ++t) {
                    const f4 w = a.wy[(t * ng + s4) * 64 + lane];
                    P[t] = mfma(w.x, yv.x, P[t]);
                    P[t] = mfma(w.y, yv.y, P[t]);
                    P[t] = mfma(w.z, yv.z, P[t]);
                    P[t] = mfma(w.w, yv.w, P[t]);
                }
            }
        }

        f16v h0[HT], h1[HT];
#pragma unroll
        for (int t = 0; t < HT; ++t) {
            h0[t] = zero;
            h1[t] = zero;
        }
        if (a.h0) {  // register i of tile t = hidden unit hid_of(16 t + i, half) of codeword col
            const float* hr = a.h0 + cwc * (int64_t)(F * L);
#pragma unroll
            for (int t = 0; t < HT; ++t)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int f = hid_of(16 * t + i, half);
                    h0[t][i] = hr[f * L];
                    if constexpr (L == 2) h1[t][i] = hr[f * L + 1];
                }
        }
        float xb = 1.0f;  // x_i: onehot index of the previous decision (or its sign); step 0: prev = +1
        const float one_or_zero = half ? 0.0f : 1.0f;

        for (int ii = 0; ii < N; ++ii) {
            const int jj = a.rev ? N - 1 - ii : ii;
            const float xbe = half ? xb : 1.0f;  // extra k-step B operand: [1, x_i]
            // ================= layer 0: acc = P + W_hh0 h0 + consts + x_i column
            {
                f16v acc[TT];
#pragma unroll
                for (int t = 0; t < 2 * HT; ++t) acc[t] = P[t];
#pragma unroll
                for (int t = 2 * HT; t < TT; ++t) acc[t] = BINIT ? cvec(G::OFF_CV + (t - 2 * HT) * 32) : zero;
                gemm_chain<TT, KG, TT, HT>(smem4, 0, 0, lane, acc, h0);
                // the [1, x_i] k-step: every tile, or (BINIT: hn tiles start from their bias) the r, z tiles only
#pragma unroll
                for (int t = 0; t < (BINIT ? 2 * HT : TT); ++t) acc[t] = mfma(smem[G::OFF_X + t * 64 + lane], xbe, acc[t]);
#pragma unroll
                for (int j = 0; j < HT; ++j) {
                    const f16v ain = mfma(smem[G::OFF_IN + j * 64 + lane], xbe, P[2 * HT + j]);
                    gru_update<FOLD>(h0[j], acc[j], acc[HT + j], ain, acc[2 * HT + j]);
                }
            }
            if constexpr (L == 2) {
                // ================= layer 1: acc1 = W_ih1 h0' (+ W_hh1 h1 on r,z rows); ahn = W_hh1_n h1
                f16v acc1[TT];
#pragma unroll
                for (int t = 0; t < TT; ++t) acc1[t] = BINIT ? cvec(G::OFF_CV + (HT + t) * 32) : zero;
                gemm_chain<TT, KG, TT, HT>(smem4, 1, 0, lane, acc1, h0);
                if constexpr (!BINIT) {
#pragma unroll
                    for (int t = 0; t < TT; ++t) acc1[t] = mfma(smem[G::OFF_X + (TT + t) * 64 + lane], one_or_zero, acc1[t]);
                }
                f16v arz[2 * HT];
#pragma unroll
                for (int t = 0; t < 2 * HT; ++t) arz[t] = acc1[t];
                gemm_chain<TT, KG, 2 * HT, HT>(smem4, 2, 0, lane, arz, h1);
                f16v ahn[HT];
#pragma unroll
                for (int j = 0; j < HT; ++j) ahn[j] = BINIT ? cvec(G::OFF_CV + (HT + TT + j) * 32) : zero;
                gemm_chain<TT, KG, HT, HT>(smem4, 2, 2 * HT, lane, ahn, h1);
#pragma unroll
                for (int j = 0; j < HT; ++j) {
                    if constexpr (!BINIT) ahn[j] = mfma(smem[G::OFF_X + (2 * TT + 2 * HT + j) * 64 + lane], one_or_zero, ahn[j]);
                    gru_update<FOLD>(h1[j], arz[j], arz[HT + j], acc1[2 * HT + j], ahn[j]);
                }
            }
            // ================= output: Linear(F, 1) on the top layer
            float part = 0.0f;
#pragma unroll
            for (int t = 0; t < HT; ++t) {
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const float wl = smem[G::OFF_WL + (half * HT + t) * 16 + i];
                    part += wl * (L == 2 ? h1[t][i] : h0[t][i]);
                }
            }
            float out;
            if constexpr (HDT > 0) {
                // out_linear_depth > 1 head (rnn_all.py:336-343: Linear(F, H), SELU, [Linear(H, H), SELU] ..., Linear(H, 1)),
                // H padded to 32 HDT with zero rows / columns: each layer is a GEMM whose accumulator tiles are,
                // register for register, the next layer's B operand (as the GRU states are)
                const float* hdf = reinterpret_cast<const float*>(a.hd);
                f16v hx[HDT];
                auto bias_init = [&](int l, f16v (&acc)[HDT]) {
                    const int boff = head_layer_off(l, F, HDT) + HDT * (l == 0 ? F / 8 : 4 * HDT) * 256;
#pragma unroll
                    for (int t = 0; t < HDT; ++t) {
                        const f4* p = reinterpret_cast<const f4*>(hdf + boff + (t * 2 + half) * 16);
                        const f4 x0 = p[0], x1 = p[1], x2 = p[2], x3 = p[3];
                        acc[t] = f16v{x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3],
                                      x2[0], x2[1], x2[2], x2[3], x3[0], x3[1], x3[2], x3[3]};
                    }
                };
                bias_init(0, hx);
                if constexpr (L == 2) gemm_chain_g<F / 8, HDT, HT>(a.hd, lane, hx, h1);
                else gemm_chain_g<F / 8, HDT, HT>(a.hd, lane, hx, h0);
#pragma unroll
                for (int t = 0; t < HDT; ++t)
#pragma unroll
                    for (int i = 0; i < 16; ++i) hx[t][i] = selu(hx[t][i]);
                for (int l = 1; l < a.hd_depth - 1; ++l) {
                    f16v hn[HDT];
                    bias_init(l, hn);
                    gemm_chain_g<4 * HDT, HDT, HDT>(a.hd + head_layer_off(l, F, HDT) / 4, lane, hn, hx);
#pragma unroll
                    for (int t = 0; t < HDT; ++t)
#pragma unroll
                        for (int i = 0; i < 16; ++i) hx[t][i] = selu(hn[t][i]);
                }
                const float* wo = hdf + head_layer_off(a.hd_depth - 1, F, HDT);
                float po = 0.0f;
#pragma unroll
                for (int t = 0; t < HDT; ++t)
#pragma unroll
                    for (int i = 0; i < 16; ++i) po = fmaf(wo[(half * HDT + t) * 16 + i], hx[t][i], po);
                out = po + __shfl_xor(po, 32, 64) + a.hd_bout;
            } else if (a.ln) {
                // LayerNorm head (rnn_all.py:387-398: linear(layernorm(out))): two-pass mean / biased variance over the
                // F units of this codeword, then sum_i w_i gamma_i (h_i - mu) rstd + (b + w . beta) with the
                // gamma-folded weights in the image (npd_rnn_create_ex)
                float s1 = 0.0f;
#pragma unroll
                for (int t = 0; t < HT; ++t)
#pragma unroll
                    for (int i = 0; i < 16; ++i) s1 += L == 2 ? h1[t][i] : h0[t][i];
                const float mu = (s1 + __shfl_xor(s1, 32, 64)) * (1.0f / (float)F);
                float s2 = 0.0f, pw = 0.0f;
#pragma unroll
                for (int t = 0; t < HT; ++t)
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const float d = (L == 2 ? h1[t][i] : h0[t][i]) - mu;
                        s2 = fmaf(d, d, s2);
                        pw = fmaf(smem[G::OFF_WL + (half * HT + t) * 16 + i], d, pw);
                    }
                const float var = (s2 + __shfl_xor(s2, 32, 64)) * (1.0f / (float)F);
                out = (pw + __shfl_xor(pw, 32, 64)) / sqrtf(var + a.ln_eps) + a.b_lin;
            } else {
                out = part + __shfl_xor(part, 32, 64) + a.b_lin;
            }
            const bool info = (a.info[jj >> 5] >> (jj & 31)) & 1u;
            float d;
            if (info) {
                d = out > 0.0f ? 1.0f : (out < 0.0f ? -1.0f : 0.0f);
            } else {
                d = a.gt ? a.gt[cwc * N + jj] : 1.0f;
            }
            if (half == 0 && valid) {
                a.decoded[cw * N + jj] = d;
                if (a.logits) a.logits[cw * N + ii] = out;
            }
            // next input: onehot(sign(d)) -> index (0.5 + 0.5*s).long() (rnn_all.py:258-260); else sign(d)
            const float sd = d > 0.0f ? 1.0f : (d < 0.0f ? -1.0f : 0.0f);
            xb = a.onehot ? (sd > 0.0f ? 1.0f : 0.0f) : sd;
        }
    }
}

// ---------------------------------------------------------------------------------- host image
template <int F, int L>
static void build_image(const float* W, int N, int onehot, std::vector<float>& img, std::vector<float>& wy,
                        float& b_lin, bool fold = false) {
    using G = Geo<F, L>;
    constexpr int TT = G::TT, HT = G::HT, KG = G::KG, KS = G::KS;
    const int Din = N + (onehot ? 2 : 1);
    // unpack
    const float* p = W;
    const float* wih[2];
    const float* whh[2];
    const float* bih[2];
    const float* bhh[2];
    for (int l = 0; l < L; ++l) {
        const int din = l == 0 ? Din : F;
        wih[l] = p; p += (size_t)3 * F * din;
        whh[l] = p; p += (size_t)3 * F * F;
        bih[l] = p; p += 3 * F;
        bhh[l] = p; p += 3 * F;
    }
    const float* wlin = p;
    b_lin = p[F];
    img.assign(G::TOTAL, 0.0f);
    // main k-steps of the three images
    const float* mats[3] = {whh[0], L == 2 ? wih[1] : nullptr, L == 2 ? whh[1] : nullptr};
    // fold: every gate row times its exp2 constant (r, z: -log2 e; n: -2 log2 e; one fp32 rounding), the kernel's
    // gate nonlinearities then take the accumulators as they are (gru_update<true>)
    auto fr = [&](int row) { return fold ? (row < 2 * F ? -1.44269504088896340736f : -2.88539008177792681472f) : 1.0f; };
    for (int g = 0; g < G::NG; ++g)
        for (int t = 0; t < TT; ++t)
            for (int s = 0; s < KS; ++s)
                for (int l = 0; l < 64; ++l) {
                    const int row = 32 * t + (l & 31);
                    const int h = hid_of(s, l >> 5);
                    img[((size_t)(g * TT + t) * KG + s / 4) * 256 + l * 4 + (s & 3)] = fr(row) * mats[g][(size_t)row * F + h];
                }
    // extra k-step A operands: column 0 pairs with B = 1, column 1 with B = x_i (layer 0) / 0 (layer 1)
    for (int t = 0; t < TT; ++t)
        for (int l = 0; l < 64; ++l) {
            const int row = 32 * t + (l & 31);
            const int kk = l >> 5;
            const bool rz = row < 2 * F;
            // layer 0, hidden-side image: r,z rows carry every input-side constant too
            float v0;
            if (kk == 0) {
                v0 = rz ? bih[0][row] + bhh[0][row] + (onehot ? wih[0][(size_t)row * Din + N] : 0.0f) : bhh[0][row];
            } else {
                v0 = rz ? (onehot ? wih[0][(size_t)row * Din + N + 1] - wih[0][(size_t)row * Din + N]
                                  : wih[0][(size_t)row * Din + N])
                        : 0.0f;
            }
            img[G::OFF_X + (0 * TT + t) * 64 + l] = fr(row) * v0;
            if (L == 2) {
                img[G::OFF_X + (1 * TT + t) * 64 + l] = fr(row) * (kk == 0 ? (rz ? bih[1][row] + bhh[1][row] : bih[1][row]) : 0.0f);
                img[G::OFF_X + (2 * TT + t) * 64 + l] = fr(row) * (kk == 0 ? (rz ? 0.0f : bhh[1][row]) : 0.0f);
            }
        }
    for (int j = 0; j < HT; ++j)
        for (int l = 0; l < 64; ++l) {
            const int row = 2 * F + 32 * j + (l & 31);
            const int kk = l >> 5;
            float v;
            if (kk == 0) v = bih[0][row] + (onehot ? wih[0][(size_t)row * Din + N] : 0.0f);
            else v = onehot ? wih[0][(size_t)row * Din + N + 1] - wih[0][(size_t)row * Din + N] : wih[0][(size_t)row * Din + N];
            img[G::OFF_IN + j * 64 + l] = fr(row) * v;
        }
    for (int hf = 0; hf < 2; ++hf)
        for (int t = 0; t < HT; ++t)
            for (int i = 0; i < 16; ++i) img[G::OFF_WL + (hf * HT + t) * 16 + i] = wlin[32 * t + (i & 3) + 8 * (i >> 2) + 4 * hf];
    for (int v = 0; v < 2 * HT + TT; ++v)
        for (int hf = 0; hf < 2; ++hf)
            for (int i = 0; i < 16; ++i) {
                const int r = (i & 3) + 8 * (i >> 2) + 4 * hf;
                float val = 0.0f;
                int row;
                if (v < HT) {  // layer-0 hn bias
                    row = 2 * F + 32 * v + r;
                    val = bhh[0][row];
                } else if (v < HT + TT) {  // layer-1 r, z (both biases) / in (b_ih) constants
                    row = 32 * (v - HT) + r;
                    val = L == 2 ? (row < 2 * F ? bih[1][row] + bhh[1][row] : bih[1][row]) : 0.0f;
                } else {  // layer-1 hn bias
                    row = 2 * F + 32 * (v - HT - TT) + r;
                    val = L == 2 ? bhh[1][row] : 0.0f;
                }
                img[G::OFF_CV + (v * 2 + hf) * 16 + i] = fr(row) * val;
            }
    // y projection: k-step s pairs y[s] (lanes 0-31) with y[s + N/2] (lanes 32-63)
    const int ng = N / 8;
    wy.assign((size_t)TT * ng * 256, 0.0f);
    for (int t = 0; t < TT; ++t)
        for (int s = 0; s < N / 2; ++s)
            for (int l = 0; l < 64; ++l) {
                const int row = 32 * t + (l & 31);
                const int k = s + (l >> 5) * (N / 2);
                wy[((size_t)t * ng + s / 4) * 256 + l * 4 + (s & 3)] = fr(row) * wih[0][(size_t)row * Din + k];
            }
}

// the out_linear_depth > 1 head's image (layout: head_layer_off): hw = the Sequential's Linear layers in order, W_0 (H, F),
// b_0 (H), [W_l (H, H), b_l (H)] for l = 1 .. depth - 2, W_last (1, H), b_last (1); H padded to 32 hdt with zeros
static void build_head_image(const float* hw, int F, int H, int depth, int hdt, std::vector<float>& img, float& bout) {
    const int HP = 32 * hdt;
    img.assign((size_t)head_layer_off(depth - 1, F, hdt) + 2 * hdt * 16, 0.0f);
    const float* p = hw;
    for (int l = 0; l < depth - 1; ++l) {
        const int K = l == 0 ? F : H, KP = l == 0 ? F : HP, KG = KP / 8;
        const float* W = p;
        const float* b = p + (size_t)H * K;
        p = b + H;
        float* im = img.data() + head_layer_off(l, F, hdt);
        for (int t = 0; t < hdt; ++t)
            for (int s = 0; s < KP / 2; ++s)
                for (int ln = 0; ln < 64; ++ln) {
                    const int row = 32 * t + (ln & 31), k = hid_of(s, ln >> 5);
                    im[((size_t)(t * KG + s / 4) * 64 + ln) * 4 + (s & 3)] = row < H && k < K ? W[(size_t)row * K + k] : 0.0f;
                }
        float* bv = im + (size_t)hdt * KG * 256;
        for (int t = 0; t < hdt; ++t)
            for (int hf = 0; hf < 2; ++hf)
                for (int i = 0; i < 16; ++i) {
                    const int row = 32 * t + (i & 3) + 8 * (i >> 2) + 4 * hf;
                    bv[(t * 2 + hf) * 16 + i] = row < H ? b[row] : 0.0f;
                }
    }
    float* wo = img.data() + head_layer_off(depth - 1, F, hdt);
    for (int hf = 0; hf < 2; ++hf)
        for (int t = 0; t < hdt; ++t)
            for (int i = 0; i < 16; ++i) {
                const int k = hid_of(16 * t + i, hf);
                wo[(hf * hdt + t) * 16 + i] = k < H ? p[k] : 0.0f;
            }
    bout = p[H];
}

template <int F, int L, int HDT = 0>
static int launch(const Args& a, hipStream_t s) {
    using G = Geo<F, L>;
    constexpr int WPB = NPD_GRU_WPB;
    auto kern = gru_decode_kernel<F, L, WPB, HDT>;
    const size_t lds = (size_t)G::TOTAL * 4;
    static bool attr = false;
    if (!attr) {
        NPD_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
        attr = true;
    }
    const int64_t tiles = (a.B + 31) / 32;
    const int64_t wgs = (tiles + WPB - 1) / WPB;
    const int grid = grid_for(wgs, 1, device_cu_count());
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * WPB), lds, s, a);
    return launch_check("gru_decode_kernel launch");
}

// =============================================================================== LSTM cells (fp32, F <= 64)
// rnn_all.py:69 offers --rnn_type LSTM; RNN_decoder's y_input test branch then carries (h, c) pairs (rnn_all.py:536-547)
// through nn.LSTM: gates i, f, g, o (PyTorch row order) = W_ih x + b_ih + W_hh h + b_hh, c' = sig(f) c + sig(i) tanh(g),
// h' = sig(o) tanh(c').  Same layout as gru_decode_kernel with 4F gate rows: images [L0 hh | L1 ih | L1 hh] of 4F x F in
// A-operand order, every gate row pre-multiplied by its exp2 constant (i, f, o: -log2 e; g: -2 log2 e), all biases
// (+ the one-hot column 0 on layer 0) as accumulator initialisation, the x_i column one [1, x_i] k-step on layer 0.
template <int F, int L>
struct LGeo {
    static constexpr int TT = 4 * F / 32;
    static constexpr int HT = F / 32;
    static constexpr int KS = F / 2;
    static constexpr int KG = KS / 4;
    static constexpr int NG = (L == 2) ? 3 : 1;
    static constexpr int G_SIZE = TT * KG * 64 * 4;
    static constexpr int OFF_X = NG * G_SIZE;           // layer-0 [1, x_i] k-step A operands [TT][64]
    static constexpr int OFF_WL = OFF_X + TT * 64;       // linear weights [half][HT][16]
    static constexpr int OFF_CV = OFF_WL + 2 * HT * 16;  // bias tiles in accumulator order: [layer][TT][half][16]
    static constexpr int TOTAL = OFF_CV + L * TT * 32;
};

__device__ __forceinline__ float sig2(float a) { return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(a)); }

template <int F, int L>
__global__ __launch_bounds__(64 * NPD_GRU_WPB) void lstm_decode_kernel(const Args a) {
    using G = LGeo<F, L>;
    constexpr int TT = G::TT, HT = G::HT, KG = G::KG;
    extern __shared__ __attribute__((aligned(16))) f4 smem4[];
    const float* smem = reinterpret_cast<const float*>(smem4);
    {
        const f4* src = reinterpret_cast<const f4*>(a.img);
        for (int i = threadIdx.x; i < G::TOTAL / 4; i += blockDim.x) smem4[i] = src[i];
        __syncthreads();
    }
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int half = lane >> 5;
    const int col = lane & 31;
    const int N = a.N;
    const int64_t ntiles = (a.B + 31) / 32;
    const f16v zero = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    auto cvec = [&](int off) -> f16v {
        const f4* p = reinterpret_cast<const f4*>(smem + off + half * 16);
        const f4 x0 = p[0], x1 = p[1], x2 = p[2], x3 = p[3];
        return f16v{x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3],
                    x2[0], x2[1], x2[2], x2[3], x3[0], x3[1], x3[2], x3[3]};
    };
    constexpr float kT = -2.88539008177792681472f;  // tanh(c) = 2 sig2(kT c) - 1
    for (int64_t tile = (int64_t)blockIdx.x * NPD_GRU_WPB + wave; tile < ntiles; tile += (int64_t)gridDim.x * NPD_GRU_WPB) {
        const int64_t cw = tile * 32 + col;
        const bool valid = cw < a.B;
        const int64_t cwc = valid ? cw : a.B - 1;
        f16v P[TT];
#pragma unroll
        for (int t = 0; t < TT; ++t) P[t] = cvec(G::OFF_CV + t * 32);
        if (a.y) {  // y = NULL: decoding_type y_h0 (no y input; the state starts from the y-MLP's output)
            const f4* yr = reinterpret_cast<const f4*>(a.y + cwc * N + half * (N / 2));
            const int ng = N / 8;
            for (int s4 = 0; s4 < ng; ++s4) {
                const f4 yv = yr[s4];
#pragma unroll
                for (int t = 0; t < TT; ++t) {
                    const f4 w = a.wy[(t * ng + s4) * 64 + lane];
                    P[t] = mfma(w.x, yv.x, P[t]);
                    P[t] = mfma(w.y, yv.y, P[t]);
                    P[t] = mfma(w.z, yv.z, P[t]);
                    P[t] = mfma(w.w, yv.w, P[t]);
                }
            }
        }
        f16v h0[HT], c0[HT], h1[HT], c1[HT];
#pragma unroll
        for (int t = 0; t < HT; ++t) {
            h0[t] = zero;
            c0[t] = zero;
            h1[t] = zero;
            c1[t] = zero;
        }
        if (a.h0) {  // y_h0: get_h0 returns (x, x) for LSTM cells (rnn_all.py:370-375): h and c both start from x
            const float* hr = a.h0 + cwc * (int64_t)(F * L);
#pragma unroll
            for (int t = 0; t < HT; ++t)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int f = hid_of(16 * t + i, half);
                    h0[t][i] = c0[t][i] = hr[f * L];
                    if constexpr (L == 2) h1[t][i] = c1[t][i] = hr[f * L + 1];
                }
        }
        float xb = 1.0f;
        auto cell = [&](f16v& h, f16v& c, const f16v (&acc)[TT], int j) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float ig = sig2(acc[j][i]), fg = sig2(acc[HT + j][i]);
                const float gg = fmaf(2.0f, sig2(acc[2 * HT + j][i]), -1.0f);
                const float og = sig2(acc[3 * HT + j][i]);
                c[i] = fmaf(fg, c[i], ig * gg);
                h[i] = og * fmaf(2.0f, sig2(kT * c[i]), -1.0f);
            }
        };
        for (int ii = 0; ii < N; ++ii) {
            const int jj = a.rev ? N - 1 - ii : ii;
            const float xbe = half ? xb : 1.0f;
            {
                f16v acc[TT];
#pragma unroll
                for (int t = 0; t < TT; ++t) acc[t] = mfma(smem[G::OFF_X + t * 64 + lane], xbe, P[t]);
                gemm_chain<TT, KG, TT, HT>(smem4, 0, 0, lane, acc, h0);
#pragma unroll
                for (int j = 0; j < HT; ++j) cell(h0[j], c0[j], acc, j);
            }
            if constexpr (L == 2) {
                f16v acc1[TT];
#pragma unroll
                for (int t = 0; t < TT; ++t) acc1[t] = cvec(G::OFF_CV + (TT + t) * 32);
                gemm_chain<TT, KG, TT, HT>(smem4, 1, 0, lane, acc1, h0);
                gemm_chain<TT, KG, TT, HT>(smem4, 2, 0, lane, acc1, h1);
#pragma unroll
                for (int j = 0; j < HT; ++j) cell(h1[j], c1[j], acc1, j);
            }
            float part = 0.0f;
#pragma unroll
            for (int t = 0; t < HT; ++t)
#pragma unroll
                for (int i = 0; i < 16; ++i) part += smem[G::OFF_WL + (half * HT + t) * 16 + i] * (L == 2 ? h1[t][i] : h0[t][i]);
            const float out = part + __shfl_xor(part, 32, 64) + a.b_lin;
            const bool info = (a.info[jj >> 5] >> (jj & 31)) & 1u;
            float d;
            if (info) d = out > 0.0f ? 1.0f : (out < 0.0f ? -1.0f : 0.0f);
            else d = a.gt ? a.gt[cwc * N + jj] : 1.0f;
            if (half == 0 && valid) {
                a.decoded[cw * N + jj] = d;
                if (a.logits) a.logits[cw * N + ii] = out;
            }
            const float sd = d > 0.0f ? 1.0f : (d < 0.0f ? -1.0f : 0.0f);
            xb = a.onehot ? (sd > 0.0f ? 1.0f : 0.0f) : sd;
        }
    }
}

// host image of lstm_decode_kernel from the npd_gru_create weight order with 4F gate rows
template <int F, int L>
static void build_image_lstm(const float* W, int N, int onehot, std::vector<float>& img, std::vector<float>& wy,
                             float& b_lin) {
    using G = LGeo<F, L>;
    constexpr int TT = G::TT, HT = G::HT, KG = G::KG, KS = G::KS;
    const int Din = N + (onehot ? 2 : 1);
    const float* p = W;
    const float *wih[2], *whh[2], *bih[2], *bhh[2];
    for (int l = 0; l < L; ++l) {
        const int din = l == 0 ? Din : F;
        wih[l] = p; p += (size_t)4 * F * din;
        whh[l] = p; p += (size_t)4 * F * F;
        bih[l] = p; p += 4 * F;
        bhh[l] = p; p += 4 * F;
    }
    const float* wlin = p;
    b_lin = p[F];
    img.assign(G::TOTAL, 0.0f);
    auto fr = [&](int row) { return (row >= 2 * F && row < 3 * F) ? -2.88539008177792681472f : -1.44269504088896340736f; };
    const float* mats[3] = {whh[0], L == 2 ? wih[1] : nullptr, L == 2 ? whh[1] : nullptr};
    for (int g = 0; g < G::NG; ++g)
        for (int t = 0; t < TT; ++t)
            for (int s = 0; s < KS; ++s)
                for (int l = 0; l < 64; ++l) {
                    const int row = 32 * t + (l & 31);
                    img[((size_t)(g * TT + t) * KG + s / 4) * 256 + l * 4 + (s & 3)] =
                        fr(row) * mats[g][(size_t)row * F + hid_of(s, l >> 5)];
                }
    // layer-0 [1, x_i] k-step: half 0 pairs with 1 (nothing left: the one-hot column 0 is in the bias tile), half 1
    // with x_i (one-hot: column 1 - column 0; sign input: its column)
    for (int t = 0; t < TT; ++t)
        for (int l = 32; l < 64; ++l) {
            const int row = 32 * t + (l & 31);
            const float v = onehot ? wih[0][(size_t)row * Din + N + 1] - wih[0][(size_t)row * Din + N]
                                   : wih[0][(size_t)row * Din + N];
            img[G::OFF_X + t * 64 + l] = fr(row) * v;
        }
    for (int hf = 0; hf < 2; ++hf)
        for (int t = 0; t < HT; ++t)
            for (int i = 0; i < 16; ++i) img[G::OFF_WL + (hf * HT + t) * 16 + i] = wlin[32 * t + (i & 3) + 8 * (i >> 2) + 4 * hf];
    for (int l = 0; l < L; ++l)
        for (int t = 0; t < TT; ++t)
            for (int hf = 0; hf < 2; ++hf)
                for (int i = 0; i < 16; ++i) {
                    const int row = 32 * t + (i & 3) + 8 * (i >> 2) + 4 * hf;
                    float v = bih[l][row] + bhh[l][row];
                    if (l == 0 && onehot) v += wih[0][(size_t)row * Din + N];
                    img[G::OFF_CV + ((l * TT + t) * 2 + hf) * 16 + i] = fr(row) * v;
                }
    const int ng = N / 8;
    wy.assign((size_t)TT * ng * 256, 0.0f);
    for (int t = 0; t < TT; ++t)
        for (int s = 0; s < N / 2; ++s)
            for (int l = 0; l < 64; ++l) {
                const int row = 32 * t + (l & 31);
                const int k = s + (l >> 5) * (N / 2);
                wy[((size_t)t * ng + s / 4) * 256 + l * 4 + (s & 3)] = fr(row) * wih[0][(size_t)row * Din + k];
            }
}

template <int F, int L>
static int launch_lstm(const Args& a, hipStream_t s) {
    using G = LGeo<F, L>;
    auto kern = lstm_decode_kernel<F, L>;
    const size_t lds = (size_t)G::TOTAL * 4;
    static bool attr = false;
    if (!attr) {
        NPD_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
        attr = true;
    }
    const int64_t tiles = (a.B + 31) / 32;
    const int64_t wgs = (tiles + NPD_GRU_WPB - 1) / NPD_GRU_WPB;
    hipLaunchKernelGGL(kern, dim3(grid_for(wgs, 1, device_cu_count())), dim3(64 * NPD_GRU_WPB), lds, s, a);
    return launch_check("lstm_decode_kernel launch");
}

// =============================================================================== split 16-bit MFMA paths
// precision 1 = bf16x3 split (a*b ~ ah*bh + ah*bl + al*bh, ~2^-16 relative per product),
// precision 2 = plain bf16 (fp32 accumulate).  v_mfma_f32_32x32x16_bf16: 16x the fp32 MFMA rate.
// precision 3 = fp16x3 split ("SPLIT 4" below): the same three products on v_mfma_f32_32x32x16_f16, whose
// 11-bit significands make hi + lo a 22-bit split (a*b to ~2^-21 relative: fp32-class, against bf16x3's
// 2^-16).  fp16's exponent range is handled by exact power-of-2 scaling: weights (and the y projection's
// weights) x 2^8 on the host, states and received words x 2^8 at the split, so every accumulator holds
// 2^16 x its value (biases / one-hot constants pre-scaled by 2^16, and the gate nonlinearities take the
// 2^-16 in their exp2 constants: all exact).  Then hi and lo stay normal fp16 for |w| >= 5e-4 and
// |h| >= 5e-4 (smaller terms contribute below 2^-33 absolute).
// Same orientation as the fp32 kernel: an h' accumulator tile converts register-for-register into
// the B fragments of the next step (registers 8s..8s+7 -> k-step s, cdna_hip_programming.md sec. 3).
// Bias / one-hot / previous-decision terms stay an exact fp32 k-step (v_mfma_f32_32x32x2_f32).
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef _Float16 hf8 __attribute__((ext_vector_type(8)));

// SPLIT: 1 = bf16, 3 = bf16 hi + lo, 4 = fp16 hi + lo (scaled), 5 = fp16 hi + lo, unscaled, gate constants folded
// into the weights (16-codeword kernels only, see build_image16)
template <int SPLIT>
struct SplitT {
    static constexpr bool kLo = SPLIT >= 3;
    static constexpr bool kF16 = SPLIT >= 4;
    static constexpr bool kFold = SPLIT == 5;  // accumulators hold -log2(e) a (r, z rows) / -2 log2(e) a (n rows)
    using V = std::conditional_t<kF16, hf8, bf8>;
    using E = std::conditional_t<kF16, _Float16, __bf16>;
    static constexpr float kIn = SPLIT == 4 ? 256.0f : 1.0f;           // B-operand scale (states, y)
    static constexpr float kAcc = SPLIT == 4 ? 1.0f / 65536.0f : 1.0f;  // accumulator -> value
    // exp2 arguments of sigmoid(a) = 1 / (1 + 2^(c1 a)) and tanh(x) = 2 / (1 + 2^(c2 x)) - 1 from the accumulators
    static constexpr float kC1 = kFold ? 1.0f : -1.44269504088896340736f * kAcc;
    static constexpr float kC2 = kFold ? 1.0f : -2.88539008177792681472f * kAcc;
};

template <int F, int L, int SPLIT>
struct GeoB {
    static constexpr int TT = 3 * F / 32, HT = F / 32, KB = F / 16;
    static constexpr int NG = (L == 2) ? 3 : 1;
    static constexpr int IMG = NG * TT * KB * 64 * 4;  // floats: one 16-B bf16x8 fragment per lane per step
    static constexpr int NS = SPLIT >= 3 ? 2 : 1;      // hi (+ lo) images
    static constexpr int OFF_X = NS * IMG;
    static constexpr int OFF_IN = OFF_X + NG * TT * 64;
    static constexpr int OFF_WL = OFF_IN + HT * 64;
    static constexpr int TOTAL = OFF_WL + 2 * HT * 16;
};

struct ArgsB {
    const float* img;
    const f4* wy;  // [TT][N/16][64] bf16x8 fragments (hi, then lo for SPLIT 3)
    const float* y;   // NULL: no y input (y_h0)
    const float* h0;  // NULL: zero initial state; else (B, F L) as Args::h0 (16-codeword kernel only)
    const float* gt;
    float* decoded;
    float* logits;
    int64_t B;
    int N;
    int rev;
    int onehot;
    float b_lin;
    int64_t wy_lo;  // offset (in f4) of the lo Wy image
    uint32_t info[kMaxWords];
    // sweep / count mode (gru16p_kernel only): y, decoded and logits are nseg segments of (B, N) back to back; with
    // counters != NULL the decision at position jj is compared with msg[cw][slot[jj]] (slot 255: not compared) and
    // counters[2 s], [2 s + 1] += bit / block errors of segment s (npd_gru_decode_count_sweep)
    const float* msg;
    unsigned long long* counters;
    int K;
    int nseg;
    uint32_t slotw[kMaxN / 4];  // byte jj & 3 of word jj >> 2 = slot of position jj (scalar-loaded per step)
};

__device__ __forceinline__ f16v mfma16(const bf8& a, const bf8& b, const f16v& c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f16v mfma16(const hf8& a, const hf8& b, const f16v& c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}


// the gate pre-activations arrive as ACC x their value (ACC a power of 2): folded into the exp2 constants
template <int SPLIT>
__device__ __forceinline__ void gru_update_fast(f16v& h, const f16v& ar, const f16v& az, const f16v& ain,
                                                const f16v& ahn) {
    constexpr float c1 = SplitT<SPLIT>::kC1, c2 = SplitT<SPLIT>::kC2;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const float r = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(c1 * ar[i]));
        const float z = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(c1 * az[i]));
        const float x = ain[i] + ahn[i] * r;
        const float nn = fmaf(2.0f, __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(c2 * x)), -1.0f);
        h[i] = (h[i] - nn) * z + nn;
    }
}

// split the state tiles into 16-bit B fragments (hi and, for SPLIT 3 / 4, lo)
template <int HT, int SPLIT>
__device__ __forceinline__ void to_frags(const f16v (&h)[HT], typename SplitT<SPLIT>::V (&hi)[2 * HT],
                                         typename SplitT<SPLIT>::V (&lo)[2 * HT]) {
    using S = SplitT<SPLIT>;
#pragma unroll
    for (int t = 0; t < HT; ++t)
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float v = h[t][8 * s + j] * S::kIn;
                const typename S::E b = (typename S::E)v;
                hi[2 * t + s][j] = b;
                if (S::kLo) lo[2 * t + s][j] = (typename S::E)(v - (float)b);
            }
}

template <int TT, int KB, int NT, int SPLIT, int IMG>
__device__ __forceinline__ void gemm_bf(const f4* __restrict__ smem4, int g, int t0, int lane, f16v (&acc)[NT],
                                        const typename SplitT<SPLIT>::V (&hi)[KB],
                                        const typename SplitT<SPLIT>::V (&lo)[KB]) {
    using V = typename SplitT<SPLIT>::V;
#pragma unroll
    for (int q = 0; q < KB; ++q) {
        V ah[NT], al[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const f4 v = smem4[((g * TT + t0 + t) * KB + q) * 64 + lane];
            ah[t] = __builtin_bit_cast(V, v);
            if (SplitT<SPLIT>::kLo)
                al[t] = __builtin_bit_cast(V, smem4[IMG / 4 + ((g * TT + t0 + t) * KB + q) * 64 + lane]);
        }
        asm volatile("" ::: "memory");
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            acc[t] = mfma16(ah[t], hi[q], acc[t]);
            if (SplitT<SPLIT>::kLo) {
                acc[t] = mfma16(ah[t], lo[q], acc[t]);
                acc[t] = mfma16(al[t], hi[q], acc[t]);
            }
        }
    }
}

template <int F, int L, int SPLIT>
__global__ __launch_bounds__(64 * NPD_GRU_BF_WPB) void gru_decode_bf_kernel(const ArgsB a) {
    using G = GeoB<F, L, SPLIT>;
    using S = SplitT<SPLIT>;
    using V = typename S::V;
    using E = typename S::E;
    constexpr int TT = G::TT, HT = G::HT, KB = G::KB, IMG = G::IMG;
    extern __shared__ __attribute__((aligned(16))) f4 smem4[];
    const float* smem = reinterpret_cast<const float*>(smem4);
    {
        const f4* src = reinterpret_cast<const f4*>(a.img);
        for (int i = threadIdx.x; i < G::TOTAL / 4; i += blockDim.x) smem4[i] = src[i];
        __syncthreads();
    }
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int half = lane >> 5;
    const int col = lane & 31;
    const int N = a.N;
    const int64_t ntiles = (a.B + 31) / 32;
    const f16v zero = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const float one_or_zero = half ? 0.0f : 1.0f;

    for (int64_t tile = (int64_t)blockIdx.x * NPD_GRU_BF_WPB + wave; tile < ntiles;
         tile += (int64_t)gridDim.x * NPD_GRU_BF_WPB) {
        const int64_t cw = tile * 32 + col;
        const bool valid = cw < a.B;
        const int64_t cwc = valid ? cw : a.B - 1;
        // ---- P = W_ih0[:, :N] . y ; k-step q covers y[16q + 8*half .. +7]
        f16v P[TT];
#pragma unroll
        for (int t = 0; t < TT; ++t) P[t] = zero;
        {
            const float* yr = a.y + cwc * N;
            const int nq = N / 16;
            for (int q = 0; q < nq; ++q) {
                const f4 y0 = *reinterpret_cast<const f4*>(yr + 16 * q + 8 * half);
                const f4 y1 = *reinterpret_cast<const f4*>(yr + 16 * q + 8 * half + 4);
                V yh, yl;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float v = (j < 4 ? y0[j] : y1[j - 4]) * S::kIn;
                    yh[j] = (E)v;
                    if (S::kLo) yl[j] = (E)(v - (float)yh[j]);
                }
#pragma unroll
                for (int t = 0; t < TT; ++t) {
                    const V wh = __builtin_bit_cast(V, a.wy[(t * nq + q) * 64 + lane]);
                    P[t] = mfma16(wh, yh, P[t]);
                    if (S::kLo) {
                        const V wl = __builtin_bit_cast(V, a.wy[a.wy_lo + (t * nq + q) * 64 + lane]);
                        P[t] = mfma16(wh, yl, P[t]);
                        P[t] = mfma16(wl, yh, P[t]);
                    }
                }
            }
        }
        f16v h0[HT], h1[HT];
#pragma unroll
        for (int t = 0; t < HT; ++t) {
            h0[t] = zero;
            h1[t] = zero;
        }
        float xb = 1.0f;
        // B fragments of h0: split once per update, used by layer 1 of this step and layer 0 of the next
        V fh[KB], fl[KB];
        to_frags<HT, SPLIT>(h0, fh, fl);
        for (int ii = 0; ii < N; ++ii) {
            const int jj = a.rev ? N - 1 - ii : ii;
            const float xbe = half ? xb : 1.0f;
            {
                f16v acc[TT];
#pragma unroll
                for (int t = 0; t < 2 * HT; ++t) acc[t] = P[t];
#pragma unroll
                for (int t = 2 * HT; t < TT; ++t) acc[t] = zero;
                gemm_bf<TT, KB, TT, SPLIT, IMG>(smem4, 0, 0, lane, acc, fh, fl);
#pragma unroll
                for (int t = 0; t < TT; ++t) acc[t] = mfma(smem[G::OFF_X + t * 64 + lane], xbe, acc[t]);
#pragma unroll
                for (int j = 0; j < HT; ++j) {
                    const f16v ain = mfma(smem[G::OFF_IN + j * 64 + lane], xbe, P[2 * HT + j]);
                    gru_update_fast<SPLIT>(h0[j], acc[j], acc[HT + j], ain, acc[2 * HT + j]);
                }
            }
            if constexpr (L == 1) to_frags<HT, SPLIT>(h0, fh, fl);
            if constexpr (L == 2) {
                V gh[KB], gl[KB];
                to_frags<HT, SPLIT>(h0, fh, fl);
                to_frags<HT, SPLIT>(h1, gh, gl);
                f16v acc1[TT];
#pragma unroll
                for (int t = 0; t < TT; ++t) acc1[t] = zero;
                gemm_bf<TT, KB, TT, SPLIT, IMG>(smem4, 1, 0, lane, acc1, fh, fl);
#pragma unroll
                for (int t = 0; t < TT; ++t) acc1[t] = mfma(smem[G::OFF_X + (TT + t) * 64 + lane], one_or_zero, acc1[t]);
                f16v arz[2 * HT];
#pragma unroll
                for (int t = 0; t < 2 * HT; ++t) arz[t] = acc1[t];
                gemm_bf<TT, KB, 2 * HT, SPLIT, IMG>(smem4, 2, 0, lane, arz, gh, gl);
                f16v ahn[HT];
#pragma unroll
                for (int j = 0; j < HT; ++j) ahn[j] = zero;
                gemm_bf<TT, KB, HT, SPLIT, IMG>(smem4, 2, 2 * HT, lane, ahn, gh, gl);
#pragma unroll
                for (int j = 0; j < HT; ++j) {
                    ahn[j] = mfma(smem[G::OFF_X + (2 * TT + 2 * HT + j) * 64 + lane], one_or_zero, ahn[j]);
                    gru_update_fast<SPLIT>(h1[j], arz[j], arz[HT + j], acc1[2 * HT + j], ahn[j]);
                }
            }
            float part = 0.0f;
#pragma unroll
            for (int t = 0; t < HT; ++t)
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    part += smem[G::OFF_WL + (half * HT + t) * 16 + i] * (L == 2 ? h1[t][i] : h0[t][i]);
            const float out = part + __shfl_xor(part, 32, 64) + a.b_lin;
            const bool info = (a.info[jj >> 5] >> (jj & 31)) & 1u;
            float d;
            if (info) d = out > 0.0f ? 1.0f : (out < 0.0f ? -1.0f : 0.0f);
            else d = a.gt ? a.gt[cwc * N + jj] : 1.0f;
            if (half == 0 && valid) {
                a.decoded[cw * N + jj] = d;
                if (a.logits) a.logits[cw * N + ii] = out;
            }
            const float sd = d > 0.0f ? 1.0f : (d < 0.0f ? -1.0f : 0.0f);
            xb = a.onehot ? (sd > 0.0f ? 1.0f : 0.0f) : sd;
        }
    }
}

static uint16_t bf16_rne(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0;  // NaN
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}
static float bf16_to_f(uint16_t b) {
    uint32_t u = (uint32_t)b << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}
// IEEE binary16, round to nearest even (finite inputs within the fp16 range; subnormals handled)
static uint16_t f16_rne(float f) {
    const _Float16 h = (_Float16)f;  // clang lowers the host conversion with round-to-nearest-even
    uint16_t b;
    memcpy(&b, &h, 2);
    return b;
}
static float f16_to_f(uint16_t b) {
    _Float16 h;
    memcpy(&h, &b, 2);
    return (float)h;
}
// 16-bit split of v: SPLIT 4 -> fp16 of v * 2^8; SPLIT 5 -> fp16 of v (lo may be subnormal); else bf16 of v
template <int SPLIT>
static void split16(float v, uint16_t& hi, uint16_t& lo) {
    if (SPLIT >= 4) {
        const float s = SPLIT == 4 ? v * 256.0f : v;
        hi = f16_rne(s);
        lo = f16_rne(s - f16_to_f(hi));
    } else {
        hi = bf16_rne(v);
        lo = bf16_rne(v - bf16_to_f(hi));
    }
}

// img: fp32 image of GeoB (bf16 fragments stored as raw bytes inside the float array)
template <int F, int L, int SPLIT>
static void build_image_bf(const float* W, int N, int onehot, std::vector<float>& img, std::vector<float>& wy,
                           float& b_lin, int64_t& wy_lo) {
    using GB = GeoB<F, L, SPLIT>;
    using G32 = Geo<F, L>;
    constexpr int TT = GB::TT, HT = GB::HT, KB = GB::KB;
    // reuse the fp32 builder for the extra / input / linear constants
    std::vector<float> img32, wy32;
    build_image<F, L>(W, N, onehot, img32, wy32, b_lin);
    img.assign(GB::TOTAL, 0.0f);
    const int Din = N + (onehot ? 2 : 1);
    const float* p = W;
    const float* wih[2];
    const float* whh[2];
    for (int l = 0; l < L; ++l) {
        const int din = l == 0 ? Din : F;
        wih[l] = p; p += (size_t)3 * F * din;
        whh[l] = p; p += (size_t)3 * F * F;
        p += 6 * F;
    }
    const float* mats[3] = {whh[0], L == 2 ? wih[1] : nullptr, L == 2 ? whh[1] : nullptr};
    uint16_t* u16 = reinterpret_cast<uint16_t*>(img.data());
    for (int g = 0; g < GB::NG; ++g)
        for (int t = 0; t < TT; ++t)
            for (int q = 0; q < KB; ++q)
                for (int l = 0; l < 64; ++l)
                    for (int j = 0; j < 8; ++j) {
                        const int row = 32 * t + (l & 31), hh = l >> 5;
                        const int th = q >> 1, s = q & 1;
                        const int colk = 32 * th + 16 * s + 8 * (j >> 2) + 4 * hh + (j & 3);
                        const float v = mats[g][(size_t)row * F + colk];
                        uint16_t hi, lo;
                        split16<SPLIT>(v, hi, lo);
                        const size_t e = ((((size_t)(g * TT + t) * KB + q) * 64 + l) * 8 + j);
                        u16[e] = hi;
                        if (SPLIT >= 3) u16[(size_t)GB::IMG * 2 + e] = lo;
                    }
    // the [1, x] k-step constants enter the accumulators directly: x 2^16 for the scaled fp16 split
    const float kc = SPLIT == 4 ? 65536.0f : 1.0f;
    for (int i = 0; i < GB::NG * TT * 64; ++i) img[GB::OFF_X + i] = img32[G32::OFF_X + i] * kc;
    for (int i = 0; i < HT * 64; ++i) img[GB::OFF_IN + i] = img32[G32::OFF_IN + i] * kc;
    for (int i = 0; i < 2 * HT * 16; ++i) img[GB::OFF_WL + i] = img32[G32::OFF_WL + i];
    // y projection fragments: k-step q pairs lanes' y[16q + 8h + j]
    const int nq = N / 16;
    const size_t per = (size_t)TT * nq * 64 * 8;  // bf16 elements per image
    wy.assign((per * (SPLIT >= 3 ? 2 : 1) + 1) / 2, 0.0f);
    uint16_t* w16 = reinterpret_cast<uint16_t*>(wy.data());
    for (int t = 0; t < TT; ++t)
        for (int q = 0; q < nq; ++q)
            for (int l = 0; l < 64; ++l)
                for (int j = 0; j < 8; ++j) {
                    const int row = 32 * t + (l & 31);
                    const int k = 16 * q + 8 * (l >> 5) + j;
                    const float v = wih[0][(size_t)row * Din + k];
                    const size_t e = (((size_t)t * nq + q) * 64 + l) * 8 + j;
                    uint16_t hi, lo;
                    split16<SPLIT>(v, hi, lo);
                    w16[e] = hi;
                    if (SPLIT >= 3) w16[per + e] = lo;
                }
    wy_lo = (int64_t)(per / 8);  // in 16-B fragments
}

template <int F, int L, int SPLIT>
static int launch_bf(const npd_gru* g, const ArgsB& a, hipStream_t s) {
    using G = GeoB<F, L, SPLIT>;
    auto kern = gru_decode_bf_kernel<F, L, SPLIT>;
    const size_t lds = (size_t)G::TOTAL * 4;
    static bool attr = false;
    if (!attr) {
        NPD_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
        attr = true;
    }
    const int64_t tiles = (a.B + 31) / 32;
    const int64_t wgs = (tiles + NPD_GRU_BF_WPB - 1) / NPD_GRU_BF_WPB;
    const int grid = grid_for(wgs, 1, device_cu_count());
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * NPD_GRU_BF_WPB), lds, s, a);
    (void)g;
    return launch_check("gru_decode_bf_kernel launch");
}

// =============================================================================== split paths, 16-codeword waves
// F = 64, 2 layers (the metric's CRISP GRU), split precisions, N a multiple of 32.  The 32-codeword split kernels
// above need ~500 registers (P, both states, the gate accumulators): one wave per SIMD, and a step is one serial
// chain (layer-0 GEMM -> update -> split -> layer-1 GEMM -> update -> output -> decision) that leaves the MFMA pipe
// idle while the wave does its VALU work.  Here a wave owns 16 codewords on v_mfma_f32_16x16x32_{f16,bf16} (the same
// FLOP per cycle as 32x32x16), so every register array halves and TWO waves share each SIMD, hiding each other's
// LDS and dependency latencies.  (They do not hide each other's VALU work behind MFMAs: measured, an fp16 MFMA wave
// and an FMA wave on one SIMD take the sum of their times, profiles/round3/coissue.txt; PMC: MFMA busy + VALU
// active ~ all SIMD cycles.  Hence the VALU trims below: no fp32 k-step MFMAs, folded gate constants, permlane
// reductions, immediate-offset LDS reads.)
// 16x16x32 maps: lane l = 16 g + c holds D[row 4g + i][codeword c] (i = 0..3), A[row c][k 8g + j], B[k 8g + j][col c].
// Hidden units form 16-row tiles ht = 0..3; K block kb (32 units) is tiles 2kb, 2kb + 1, with MFMA k index 8g + j
// <-> hidden unit 16 (2kb + (j >> 2)) + 4g + (j & 3): an updated state tile converts register for register into the
// next GEMM's B fragment (no lane movement); the host permutes the weight images to match.
// Constants: layer 0's biases and one-hot column 0 enter P once per codeword, the x_i column is one FMA per
// accumulator element, layer 1's biases initialise its accumulators from LDS: no fp32 k-step MFMAs.
// The arithmetic per element (split products, fp32 accumulation, gate nonlinearities) is the 32-codeword kernels'.
struct Geo16 {
    static constexpr int RT = 12, KB = 2, NG = 3;    // 16-row gate tiles, 32-unit K blocks, weight matrices
    static constexpr int IMG4 = NG * RT * KB * 64;   // 16-B fragments per split image
    // fragment (matrix g, row tile t, K block kb, part p = hi / lo) of lane l at f4 index (((g RT + t) KB + kb) 2 + p) 64 + l:
    // a matrix spans 48 KB, so every read of a GEMM is an immediate offset (< 64 KB) from one per-lane base
    static constexpr int G_BYTES = RT * KB * 2 * 1024;
    static constexpr int OFF_C = 2 * IMG4 * 4;       // floats: constants after the weight fragments
    static constexpr int C0L0 = OFF_C, C1L0 = OFF_C + 192, BHN0 = OFF_C + 384, C0L1 = OFF_C + 448,
                         BHN1 = OFF_C + 640, WLIN = OFF_C + 704, TOTAL = OFF_C + 768;
};

__device__ __forceinline__ f4 mfma16s(const hf8& a, const hf8& b, const f4& c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f4 mfma16s(const bf8& a, const bf8& b, const f4& c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// B fragments of a state: fragment kb, element j = tile 2kb + (j >> 2), register j & 3 (hi and, split, lo)
template <int SPLIT>
__device__ __forceinline__ void split16s(const f4 (&h)[4], typename SplitT<SPLIT>::V (&hi)[2],
                                         typename SplitT<SPLIT>::V (&lo)[2]) {
    using S = SplitT<SPLIT>;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float v = h[2 * kb + (j >> 2)][j & 3] * S::kIn;
            const typename S::E b = (typename S::E)v;
            hi[kb][j] = b;
            if (S::kLo) lo[kb][j] = (typename S::E)(v - (float)b);
        }
}

// LDS fragment of the 16-codeword image: wb = this lane's byte base of the matrix (laundered once per kernel)
__device__ __forceinline__ f4 frag16(const f4* __restrict__ smem4, uint32_t wb, int t, int kb, int part) {
    return *reinterpret_cast<const f4*>(reinterpret_cast<const char*>(smem4) + wb +
                                        ((t * Geo16::KB + kb) * 2 + part) * 1024);
}

// (p_row0 + p_row1) + (p_row2 + p_row3) over the four 16-lane rows, the same in every lane (the order of
// __shfl_xor 16 then 32) on v_permlane16_swap / v_permlane32_swap: VALU, no LDS round trip
__device__ __forceinline__ float sum_rows16(float p) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(p), __float_as_uint(p), false, false);
    const float s = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    const auto r2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(s), false, false);
    return __uint_as_float(r2[0]) + __uint_as_float(r2[1]);
}

__device__ __forceinline__ f4 fma4(float x, const f4& c, const f4& p) {
    return f4{fmaf(x, c[0], p[0]), fmaf(x, c[1], p[1]), fmaf(x, c[2], p[2]), fmaf(x, c[3], p[3])};
}

#define NPD_GRU16_WPB 8
// ---- the step is software-pipelined (measured 14.86 -> 14.42 ms per 2^20 words against the plain tile-by-tile
// order, profiles/round3/gru_split_ab.txt; the plain order was removed in round 4).  A wave's own VALU instructions issue in the gaps of its 16-bit
// MFMAs (8 of the 16 cycles of a 16x16x32 are busy for vector issue, MI355X_MICROARCH.md), while another wave's
// do not (profiles/round3/coissue.txt: an fp16 MFMA wave and an FMA wave on one SIMD take the sum of their times).
// So each hidden tile's GEMM carries the update of the PREVIOUS tile (cut into 12 chunks of ~5 instructions:
// element i, stage 0 exp2s / 1 rcps + n-gate input + exp2 / 2 rcp + blend), spread over its MFMA triples between
// sched_barrier fences; the h1 update of tile 3, the output, the decision and the h1 split ride on the NEXT step's
// layer-0 tile-0 GEMM (which needs only h0', not x_i: the x_i column and P are added after it).
template <int SPLIT>
struct Upd4 {
    f4 er, ez, en, z;
    template <int C>
    __device__ __forceinline__ void step(f4& h, const f4& ar, const f4& az, const f4& ain, const f4& ahn) {
        constexpr float c1 = SplitT<SPLIT>::kC1, c2 = SplitT<SPLIT>::kC2;
        constexpr int i = C / 3, st = C % 3;
        if constexpr (st == 0) {
            er[i] = __builtin_amdgcn_exp2f(c1 * ar[i]);
            ez[i] = __builtin_amdgcn_exp2f(c1 * az[i]);
        } else if constexpr (st == 1) {
            const float r = __builtin_amdgcn_rcpf(1.0f + er[i]);
            z[i] = __builtin_amdgcn_rcpf(1.0f + ez[i]);
            en[i] = __builtin_amdgcn_exp2f(c2 * (ain[i] + ahn[i] * r));
        } else {
            const float nn = fmaf(2.0f, __builtin_amdgcn_rcpf(1.0f + en[i]), -1.0f);
            h[i] = (h[i] - nn) * z[i] + nn;
        }
    }
};

template <int SPLIT>
__device__ __forceinline__ void split_kb(const f4 (&h)[4], int kb, typename SplitT<SPLIT>::V (&hi)[2],
                                         typename SplitT<SPLIT>::V (&lo)[2]) {
    using S = SplitT<SPLIT>;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float v = h[2 * kb + (j >> 2)][j & 3] * S::kIn;
        const typename S::E b = (typename S::E)v;
        hi[kb][j] = b;
        if (S::kLo) lo[kb][j] = (typename S::E)(v - (float)b);
    }
}


// A fragments (hi, lo) of one K block of a GEMM's NU row tiles
template <int SPLIT, int NU>
struct Frag16 {
    typename SplitT<SPLIT>::V h[NU], l[NU];
};
template <int SPLIT, int NU>
__device__ __forceinline__ void load_kb16(const f4* __restrict__ smem4, uint32_t wb, const int (&t)[NU], int kb,
                                          Frag16<SPLIT, NU>& f) {
    using V = typename SplitT<SPLIT>::V;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        f.h[u] = __builtin_bit_cast(V, frag16(smem4, wb, t[u], kb, 0));
        if (SplitT<SPLIT>::kLo) f.l[u] = __builtin_bit_cast(V, frag16(smem4, wb, t[u], kb, 1));
    }
}

// acc[u] += W_g[row tile t[u]] . state (both K blocks); work(IC<c>) for chunks C0 .. C0 + NCH - 1 spread evenly
// over the 2 NU MFMA triples, one sched_barrier-fenced region per triple.  The K block 0 fragments arrive in `cur`,
// loaded by the previous GEMM, and this GEMM loads the next one's (matrix base wbn, tiles tn) into it once its own
// K block 0 triples have issued, so no GEMM starts on an LDS round trip (measured 13.08-13.13 against 13.21-13.25 ms
// per 2^20 words with each GEMM loading its own fragments, profiles/round5/gru16_ab.txt).
template <int SPLIT, int NU, int C0, int NCH, typename Work>
__device__ __forceinline__ void gemm16i(const f4* __restrict__ smem4, uint32_t wb, const int (&t)[NU],
                                        f4 (&acc)[NU], const typename SplitT<SPLIT>::V (&bh)[2],
                                        const typename SplitT<SPLIT>::V (&bl)[2], Frag16<SPLIT, NU>& cur,
                                        uint32_t wbn, const int (&tn)[NU], Work&& work) {
    constexpr int NT = 2 * NU;
    Frag16<SPLIT, NU> f[2];  // f[1]: this GEMM's K block 1 (K block 0 is `cur`)
    load_kb16<SPLIT, NU>(smem4, wb, t, 1, f[1]);
    asm volatile("" ::: "memory");  // keeps the (loop-invariant) LDS fragment reads in the step loop
    static_for<0, NT>([&](auto trc) {
        constexpr int tr = decltype(trc)::value;
        constexpr int kb = tr / NU, u = tr % NU;
        const Frag16<SPLIT, NU>& F = kb == 0 ? cur : f[kb];
        acc[u] = mfma16s(F.h[u], bh[kb], acc[u]);
        if (SplitT<SPLIT>::kLo) {
            acc[u] = mfma16s(F.h[u], bl[kb], acc[u]);
            acc[u] = mfma16s(F.l[u], bh[kb], acc[u]);
        }
        if constexpr (tr == NU - 1) {
            asm volatile("" ::: "memory");
            load_kb16<SPLIT, NU>(smem4, wbn, tn, 0, cur);
        }
        static_for<C0 + NCH * tr / NT, C0 + NCH * (tr + 1) / NT>([&](auto cc) { work(cc); });
        __builtin_amdgcn_sched_barrier(0);
    });
}

template <int SPLIT>
__global__ __launch_bounds__(64 * NPD_GRU16_WPB) void gru16p_kernel(const ArgsB a) {
    using G = Geo16;
    using S = SplitT<SPLIT>;
    using V = typename S::V;
    using E = typename S::E;
    extern __shared__ __attribute__((aligned(16))) f4 smem4[];
    {
        const f4* src = reinterpret_cast<const f4*>(a.img);
        for (int i = threadIdx.x; i < G::TOTAL / 4; i += blockDim.x) smem4[i] = src[i];
        __syncthreads();
    }
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int g4 = lane >> 4;
    const int col = lane & 15;
    const int N = a.N;
    const int nkb = N / 32;
    const int64_t tps = (a.B + 15) / 16;  // tiles per segment
    const int64_t ntiles = tps * (a.nseg > 1 ? a.nseg : 1);
    const bool count = a.counters != nullptr;
    uint32_t be_w = 0, bl_w = 0;  // this wave's bit / block errors of the current segment (wave-uniform)
    // per-lane LDS byte bases, laundered so that every fragment / constant read is base + immediate offset
    uint32_t wbs[3];
#pragma unroll
    for (int g = 0; g < 3; ++g) {
        uint32_t v = g * G::G_BYTES + lane * 16;
        asm volatile("" : "+v"(v));
        wbs[g] = v;
    }
    uint32_t cb = (G::OFF_C + 4 * g4) * 4;
    asm volatile("" : "+v"(cb));
    auto c4 = [&](int off, int t) -> f4 {
        return *reinterpret_cast<const f4*>(reinterpret_cast<const char*>(smem4) + cb + (off - G::OFF_C + 16 * t) * 4);
    };
    const f4 zero = {0.f, 0.f, 0.f, 0.f};
    constexpr int T0[3] = {0, 4, 8};
    auto nowork = [](auto) {};

    for (int64_t tile = (int64_t)blockIdx.x * NPD_GRU16_WPB + wave; tile < ntiles;
         tile += (int64_t)gridDim.x * NPD_GRU16_WPB) {
        const int64_t seg = tile / tps;
        const int64_t cw = (tile - seg * tps) * 16 + col;  // codeword within the segment
        const bool valid = cw < a.B;
        const int64_t cwc = valid ? cw : a.B - 1;
        const int64_t rowoff = (seg * a.B + cw) * N;       // this codeword's row of y / decoded / logits
        // count mode: the codeword's messages as 2-bit codes of rint(msg) (-1: 0, +1: 1, 0: 2, else 3; the decision
        // d is in {-1, 0, +1}), slot sl held by row sl & 3 at bits 2 (q & 15) of word q >> 4, q = sl >> 2: 4 registers
        // cover K <= 256, loaded once per tile, so no step waits on a message load
        uint32_t mc[4] = {0u, 0u, 0u, 0u};
        if (count) {
            const float* mr = a.msg + cwc * a.K;
#pragma unroll
            for (int w = 0; w < 4; ++w)
                for (int j = 0; j < 16; ++j) {
                    const int sl = 4 * (16 * w + j) + g4;
                    if (sl >= a.K) break;
                    const float v = rintf(mr[sl]);
                    const uint32_t code = v == -1.0f ? 0u : v == 1.0f ? 1u : v == 0.0f ? 2u : 3u;
                    mc[w] |= code << (2 * j);
                }
        }
        uint32_t nerr = 0;  // this row's share of the codeword's bit errors
        f4 P[G::RT];
#pragma unroll
        for (int t = 0; t < G::RT; ++t) P[t] = c4(G::C0L0, t);
        if (a.y) {
            const float* yr = a.y + (seg * a.B + cwc) * N;
            for (int kb = 0; kb < nkb; ++kb) {
                const f4 y0 = *reinterpret_cast<const f4*>(yr + 32 * kb + 8 * g4);
                const f4 y1 = *reinterpret_cast<const f4*>(yr + 32 * kb + 8 * g4 + 4);
                V yh, yl;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float v = (j < 4 ? y0[j] : y1[j - 4]) * S::kIn;
                    yh[j] = (E)v;
                    if (S::kLo) yl[j] = (E)(v - (float)yh[j]);
                }
#pragma unroll
                for (int t = 0; t < G::RT; ++t) {
                    const V wh = __builtin_bit_cast(V, a.wy[(t * nkb + kb) * 64 + lane]);
                    P[t] = mfma16s(wh, yh, P[t]);
                    if (S::kLo) {
                        const V wl = __builtin_bit_cast(V, a.wy[a.wy_lo + (t * nkb + kb) * 64 + lane]);
                        P[t] = mfma16s(wh, yl, P[t]);
                        P[t] = mfma16s(wl, yh, P[t]);
                    }
                }
            }
        }
        f4 h0[4], h1[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            h0[t] = zero;
            h1[t] = zero;
        }
        if (a.h0) {  // register e of tile t = hidden unit 16 t + 4 g4 + e of codeword col (F = 64, 2 layers)
            const float* hr = a.h0 + (seg * a.B + cwc) * 128;
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int f = 16 * t + 4 * g4 + e;
                    h0[t][e] = hr[2 * f];
                    h1[t][e] = hr[2 * f + 1];
                }
        }
        V fh[2], fl[2], gh[2], gl[2];
        split16s<SPLIT>(h0, fh, fl);
        split16s<SPLIT>(h1, gh, gl);
        float xb = 1.0f;
        // layer 0, hidden tile 0 of step 0: W_hh0 h0 part (the x_i column and P are added at the top of the step)
        f4 a0[3] = {zero, zero, c4(G::BHN0, 0)};
        constexpr int T1[3] = {1, 5, 9};
        Frag16<SPLIT, 3> cur;
        load_kb16<SPLIT, 3>(smem4, wbs[0], T0, 0, cur);
        gemm16i<SPLIT, 3, 0, 0>(smem4, wbs[0], T0, a0, fh, fl, cur, wbs[0], T1, nowork);
        for (int ii = 0; ii < N; ++ii) {
            const int jj = a.rev ? N - 1 - ii : ii;
            Upd4<SPLIT> u;
            // count mode: this step's message slot (255: not compared), from the kernel arguments by a scalar load
            const int sl = count ? (int)((a.slotw[jj >> 2] >> (8 * (jj & 3))) & 255u) : 255;
            // ================= layer 0
            f4 ap[3] = {a0[0] + fma4(xb, c4(G::C1L0, 0), P[0]), a0[1] + fma4(xb, c4(G::C1L0, 4), P[4]), a0[2]};
            f4 ainp = fma4(xb, c4(G::C1L0, 8), P[8]);
            static_for<1, 4>([&](auto htc) {
                constexpr int ht = decltype(htc)::value;
                const int T[3] = {ht, 4 + ht, 8 + ht};
                f4 acc[3] = {fma4(xb, c4(G::C1L0, ht), P[ht]), fma4(xb, c4(G::C1L0, 4 + ht), P[4 + ht]),
                             c4(G::BHN0, ht)};
                constexpr int TN[3] = {ht < 3 ? ht + 1 : 0, ht < 3 ? 5 + ht : 4, ht < 3 ? 9 + ht : 8};
                gemm16i<SPLIT, 3, 0, 12>(smem4, wbs[0], T, acc, fh, fl, cur, wbs[ht < 3 ? 0 : 2], TN, [&](auto cc) {
                    u.template step<decltype(cc)::value>(h0[ht - 1], ap[0], ap[1], ainp, ap[2]);
                });
                ainp = fma4(xb, c4(G::C1L0, 8 + ht), P[8 + ht]);
#pragma unroll
                for (int k = 0; k < 3; ++k) ap[k] = acc[k];
            });
            // ================= layer 1, hidden tile 0: W_hh1 h1 beside h0 tile 3's update and the h0' split
            f4 b[3] = {c4(G::C0L1, 0), c4(G::C0L1, 4), c4(G::BHN1, 0)};
            gemm16i<SPLIT, 3, 0, 14>(smem4, wbs[2], T0, b, gh, gl, cur, wbs[1], T0, [&](auto cc) {
                constexpr int c = decltype(cc)::value;
                if constexpr (c < 12) u.template step<c>(h0[3], ap[0], ap[1], ainp, ap[2]);
                else split_kb<SPLIT>(h0, c - 12, fh, fl);
            });
            f4 bi[3] = {b[0], b[1], c4(G::C0L1, 8)};
            gemm16i<SPLIT, 3, 0, 0>(smem4, wbs[1], T0, bi, fh, fl, cur, wbs[2], T1, nowork);
            f4 q[4] = {bi[0], bi[1], bi[2], b[2]};  // r, z, in, hn of the previous layer-1 tile
            float part = 0.0f;
            static_for<1, 4>([&](auto htc) {
                constexpr int ht = decltype(htc)::value;
                const int T[3] = {ht, 4 + ht, 8 + ht};
                f4 bb[3] = {c4(G::C0L1, ht), c4(G::C0L1, 4 + ht), c4(G::BHN1, ht)};
                auto work = [&](auto cc) {
                    constexpr int c = decltype(cc)::value;
                    if constexpr (c < 12) {
                        u.template step<c>(h1[ht - 1], q[0], q[1], q[2], q[3]);
                    } else {
                        const f4 wl = c4(G::WLIN, ht - 1);
#pragma unroll
                        for (int i = 0; i < 4; ++i) part = fmaf(wl[i], h1[ht - 1][i], part);
                    }
                };
                gemm16i<SPLIT, 3, 0, 7>(smem4, wbs[2], T, bb, gh, gl, cur, wbs[1], T, work);
                f4 bbi[3] = {bb[0], bb[1], c4(G::C0L1, 8 + ht)};
                constexpr int TN[3] = {ht < 3 ? ht + 1 : 0, ht < 3 ? 5 + ht : 4, ht < 3 ? 9 + ht : 8};
                gemm16i<SPLIT, 3, 7, 6>(smem4, wbs[1], T, bbi, fh, fl, cur, wbs[ht < 3 ? 2 : 0], TN, work);
                q[0] = bbi[0];
                q[1] = bbi[1];
                q[2] = bbi[2];
                q[3] = bb[2];
            });
            // ================= tail: next step's layer-0 tile-0 GEMM beside h1 tile 3's update, the output, the
            // decision and the h1 split
            a0[0] = zero;
            a0[1] = zero;
            a0[2] = c4(G::BHN0, 0);
            gemm16i<SPLIT, 3, 0, 15>(smem4, wbs[0], T0, a0, fh, fl, cur, wbs[0], T1, [&](auto cc) {
                constexpr int c = decltype(cc)::value;
                if constexpr (c < 12) {
                    u.template step<c>(h1[3], q[0], q[1], q[2], q[3]);
                } else if constexpr (c == 12) {
                    const f4 wl = c4(G::WLIN, 3);
#pragma unroll
                    for (int i = 0; i < 4; ++i) part = fmaf(wl[i], h1[3][i], part);
                    const float out = sum_rows16(part) + a.b_lin;
                    const bool info = (a.info[jj >> 5] >> (jj & 31)) & 1u;
                    float d;
                    if (info) d = out > 0.0f ? 1.0f : (out < 0.0f ? -1.0f : 0.0f);
                    else d = a.gt ? a.gt[(seg * a.B + cwc) * N + jj] : 1.0f;
                    if (g4 == 0 && valid) {
                        if (a.decoded) a.decoded[rowoff + jj] = d;
                        if (a.logits) a.logits[rowoff + ii] = out;
                    }
                    if (sl != 255) {  // count_errors_kernel's test, rint(msg) != rint(d), on the 2-bit codes
                        const int q = sl >> 2, w = q >> 4;
                        const uint32_t mw = w == 0 ? mc[0] : w == 1 ? mc[1] : w == 2 ? mc[2] : mc[3];
                        const uint32_t dc = d > 0.0f ? 1u : (d < 0.0f ? 0u : 2u);
                        nerr += (g4 == (sl & 3) && ((mw >> (2 * (q & 15))) & 3u) != dc) ? 1u : 0u;
                    }
                    const float sd = d > 0.0f ? 1.0f : (d < 0.0f ? -1.0f : 0.0f);
                    xb = a.onehot ? (sd > 0.0f ? 1.0f : 0.0f) : sd;
                } else {
                    split_kb<SPLIT>(h1, c - 13, gh, gl);
                }
            });
        }
        if (count) {
            // the 16 codewords' errors: each row counted its slots; sum the four rows of every codeword
            nerr += __shfl_xor(nerr, 16, 64);
            nerr += __shfl_xor(nerr, 32, 64);
            const bool mine = g4 == 0 && valid;
            bl_w += (uint32_t)__builtin_popcountll(__ballot(mine && nerr != 0u));
            uint32_t e = mine ? nerr : 0u;
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) e += __shfl_xor(e, o, 64);
            be_w += (uint32_t)__builtin_amdgcn_readfirstlane(e);
            // flush when this wave's next tile is in another segment (or there is none): one atomic pair per
            // wave and segment
            const int64_t nt = tile + (int64_t)gridDim.x * NPD_GRU16_WPB;
            if (nt >= ntiles || nt / tps != seg) {
                if (lane == 0 && (be_w | bl_w)) {
                    atomicAdd(a.counters + 2 * seg, (unsigned long long)be_w);
                    atomicAdd(a.counters + 2 * seg + 1, (unsigned long long)bl_w);
                }
                be_w = bl_w = 0;
            }
        }
    }
}

// image of gru16p_kernel: weight fragments (hi, lo) in the 16x16x32 A-operand order, constants x kc
template <int SPLIT>
static void build_image16(const float* W, int N, int onehot, std::vector<float>& img, std::vector<float>& wy,
                          int64_t& wy_lo) {
    using G = Geo16;
    constexpr int F = 64, L = 2;
    const int Din = N + (onehot ? 2 : 1);
    const float* p = W;
    const float* wih[2];
    const float* whh[2];
    const float* bih[2];
    const float* bhh[2];
    for (int l = 0; l < L; ++l) {
        const int din = l == 0 ? Din : F;
        wih[l] = p; p += (size_t)3 * F * din;
        whh[l] = p; p += (size_t)3 * F * F;
        bih[l] = p; p += 3 * F;
        bhh[l] = p; p += 3 * F;
    }
    const float* wlin = p;
    img.assign(G::TOTAL, 0.0f);
    const float* mats[3] = {whh[0], wih[1], whh[1]};
    // SPLIT 5: every gate row pre-multiplied by its exp2 constant (r, z: -log2 e; n: -2 log2 e; one fp32 rounding)
    auto fold = [&](int row) { return SPLIT == 5 ? (row < 2 * F ? -1.44269504088896340736f : -2.88539008177792681472f) : 1.0f; };
    uint16_t* u16 = reinterpret_cast<uint16_t*>(img.data());
    for (int g = 0; g < G::NG; ++g)
        for (int t = 0; t < G::RT; ++t)
            for (int kb = 0; kb < G::KB; ++kb)
                for (int l = 0; l < 64; ++l)
                    for (int j = 0; j < 8; ++j) {
                        const int row = 16 * t + (l & 15);
                        const int hid = 16 * (2 * kb + (j >> 2)) + 4 * (l >> 4) + (j & 3);
                        uint16_t hi, lo;
                        split16<SPLIT>(fold(row) * mats[g][(size_t)row * F + hid], hi, lo);
                        const size_t e = (((((size_t)(g * G::RT + t) * G::KB + kb) * 2) * 64 + l) * 8 + j);
                        u16[e] = hi;
                        if (SPLIT >= 3) u16[e + 64 * 8] = lo;
                    }
    const float kc = SPLIT == 4 ? 65536.0f : 1.0f;
    auto col = [&](int row, int k) { return wih[0][(size_t)row * Din + k]; };
    for (int row = 0; row < 3 * F; ++row) {
        const bool rz = row < 2 * F;
        // x_i enters as c0 + x_i c1 (one-hot: columns N, N + 1 -> c0 = w_N, c1 = w_{N+1} - w_N; else c1 = w_N)
        const float c0x = onehot ? col(row, N) : 0.0f;
        const float c1x = onehot ? col(row, N + 1) - col(row, N) : col(row, N);
        img[G::C0L0 + row] = fold(row) * (kc * (rz ? bih[0][row] + bhh[0][row] + c0x : bih[0][row] + c0x));
        img[G::C1L0 + row] = fold(row) * (kc * c1x);
        img[G::C0L1 + row] = fold(row) * (kc * (rz ? bih[1][row] + bhh[1][row] : bih[1][row]));
    }
    for (int j = 0; j < F; ++j) {
        img[G::BHN0 + j] = fold(2 * F + j) * (kc * bhh[0][2 * F + j]);
        img[G::BHN1 + j] = fold(2 * F + j) * (kc * bhh[1][2 * F + j]);
        img[G::WLIN + j] = wlin[j];
    }
    const int nkb = N / 32;
    const size_t per = (size_t)G::RT * nkb * 64 * 8;  // 16-bit elements per y-projection image
    wy.assign((per * (SPLIT >= 3 ? 2 : 1) + 1) / 2, 0.0f);
    uint16_t* w16 = reinterpret_cast<uint16_t*>(wy.data());
    for (int t = 0; t < G::RT; ++t)
        for (int kb = 0; kb < nkb; ++kb)
            for (int l = 0; l < 64; ++l)
                for (int j = 0; j < 8; ++j) {
                    const int row = 16 * t + (l & 15);
                    const int k = 32 * kb + 8 * (l >> 4) + j;
                    uint16_t hi, lo;
                    split16<SPLIT>(fold(row) * col(row, k), hi, lo);
                    const size_t e = (((size_t)t * nkb + kb) * 64 + l) * 8 + j;
                    w16[e] = hi;
                    if (SPLIT >= 3) w16[per + e] = lo;
                }
    wy_lo = (int64_t)(per / 8);
}

template <int SPLIT>
static int launch16(const ArgsB& a, hipStream_t s) {
    auto kern = gru16p_kernel<SPLIT>;
    static bool attr = false;
    if (!attr) {
        NPD_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
        attr = true;
    }
    const int64_t tiles = (a.B + 15) / 16 * (a.nseg > 1 ? a.nseg : 1);
    const int64_t wgs = (tiles + NPD_GRU16_WPB - 1) / NPD_GRU16_WPB;
    const int grid = grid_for(wgs, 1, device_cu_count());
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * NPD_GRU16_WPB), (size_t)Geo16::TOTAL * 4, s, a);
    return launch_check("gru16p_kernel launch");
}

// =============================================================================== wide hidden sizes
// F = 128 / 256 / 512 (the CRISP curriculum trains F = 512, 2 layers: run_crisp.sh).  The weights
// (3 x 3F x F fp32 = 9.4 MB at F = 512) no longer fit in LDS, so the per-step matvecs of a 32-codeword
// tile become weight-streaming GEMMs: one workgroup of NW = min(8, F/32) waves owns 32 codewords, each
// wave owns HPW = F/32/NW hidden tiles (its r, z, n gate rows), the A operands stream from L2 / MALL in
// the same permuted image as the narrow kernel (prefetched one 4-k-step group ahead), and the hidden
// states of both layers live in LDS in B-operand order (k-step s, lane half, codeword): a wave writes
// its updated tiles with 16-B stores and every wave reads the whole state with ds_read_b128.  The y
// projection W_ih0[:, :N] y is recomputed every step from an LDS copy of the tile's received words
// (+ N/2 k-steps per 3F x F matvec: < 5 % of the step's MFMAs) instead of holding 3F x 32 values in
// registers.  Barriers separate each layer's GEMM (reads the old state) from its update (overwrites
// it); the output Linear(F, 1) is reduced across waves through LDS in a fixed order.
template <int F>
struct WideGeo {
    static constexpr int HT = F / 32;
    static constexpr int NW = HT < 8 ? HT : 8;
    static constexpr int HPW = HT / NW;
};

int wide_lds_bytes(int N, int F, int L) {
    const int nw = (F / 32) < 8 ? F / 32 : 8;
    return (L * F * 32 + N * 32 + nw * 32) * 4;
}

// acc[D0|D1|D2][j] += W[tiles k*HT + jt0 + j, k = 0, 1, 2] . B over kg groups of 4 k-steps.
// W: f4 image of one matrix ([tile][group][lane]), B: LDS state in B-operand order ([group][lane]).
template <int HPW, int D0, int D1, int D2>
__device__ __forceinline__ void wide_chain(const f4* __restrict__ W, int kg, int HT, int jt0,
                                           const f4* __restrict__ Bs, int lane, f16v (&acc)[4][HPW]) {
    constexpr int D[3] = {D0, D1, D2};
    f4 wc[3][HPW];
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int j = 0; j < HPW; ++j) wc[k][j] = W[((size_t)(k * HT + jt0 + j) * kg + 0) * 64 + lane];
    for (int q = 0; q < kg; ++q) {
        f4 wn[3][HPW];
        if (q + 1 < kg) {
#pragma unroll
            for (int k = 0; k < 3; ++k)
#pragma unroll
                for (int j = 0; j < HPW; ++j) wn[k][j] = W[((size_t)(k * HT + jt0 + j) * kg + q + 1) * 64 + lane];
        }
        const f4 b = Bs[q * 64 + lane];
        asm volatile("" ::: "memory");
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int k = 0; k < 3; ++k)
#pragma unroll
                for (int j = 0; j < HPW; ++j) acc[D[k]][j] = mfma(wc[k][j][e], b[e], acc[D[k]][j]);
        if (q + 1 < kg) {
#pragma unroll
            for (int k = 0; k < 3; ++k)
#pragma unroll
                for (int j = 0; j < HPW; ++j) wc[k][j] = wn[k][j];
        }
    }
}

// one hidden tile's GRU update against its old value in the LDS state (B-operand order)
template <int HPW>
__device__ __forceinline__ void wide_update(f4* __restrict__ Hs, int jt, int lane, f16v& hv, const f16v& ar,
                                            const f16v& az, const f16v& ain, const f16v& ahn) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const f4 v = Hs[(4 * jt + q) * 64 + lane];
#pragma unroll
        for (int e = 0; e < 4; ++e) hv[4 * q + e] = v[e];
    }
    gru_update(hv, ar, az, ain, ahn);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        f4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = hv[4 * q + e];
        Hs[(4 * jt + q) * 64 + lane] = v;
    }
}

template <int F, int L>
__global__ __launch_bounds__(64 * WideGeo<F>::NW) void gru_wide_kernel(const Args a) {
    using G = Geo<F, L>;
    using WG = WideGeo<F>;
    constexpr int TT = G::TT, HT = G::HT, KG = G::KG, NW = WG::NW, HPW = WG::HPW;
    extern __shared__ __attribute__((aligned(16))) f4 lds4[];
    const int N = a.N;
    f4* const Hs0 = lds4;
    f4* const Hs1 = lds4 + (L == 2 ? F * 8 : 0);
    f4* const Ys = lds4 + L * F * 8;
    float* const part = reinterpret_cast<float*>(Ys + N * 8);
    const float* img = a.img;
    const f4* W0 = reinterpret_cast<const f4*>(img);
    const f4* W1 = reinterpret_cast<const f4*>(img + (size_t)G::G_SIZE);
    const f4* W2 = reinterpret_cast<const f4*>(img + 2 * (size_t)G::G_SIZE);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int half = lane >> 5;
    const int col = lane & 31;
    const int jt0 = wave * HPW;
    const int ng = N / 8;
    const int64_t ntiles = (a.B + 31) / 32;
    const f16v zero = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const float one_or_zero = half ? 0.0f : 1.0f;
    constexpr int R = 0, Z = 1, IN = 2, HN = 3;

    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t cw = tile * 32 + col;
        const bool valid = cw < a.B;
        const int64_t cwc = valid ? cw : a.B - 1;
        __syncthreads();  // the previous tile's last readers are done
        {
            if (a.y) {
                const f4* yr = reinterpret_cast<const f4*>(a.y + cwc * N + half * (N / 2));
                for (int q = wave; q < ng; q += NW) Ys[q * 64 + lane] = yr[q];
            }
            // states: f4 (4 jt + q) * 64 + lane of layer l holds units hid_of(16 jt + 4 q + e, lane >> 5), e < 4, of
            // codeword tile * 32 + (lane & 31): zero, or the initial state a.h0 (B, F L)
            for (int i = threadIdx.x; i < L * F * 8; i += NW * 64) {
                f4 v = f4{0.f, 0.f, 0.f, 0.f};
                if (a.h0) {
                    const int l = i / (F * 8), idx = i - l * F * 8;
                    const int ln = idx & 63, jq = idx >> 6;
                    int64_t c = tile * 32 + (ln & 31);
                    if (c >= a.B) c = a.B - 1;
                    const float* hr = a.h0 + c * (int64_t)(F * L) + l;
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = hr[hid_of(16 * (jq >> 2) + 4 * (jq & 3) + e, ln >> 5) * L];
                }
                lds4[i] = v;
            }
        }
        __syncthreads();
        float xb = 1.0f;
        for (int ii = 0; ii < N; ++ii) {
            const int jj = a.rev ? N - 1 - ii : ii;
            const float xbe = half ? xb : 1.0f;
            f16v acc[4][HPW];
            f16v top[HPW];
            // ================= layer 0: P = W_ih0[:, :N] y (r, z, in), then W_hh0 h0 (r, z, hn), then consts
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int j = 0; j < HPW; ++j) acc[k][j] = zero;
            if (a.y) wide_chain<HPW, R, Z, IN>(a.wy, ng, HT, jt0, Ys, lane, acc);
            wide_chain<HPW, R, Z, HN>(W0, KG, HT, jt0, Hs0, lane, acc);
#pragma unroll
            for (int j = 0; j < HPW; ++j) {
                const int jt = jt0 + j;
                acc[R][j] = mfma(img[G::OFF_X + (0 * TT + jt) * 64 + lane], xbe, acc[R][j]);
                acc[Z][j] = mfma(img[G::OFF_X + (0 * TT + HT + jt) * 64 + lane], xbe, acc[Z][j]);
                acc[HN][j] = mfma(img[G::OFF_X + (0 * TT + 2 * HT + jt) * 64 + lane], xbe, acc[HN][j]);
                acc[IN][j] = mfma(img[G::OFF_IN + jt * 64 + lane], xbe, acc[IN][j]);
            }
            __syncthreads();  // every wave has read h0
#pragma unroll
            for (int j = 0; j < HPW; ++j) wide_update<HPW>(Hs0, jt0 + j, lane, top[j], acc[R][j], acc[Z][j], acc[IN][j], acc[HN][j]);
            __syncthreads();  // h0' complete
            if constexpr (L == 2) {
                // ================= layer 1: W_ih1 h0' (r, z, in) + consts, W_hh1 h1 (r, z, hn) + b_hn
#pragma unroll
                for (int k = 0; k < 4; ++k)
#pragma unroll
                    for (int j = 0; j < HPW; ++j) acc[k][j] = zero;
                wide_chain<HPW, R, Z, IN>(W1, KG, HT, jt0, Hs0, lane, acc);
#pragma unroll
                for (int j = 0; j < HPW; ++j) {
                    const int jt = jt0 + j;
                    acc[R][j] = mfma(img[G::OFF_X + (TT + jt) * 64 + lane], one_or_zero, acc[R][j]);
                    acc[Z][j] = mfma(img[G::OFF_X + (TT + HT + jt) * 64 + lane], one_or_zero, acc[Z][j]);
                    acc[IN][j] = mfma(img[G::OFF_X + (TT + 2 * HT + jt) * 64 + lane], one_or_zero, acc[IN][j]);
                }
                wide_chain<HPW, R, Z, HN>(W2, KG, HT, jt0, Hs1, lane, acc);
#pragma unroll
                for (int j = 0; j < HPW; ++j)
                    acc[HN][j] = mfma(img[G::OFF_X + (2 * TT + 2 * HT + jt0 + j) * 64 + lane], one_or_zero, acc[HN][j]);
                __syncthreads();  // every wave has read h1
#pragma unroll
                for (int j = 0; j < HPW; ++j)
                    wide_update<HPW>(Hs1, jt0 + j, lane, top[j], acc[R][j], acc[Z][j], acc[IN][j], acc[HN][j]);
            }
            // ================= output: Linear(F, 1) on the top layer, reduced over the waves in a fixed order
            float p = 0.0f;
#pragma unroll
            for (int j = 0; j < HPW; ++j)
#pragma unroll
                for (int i = 0; i < 16; ++i) p += img[G::OFF_WL + (half * HT + jt0 + j) * 16 + i] * top[j][i];
            p += __shfl_xor(p, 32, 64);
            if (half == 0) part[wave * 32 + col] = p;
            __syncthreads();
            float out = 0.0f;
#pragma unroll
            for (int w = 0; w < NW; ++w) out += part[w * 32 + col];
            out += a.b_lin;
            const bool info = (a.info[jj >> 5] >> (jj & 31)) & 1u;
            float d;
            if (info) d = out > 0.0f ? 1.0f : (out < 0.0f ? -1.0f : 0.0f);
            else d = a.gt ? a.gt[cwc * N + jj] : 1.0f;
            if (wave == 0 && half == 0 && valid) {
                a.decoded[cw * N + jj] = d;
                if (a.logits) a.logits[cw * N + ii] = out;
            }
            const float sd = d > 0.0f ? 1.0f : (d < 0.0f ? -1.0f : 0.0f);
            xb = a.onehot ? (sd > 0.0f ? 1.0f : 0.0f) : sd;
        }
    }
}

// ------------------------------------------------------------------ LSTM cells beyond the LDS (F = 64 x 2, F >= 128)
// gru_wide_kernel's scheme with LSTM cells: the build_image_lstm weight images (gate rows pre-scaled by their exp2
// constants, biases as accumulator initialisation) stay in HBM / L2, the hidden states of the 32-codeword tile sit in
// LDS in B-operand order, each wave owns HPW hidden tiles and computes all four gates (i, f, g, o) of them, and keeps
// their cell states c in registers (accumulator layout = the tile's hidden units of the lane's codeword).
template <int HPW>
__device__ __forceinline__ void wide_chain4(const f4* __restrict__ W, int kg, int HT, int jt0, const f4* __restrict__ Bs,
                                            int lane, f16v (&acc)[4][HPW]) {
    f4 wc[4][HPW];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int j = 0; j < HPW; ++j) wc[k][j] = W[((size_t)(k * HT + jt0 + j) * kg + 0) * 64 + lane];
    for (int q = 0; q < kg; ++q) {
        f4 wn[4][HPW];
        if (q + 1 < kg) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int j = 0; j < HPW; ++j) wn[k][j] = W[((size_t)(k * HT + jt0 + j) * kg + q + 1) * 64 + lane];
        }
        const f4 b = Bs[q * 64 + lane];
        asm volatile("" ::: "memory");
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int j = 0; j < HPW; ++j) acc[k][j] = mfma(wc[k][j][e], b[e], acc[k][j]);
        if (q + 1 < kg) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int j = 0; j < HPW; ++j) wc[k][j] = wn[k][j];
        }
    }
}

template <int F, int L>
__global__ __launch_bounds__(64 * WideGeo<F>::NW) void lstm_wide_kernel(const Args a) {
    using G = LGeo<F, L>;
    using WG = WideGeo<F>;
    constexpr int TT = G::TT, HT = G::HT, KG = G::KG, NW = WG::NW, HPW = WG::HPW;
    extern __shared__ __attribute__((aligned(16))) f4 lds4[];
    const int N = a.N;
    f4* const Hs0 = lds4;
    f4* const Hs1 = lds4 + (L == 2 ? F * 8 : 0);
    f4* const Ys = lds4 + L * F * 8;
    float* const part = reinterpret_cast<float*>(Ys + N * 8);
    const float* img = a.img;
    const f4* W0 = reinterpret_cast<const f4*>(img);
    const f4* W1 = reinterpret_cast<const f4*>(img + (size_t)G::G_SIZE);
    const f4* W2 = reinterpret_cast<const f4*>(img + 2 * (size_t)G::G_SIZE);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int half = lane >> 5;
    const int col = lane & 31;
    const int jt0 = wave * HPW;
    const int ng = N / 8;
    const int64_t ntiles = (a.B + 31) / 32;
    auto cvec = [&](int off) -> f16v {
        const f4* p = reinterpret_cast<const f4*>(img + off + half * 16);
        const f4 x0 = p[0], x1 = p[1], x2 = p[2], x3 = p[3];
        return f16v{x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3],
                    x2[0], x2[1], x2[2], x2[3], x3[0], x3[1], x3[2], x3[3]};
    };
    constexpr float kT = -2.88539008177792681472f;  // tanh(c) = 2 sig2(kT c) - 1
    // c' = sig(f) c + sig(i) tanh(g), h' = sig(o) tanh(c') on hidden tile jt; h' to the LDS state (B-operand order)
    auto cell = [&](f4* Hs, int jt, f16v& c, f16v& h, const f16v& ai, const f16v& af, const f16v& ag, const f16v& ao) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const float ig = sig2(ai[i]), fg = sig2(af[i]);
            const float gg = fmaf(2.0f, sig2(ag[i]), -1.0f);
            const float og = sig2(ao[i]);
            c[i] = fmaf(fg, c[i], ig * gg);
            h[i] = og * fmaf(2.0f, sig2(kT * c[i]), -1.0f);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) Hs[(4 * jt + q) * 64 + lane] = f4{h[4 * q], h[4 * q + 1], h[4 * q + 2], h[4 * q + 3]};
    };
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t cw = tile * 32 + col;
        const bool valid = cw < a.B;
        const int64_t cwc = valid ? cw : a.B - 1;
        __syncthreads();  // the previous tile's last readers are done
        if (a.y) {
            const f4* yr = reinterpret_cast<const f4*>(a.y + cwc * N + half * (N / 2));
            for (int q = wave; q < ng; q += NW) Ys[q * 64 + lane] = yr[q];
        }
        // h states in LDS and this wave's c states in registers: zero, or (y_h0) both from a.h0 (B, F L), element
        // f L + l (get_h0 returns (x, x) for LSTM cells, rnn_all.py:370-375)
        for (int i = threadIdx.x; i < L * F * 8; i += NW * 64) {
            f4 v = f4{0.f, 0.f, 0.f, 0.f};
            if (a.h0) {
                const int l = i / (F * 8), idx = i - l * F * 8;
                const int ln = idx & 63, jq = idx >> 6;
                int64_t c = tile * 32 + (ln & 31);
                if (c >= a.B) c = a.B - 1;
                const float* hr = a.h0 + c * (int64_t)(F * L) + l;
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = hr[hid_of(16 * (jq >> 2) + 4 * (jq & 3) + e, ln >> 5) * L];
            }
            lds4[i] = v;
        }
        f16v c0[HPW], c1[HPW], top[HPW];
#pragma unroll
        for (int j = 0; j < HPW; ++j)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                float v0 = 0.0f, v1 = 0.0f;
                if (a.h0) {
                    const float* hr = a.h0 + cwc * (int64_t)(F * L) + hid_of(16 * (jt0 + j) + i, half) * L;
                    v0 = hr[0];
                    if constexpr (L == 2) v1 = hr[1];
                }
                c0[j][i] = v0;
                c1[j][i] = v1;
            }
        __syncthreads();
        float xb = 1.0f;
        for (int ii = 0; ii < N; ++ii) {
            const int jj = a.rev ? N - 1 - ii : ii;
            const float xbe = half ? xb : 1.0f;
            f16v acc[4][HPW];
            // ================= layer 0: biases, W_ih0[:, :N] y, W_hh0 h0, the [1, x_i] k-step
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int j = 0; j < HPW; ++j) acc[k][j] = cvec(G::OFF_CV + (k * HT + jt0 + j) * 32);
            if (a.y) wide_chain4<HPW>(a.wy, ng, HT, jt0, Ys, lane, acc);
            wide_chain4<HPW>(W0, KG, HT, jt0, Hs0, lane, acc);
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int j = 0; j < HPW; ++j) acc[k][j] = mfma(img[G::OFF_X + (k * HT + jt0 + j) * 64 + lane], xbe, acc[k][j]);
            __syncthreads();  // every wave has read h0
#pragma unroll
            for (int j = 0; j < HPW; ++j) cell(Hs0, jt0 + j, c0[j], top[j], acc[0][j], acc[1][j], acc[2][j], acc[3][j]);
            __syncthreads();  // h0' complete
            if constexpr (L == 2) {
                // ================= layer 1: biases, W_ih1 h0', W_hh1 h1
#pragma unroll
                for (int k = 0; k < 4; ++k)
#pragma unroll
                    for (int j = 0; j < HPW; ++j) acc[k][j] = cvec(G::OFF_CV + (TT + k * HT + jt0 + j) * 32);
                wide_chain4<HPW>(W1, KG, HT, jt0, Hs0, lane, acc);
                wide_chain4<HPW>(W2, KG, HT, jt0, Hs1, lane, acc);
                __syncthreads();  // every wave has read h1
#pragma unroll
                for (int j = 0; j < HPW; ++j)
                    cell(Hs1, jt0 + j, c1[j], top[j], acc[0][j], acc[1][j], acc[2][j], acc[3][j]);
            }
            // ================= output: Linear(F, 1) on the top layer, reduced over the waves in a fixed order
            float p = 0.0f;
#pragma unroll
            for (int j = 0; j < HPW; ++j)
#pragma unroll
                for (int i = 0; i < 16; ++i) p += img[G::OFF_WL + (half * HT + jt0 + j) * 16 + i] * top[j][i];
            p += __shfl_xor(p, 32, 64);
            if (half == 0) part[wave * 32 + col] = p;
            __syncthreads();
            float out = 0.0f;
#pragma unroll
            for (int w = 0; w < NW; ++w) out += part[w * 32 + col];
            out += a.b_lin;
            const bool info = (a.info[jj >> 5] >> (jj & 31)) & 1u;
            float d;
            if (info) d = out > 0.0f ? 1.0f : (out < 0.0f ? -1.0f : 0.0f);
            else d = a.gt ? a.gt[cwc * N + jj] : 1.0f;
            if (wave == 0 && half == 0 && valid) {
                a.decoded[cw * N + jj] = d;
                if (a.logits) a.logits[cw * N + ii] = out;
            }
            const float sd = d > 0.0f ? 1.0f : (d < 0.0f ? -1.0f : 0.0f);
            xb = a.onehot ? (sd > 0.0f ? 1.0f : 0.0f) : sd;
        }
    }
}

template <int F, int L>
static int launch_lstm_wide(const Args& a, int N, hipStream_t s) {
    using WG = WideGeo<F>;
    auto kern = lstm_wide_kernel<F, L>;
    const size_t lds = (size_t)wide_lds_bytes(N, F, L);
    static bool attr = false;
    if (!attr) {
        NPD_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
        attr = true;
    }
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, 64 * WG::NW, lds) != hipSuccess || occ <= 0) {
        (void)hipGetLastError();
        occ = 1;
    }
    const int64_t tiles = (a.B + 31) / 32;
    const int grid = grid_for(tiles, occ, device_cu_count());
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * WG::NW), lds, s, a);
    return launch_check("lstm_wide_kernel launch");
}

template <int F, int L>
static int launch_wide(const Args& a, int N, hipStream_t s) {
    using WG = WideGeo<F>;
    auto kern = gru_wide_kernel<F, L>;
    const size_t lds = (size_t)wide_lds_bytes(N, F, L);
    static bool attr = false;
    if (!attr) {
        NPD_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
        attr = true;
    }
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, 64 * WG::NW, lds) != hipSuccess || occ <= 0) {
        (void)hipGetLastError();
        occ = 1;
    }
    const int64_t tiles = (a.B + 31) / 32;
    const int grid = grid_for(tiles, occ, device_cu_count());
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * WG::NW), lds, s, a);
    return launch_check("gru_wide_kernel launch");
}

}  // namespace gru
}  // namespace npd

using namespace npd;

static int create_lstm(int N, int F, int layers, int onehot, const float* weights, int64_t n_weights, int precision,
                       npd_gru** out) {
    NPD_ARG(F == 32 || F == 64 || F == 128 || F == 256 || F == 512,
            "npd_rnn_create: LSTM hidden size F must be 32, 64, 128, 256 or 512");
    NPD_ARG(F <= 64 || gru::wide_lds_bytes(N, F, layers) <= 160 * 1024,
            "npd_rnn_create: an LSTM with F = 512 and 2 layers needs N <= 128 (LDS holds both states and the tile's y)");
    NPD_ARG(precision == 0, "npd_rnn_create: LSTM cells run fp32 (precision 0)");
    const int Din = N + (onehot ? 2 : 1);
    int64_t expect = (int64_t)4 * F * Din + (int64_t)4 * F * F + 8 * F;
    if (layers == 2) expect += (int64_t)8 * F * F + 8 * F;
    expect += F + 1;
    NPD_ARG(n_weights == expect, "npd_rnn_create: weight count does not match (LSTM, N, F, layers, onehot)");
    std::vector<float> img, wy;
    float b_lin = 0.0f;
    // F = 32 (1-2 layers) and F = 64 x 1: LDS-resident weights (lstm_decode_kernel); else lstm_wide_kernel
#define NPD_LSTM_IMG(FF, LL) gru::build_image_lstm<FF, LL>(weights, N, onehot, img, wy, b_lin)
    if (F == 512) { if (layers == 2) NPD_LSTM_IMG(512, 2); else NPD_LSTM_IMG(512, 1); }
    else if (F == 256) { if (layers == 2) NPD_LSTM_IMG(256, 2); else NPD_LSTM_IMG(256, 1); }
    else if (F == 128) { if (layers == 2) NPD_LSTM_IMG(128, 2); else NPD_LSTM_IMG(128, 1); }
    else if (F == 64) { if (layers == 2) NPD_LSTM_IMG(64, 2); else NPD_LSTM_IMG(64, 1); }
    else if (layers == 2) NPD_LSTM_IMG(32, 2);
    else NPD_LSTM_IMG(32, 1);
#undef NPD_LSTM_IMG
    npd_gru* g = new (std::nothrow) npd_gru;
    if (!g) return fail(NPD_ENOMEM, "npd_rnn_create: out of memory");
    memset(g, 0, sizeof(*g));
    g->N = N; g->F = F; g->layers = layers; g->onehot = onehot; g->precision = 0; g->b_lin = b_lin; g->cell = 1;
    g->img_floats = (int64_t)img.size();
    hipError_t e = hipGetDevice(&g->device);
    if (e == hipSuccess) e = hipMalloc(&g->img, img.size() * 4);
    if (e == hipSuccess) e = hipMalloc(&g->wy, wy.size() * 4);
    if (e == hipSuccess) e = hipMemcpy(g->img, img.data(), img.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(g->wy, wy.data(), wy.size() * 4, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        if (g->img) (void)hipFree(g->img);
        if (g->wy) (void)hipFree(g->wy);
        delete g;
        return hip_fail(e, "npd_rnn_create");
    }
    *out = g;
    return NPD_OK;
}

extern "C" int npd_rnn_create(int cell, int N, int F, int layers, int onehot, const float* weights, int64_t n_weights,
                              int precision, npd_gru** out) {
    NPD_ARG(out != nullptr, "npd_rnn_create: out is NULL");
    *out = nullptr;
    NPD_ARG(cell == 0 || cell == 1, "npd_rnn_create: cell must be 0 (GRU) or 1 (LSTM)");
    if (cell == 0) return npd_gru_create(N, F, layers, onehot, weights, n_weights, precision, out);
    NPD_ARG(weights != nullptr, "npd_rnn_create: weights is NULL");
    NPD_ARG(N >= 8 && N <= kMaxN && N % 8 == 0, "npd_rnn_create: N must be a multiple of 8 in [8, 256]");
    NPD_ARG(layers == 1 || layers == 2, "npd_rnn_create: 1 or 2 layers supported");
    return create_lstm(N, F, layers, onehot, weights, n_weights, precision, out);
}

static int attach_head(npd_gru* g, int F, int head_depth, int head_hidden, const float* head_weights, int64_t n_head) {
    const int H = head_hidden;
    int64_t expect = (int64_t)H * F + H + (int64_t)(head_depth - 2) * (H * H + H) + H + 1;
    NPD_ARG(n_head == expect, "npd_rnn_create_ex: head weight count does not match (F, head_depth, head_hidden)");
    const int hdt = H <= 32 ? 1 : H <= 64 ? 2 : 4;
    std::vector<float> img;
    float bout = 0.0f;
    gru::build_head_image(head_weights, F, H, head_depth, hdt, img, bout);
    hipError_t e = hipMalloc(&g->hd, img.size() * 4);
    if (e == hipSuccess) e = hipMemcpy(g->hd, img.data(), img.size() * 4, hipMemcpyHostToDevice);
    if (e != hipSuccess) return hip_fail(e, "npd_rnn_create_ex (head)");
    g->hd_depth = head_depth;
    g->hd_tiles = hdt;
    g->hd_bout = bout;
    return NPD_OK;
}

extern "C" int npd_rnn_create_ex(int cell, int N, int F, int layers, int onehot, const float* weights,
                                 int64_t n_weights, int precision, const float* ln_weight, const float* ln_bias,
                                 float ln_eps, int head_depth, int head_hidden, const float* head_weights,
                                 int64_t n_head, npd_gru** out) {
    NPD_ARG(out != nullptr, "npd_rnn_create_ex: out is NULL");
    *out = nullptr;
    NPD_ARG(head_depth == 1 || (head_depth >= 2 && head_depth <= 8), "npd_rnn_create_ex: head_depth must be 1 .. 8");
    if (head_depth > 1) {
        NPD_ARG(head_weights != nullptr && weights != nullptr, "npd_rnn_create_ex: null pointer");
        NPD_ARG(ln_weight == nullptr, "npd_rnn_create_ex: a LayerNorm before an out_linear_depth > 1 head is not fused");
        NPD_ARG(cell == 0 && precision == 0 && (F == 32 || F == 64) && head_hidden >= 1 && head_hidden <= 128,
                "npd_rnn_create_ex: the out_linear_depth > 1 head runs on the fp32 GRU kernel (cell 0, precision 0, "
                "F 32 or 64, head_hidden 1 .. 128)");
        int rc = npd_gru_create(N, F, layers, onehot, weights, n_weights, 0, out);
        if (rc != NPD_OK) return rc;
        rc = attach_head(*out, F, head_depth, head_hidden, head_weights, n_head);
        if (rc != NPD_OK) {
            npd_gru_destroy(*out);
            *out = nullptr;
        }
        return rc;
    }
    if (ln_weight == nullptr) return npd_rnn_create(cell, N, F, layers, onehot, weights, n_weights, precision, out);
    NPD_ARG(weights != nullptr && ln_bias != nullptr, "npd_rnn_create_ex: null pointer");
    NPD_ARG(cell == 0 && precision == 0 && (F == 32 || F == 64),
            "npd_rnn_create_ex: the LayerNorm head runs on the fp32 GRU kernel (cell 0, precision 0, F 32 or 64)");
    NPD_ARG(n_weights > F, "npd_rnn_create_ex: weight count too small");
    // fold the LayerNorm's affine part into the output Linear: w' = w gamma, b' = b + sum w beta (in order, fp32)
    std::vector<float> w(weights, weights + n_weights);
    float* wl = w.data() + n_weights - F - 1;
    float bsum = w[n_weights - 1];
    for (int i = 0; i < F; ++i) {
        bsum += wl[i] * ln_bias[i];
        wl[i] *= ln_weight[i];
    }
    w[n_weights - 1] = bsum;
    const int rc = npd_gru_create(N, F, layers, onehot, w.data(), n_weights, 0, out);
    if (rc != NPD_OK) return rc;
    (*out)->ln = 1;
    (*out)->ln_eps = ln_eps;
    return NPD_OK;
}

extern "C" int npd_gru_create(int N, int F, int layers, int onehot, const float* weights, int64_t n_weights,
                              int precision, npd_gru** out) {
    NPD_ARG(out != nullptr, "npd_gru_create: out is NULL");
    *out = nullptr;
    NPD_ARG(weights != nullptr, "npd_gru_create: weights is NULL");
    NPD_ARG(N >= 8 && N <= kMaxN && N % 8 == 0, "npd_gru_create: N must be a multiple of 8 in [8, 256]");
    NPD_ARG(F == 32 || F == 64 || F == 128 || F == 256 || F == 512,
            "npd_gru_create: hidden size F must be 32, 64, 128, 256 or 512");
    NPD_ARG(F <= 64 || precision == 0, "npd_gru_create: the bf16 kernels cover F <= 64; F > 64 runs fp32");
    NPD_ARG(F <= 64 || gru::wide_lds_bytes(N, F, layers) <= 160 * 1024,
            "npd_gru_create: F = 512 with 2 layers needs N <= 128 (LDS holds both states and the tile's y)");
    NPD_ARG(layers == 1 || layers == 2, "npd_gru_create: 1 or 2 GRU layers supported");
    NPD_ARG(precision >= 0 && precision <= 3,
            "npd_gru_create: precision must be 0 (fp32), 1 (bf16x3), 2 (bf16) or 3 (fp16x3)");
    NPD_ARG(precision == 0 || N % 16 == 0, "npd_gru_create: bf16 paths need N % 16 == 0");
    const int Din = N + (onehot ? 2 : 1);
    int64_t expect = (int64_t)3 * F * Din + (int64_t)3 * F * F + 6 * F;
    if (layers == 2) expect += (int64_t)6 * F * F + 6 * F;
    expect += F + 1;
    NPD_ARG(n_weights == expect, "npd_gru_create: weight count does not match (N, F, layers, onehot)");
    std::vector<float> img, wy;
    float b_lin = 0.0f;
    int64_t wy_lo = 0;
#define NPD_BUILD(FF, LL)                                                                              \
    do {                                                                                               \
        if (precision == 0) gru::build_image<FF, LL>(weights, N, onehot, img, wy, b_lin, true);           \
        else if (precision == 1) gru::build_image_bf<FF, LL, 3>(weights, N, onehot, img, wy, b_lin, wy_lo); \
        else if (precision == 3) gru::build_image_bf<FF, LL, 4>(weights, N, onehot, img, wy, b_lin, wy_lo); \
        else gru::build_image_bf<FF, LL, 1>(weights, N, onehot, img, wy, b_lin, wy_lo);               \
    } while (0)
    if (F == 512 && layers == 2) gru::build_image<512, 2>(weights, N, onehot, img, wy, b_lin);
    else if (F == 512) gru::build_image<512, 1>(weights, N, onehot, img, wy, b_lin);
    else if (F == 256 && layers == 2) gru::build_image<256, 2>(weights, N, onehot, img, wy, b_lin);
    else if (F == 256) gru::build_image<256, 1>(weights, N, onehot, img, wy, b_lin);
    else if (F == 128 && layers == 2) gru::build_image<128, 2>(weights, N, onehot, img, wy, b_lin);
    else if (F == 128) gru::build_image<128, 1>(weights, N, onehot, img, wy, b_lin);
    else if (F == 64 && layers == 2) NPD_BUILD(64, 2);
    else if (F == 64) NPD_BUILD(64, 1);
    else if (layers == 2) NPD_BUILD(32, 2);
    else NPD_BUILD(32, 1);
#undef NPD_BUILD
    npd_gru* g = new (std::nothrow) npd_gru;
    if (!g) return fail(NPD_ENOMEM, "npd_gru_create: out of memory");
    memset(g, 0, sizeof(*g));
    g->N = N; g->F = F; g->layers = layers; g->onehot = onehot; g->precision = precision; g->b_lin = b_lin;
    g->img_floats = (int64_t)img.size();
    g->wy_lo = wy_lo;
    std::vector<float> img16, wy16;
    if (precision != 0 && F == 64 && layers == 2 && N % 32 == 0) {
        // fp16x3 here is the unscaled split with the gate constants folded into the weights (SPLIT 5); the
        // 32-codeword kernels (other shapes) run the x 2^8-scaled split (SPLIT 4)
        g->split16 = precision == 1 ? 3 : precision == 3 ? 5 : 1;
        if (precision == 1) gru::build_image16<3>(weights, N, onehot, img16, wy16, g->wy16_lo);
        else if (precision == 3) gru::build_image16<5>(weights, N, onehot, img16, wy16, g->wy16_lo);
        else gru::build_image16<1>(weights, N, onehot, img16, wy16, g->wy16_lo);
    }
    hipError_t e = hipGetDevice(&g->device);
    if (e == hipSuccess) e = hipMalloc(&g->img, img.size() * 4);
    if (e == hipSuccess) e = hipMalloc(&g->wy, wy.size() * 4);
    if (e == hipSuccess) e = hipMemcpy(g->img, img.data(), img.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(g->wy, wy.data(), wy.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess && !img16.empty()) {
        e = hipMalloc(&g->img16, img16.size() * 4);
        if (e == hipSuccess) e = hipMalloc(&g->wy16, wy16.size() * 4);
        if (e == hipSuccess) e = hipMemcpy(g->img16, img16.data(), img16.size() * 4, hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(g->wy16, wy16.data(), wy16.size() * 4, hipMemcpyHostToDevice);
    }
    if (e != hipSuccess) {
        if (g->img) (void)hipFree(g->img);
        if (g->wy) (void)hipFree(g->wy);
        if (g->img16) (void)hipFree(g->img16);
        if (g->wy16) (void)hipFree(g->wy16);
        delete g;
        return hip_fail(e, "npd_gru_create");
    }
    *out = g;
    return NPD_OK;
}

extern "C" int npd_gru_destroy(npd_gru* g) {
    if (!g) return NPD_OK;
    if (g->img) (void)hipFree(g->img);
    if (g->wy) (void)hipFree(g->wy);
    if (g->img16) (void)hipFree(g->img16);
    if (g->wy16) (void)hipFree(g->wy16);
    if (g->hd) (void)hipFree(g->hd);
    delete g;
    return NPD_OK;
}

extern "C" int npd_gru_decode_ex(const npd_gru* g, const float* y, const float* h0, const uint8_t* is_info, int reverse,
                                 const float* gt, float* decoded, float* logits, int64_t B, void* stream) {
    NPD_ARG(g != nullptr, "npd_gru_decode: gru is NULL");
    NPD_ARG(B >= 0, "npd_gru_decode: B < 0");
    if (B == 0) return NPD_OK;
    NPD_ARG(decoded != nullptr && is_info != nullptr, "npd_gru_decode: null pointer");
    NPD_ARG(y != nullptr || h0 != nullptr, "npd_gru_decode: y and h0 both NULL");
    NPD_ARG(((uintptr_t)y & 15) == 0, "npd_gru_decode: y must be 16-byte aligned");
    NPD_ARG(h0 == nullptr || g->precision == 0 || g->img16 != nullptr,
            "npd_gru_decode: an initial state (y_h0) needs precision 0 (fp32) or the 16-codeword split kernel "
            "(F = 64, 2 layers, N % 32 == 0)");
    NPD_ARG(y != nullptr || g->precision == 0 || g->img16 != nullptr,
            "npd_gru_decode: y = NULL (y_h0) needs precision 0 (fp32) or the 16-codeword split kernel");
    NPD_ARG(g->cell == 0 || ((y != nullptr) != (h0 != nullptr) && g->precision == 0),
            "npd_gru_decode: LSTM cells decode y_input (y, no initial state) or y_h0 (initial state, no y), fp32");
    gru::Args a{};
    a.img = g->img;
    a.wy = reinterpret_cast<const gru::f4*>(g->wy);
    a.y = y;
    a.h0 = h0;
    a.gt = gt;
    a.decoded = decoded;
    a.logits = logits;
    a.B = B;
    a.N = g->N;
    a.rev = reverse ? 1 : 0;
    a.onehot = g->onehot;
    a.b_lin = g->b_lin;
    a.ln = g->ln;
    a.ln_eps = g->ln_eps;
    a.hd = reinterpret_cast<const gru::f4*>(g->hd);
    a.hd_depth = g->hd_depth;
    a.hd_bout = g->hd_bout;
    for (int w = 0; w < kMaxWords; ++w) a.info[w] = 0;
    for (int i = 0; i < g->N; ++i)
        if (is_info[i]) a.info[i >> 5] |= 1u << (i & 31);
    hipStream_t s = (hipStream_t)stream;
    if (g->cell == 1) {
        const int N = g->N;
        if (g->F == 512) return g->layers == 2 ? gru::launch_lstm_wide<512, 2>(a, N, s) : gru::launch_lstm_wide<512, 1>(a, N, s);
        if (g->F == 256) return g->layers == 2 ? gru::launch_lstm_wide<256, 2>(a, N, s) : gru::launch_lstm_wide<256, 1>(a, N, s);
        if (g->F == 128) return g->layers == 2 ? gru::launch_lstm_wide<128, 2>(a, N, s) : gru::launch_lstm_wide<128, 1>(a, N, s);
        if (g->F == 64) return g->layers == 2 ? gru::launch_lstm_wide<64, 2>(a, N, s) : gru::launch_lstm<64, 1>(a, s);
        return g->layers == 2 ? gru::launch_lstm<32, 2>(a, s) : gru::launch_lstm<32, 1>(a, s);
    }
    if (g->precision != 0) {
        gru::ArgsB b{};
        b.img = g->img;
        b.wy = reinterpret_cast<const gru::f4*>(g->wy);
        b.y = y; b.h0 = h0; b.gt = gt; b.decoded = decoded; b.logits = logits; b.B = B; b.N = g->N;
        b.rev = a.rev; b.onehot = a.onehot; b.b_lin = g->b_lin; b.wy_lo = g->wy_lo;
        b.nseg = 1;
        for (int w = 0; w < kMaxWords; ++w) b.info[w] = a.info[w];
        if (g->img16) {
            b.img = g->img16;
            b.wy = reinterpret_cast<const gru::f4*>(g->wy16);
            b.wy_lo = g->wy16_lo;
            return g->split16 == 3 ? gru::launch16<3>(b, s) : g->split16 == 5 ? gru::launch16<5>(b, s)
                                   : gru::launch16<1>(b, s);
        }
#define NPD_LBF(FF, LL)                                                                                   \
        return g->precision == 1   ? gru::launch_bf<FF, LL, 3>(g, b, s)                                     \
               : g->precision == 3 ? gru::launch_bf<FF, LL, 4>(g, b, s)                                     \
                                   : gru::launch_bf<FF, LL, 1>(g, b, s)
        if (g->F == 64 && g->layers == 2) NPD_LBF(64, 2);
        if (g->F == 64) NPD_LBF(64, 1);
        if (g->layers == 2) NPD_LBF(32, 2);
        NPD_LBF(32, 1);
#undef NPD_LBF
    }
    if (g->F > 64) {
        if (g->F == 512) return g->layers == 2 ? gru::launch_wide<512, 2>(a, g->N, s) : gru::launch_wide<512, 1>(a, g->N, s);
        if (g->F == 256) return g->layers == 2 ? gru::launch_wide<256, 2>(a, g->N, s) : gru::launch_wide<256, 1>(a, g->N, s);
        return g->layers == 2 ? gru::launch_wide<128, 2>(a, g->N, s) : gru::launch_wide<128, 1>(a, g->N, s);
    }
    if (g->hd != nullptr) {  // out_linear_depth > 1 head (npd_rnn_create_ex): 1, 2 or 4 tiles of 32 head units
#define NPD_LHD(FF, LL) \
        return g->hd_tiles == 1 ? gru::launch<FF, LL, 1>(a, s) : g->hd_tiles == 2 ? gru::launch<FF, LL, 2>(a, s) \
                                                                                   : gru::launch<FF, LL, 4>(a, s)
        if (g->F == 64 && g->layers == 2) NPD_LHD(64, 2);
        if (g->F == 64) NPD_LHD(64, 1);
        if (g->layers == 2) NPD_LHD(32, 2);
        NPD_LHD(32, 1);
#undef NPD_LHD
    }
    if (g->F == 64 && g->layers == 2) return gru::launch<64, 2>(a, s);
    if (g->F == 64) return gru::launch<64, 1>(a, s);
    if (g->layers == 2) return gru::launch<32, 2>(a, s);
    return gru::launch<32, 1>(a, s);
}

extern "C" int npd_gru_decode_count_sweep(const npd_gru* g, int n_seg, const float* y, const uint8_t* is_info,
                                          int reverse, const float* msg, int K, const int32_t* cols, float* decoded,
                                          int64_t B, unsigned long long* counters, void* stream) {
    NPD_ARG(g != nullptr, "npd_gru_decode_count_sweep: gru is NULL");
    NPD_ARG(B >= 0 && n_seg >= 0 && K >= 0, "npd_gru_decode_count_sweep: negative size");
    if (B == 0 || n_seg == 0) return NPD_OK;
    NPD_ARG(y != nullptr && is_info != nullptr && counters != nullptr && (K == 0 || (msg != nullptr && cols != nullptr)),
            "npd_gru_decode_count_sweep: null pointer");
    NPD_ARG(((uintptr_t)y & 15) == 0, "npd_gru_decode_count_sweep: y must be 16-byte aligned");
    NPD_ARG(K <= g->N, "npd_gru_decode_count_sweep: K > N");
    uint8_t slot[kMaxN];
    memset(slot, 255, sizeof(slot));
    for (int k = 0; k < K; ++k) {
        NPD_ARG(cols[k] >= 0 && cols[k] < g->N, "npd_gru_decode_count_sweep: column out of range");
        NPD_ARG(slot[cols[k]] == 255, "npd_gru_decode_count_sweep: repeated column");
        slot[cols[k]] = (uint8_t)k;
    }
    hipStream_t s = (hipStream_t)stream;
    if (g->img16 == nullptr || g->cell != 0) {
        // other kernels: one decode and one column count per segment (the same counts), into the caller's decoded
        NPD_ARG(decoded != nullptr, "npd_gru_decode_count_sweep: handles other than the 16-codeword split kernel (F = 64, "
                                    "2 layers, N % 32 == 0, precision != 0) need decoded (n_seg, B, N)");
        const int64_t rows = B * g->N;
        for (int sg = 0; sg < n_seg; ++sg) {
            int rc = npd_gru_decode_ex(g, y + sg * rows, nullptr, is_info, reverse, nullptr, decoded + sg * rows, nullptr,
                                       B, stream);
            if (rc == NPD_OK && K > 0)
                rc = npd_count_errors_cols(msg, decoded + sg * rows, B, K, g->N, cols, counters + 2 * sg, stream);
            if (rc != NPD_OK) return rc;
        }
        return NPD_OK;
    }
    gru::ArgsB b{};
    b.img = g->img16;
    b.wy = reinterpret_cast<const gru::f4*>(g->wy16);
    b.wy_lo = g->wy16_lo;
    b.y = y; b.h0 = nullptr; b.gt = nullptr; b.decoded = decoded; b.logits = nullptr; b.B = B; b.N = g->N;
    b.rev = reverse ? 1 : 0; b.onehot = g->onehot; b.b_lin = g->b_lin;
    for (int w = 0; w < kMaxWords; ++w) b.info[w] = 0;
    for (int i = 0; i < g->N; ++i)
        if (is_info[i]) b.info[i >> 5] |= 1u << (i & 31);
    b.msg = msg; b.counters = counters; b.K = K; b.nseg = n_seg;
    memcpy(b.slotw, slot, sizeof(slot));
    return g->split16 == 3 ? gru::launch16<3>(b, s) : g->split16 == 5 ? gru::launch16<5>(b, s) : gru::launch16<1>(b, s);
}

extern "C" int npd_gru_decode(const npd_gru* g, const float* y, const uint8_t* is_info, int reverse, const float* gt,
                              float* decoded, float* logits, int64_t B, void* stream) {
    if (B > 0 && y == nullptr) return fail(NPD_EINVAL, "npd_gru_decode: null pointer");
    return npd_gru_decode_ex(g, y, nullptr, is_info, reverse, gt, decoded, logits, B, stream);
}

// ---------------------------------------------------------------------------------- y MLP (decoding_type 'y_h0')
// One Linear layer + activation of RNN_Model.get_h0 / get_Fy (rnn_all.py:362-385): out[b][j] = act(sum_k x[b][k]
// W[j][k] + bias[j]), fp32, k summed in order.  64 x 64 outputs per 256-thread block (4 x 4 per thread, strided by
// 16 so a row's 16 lanes read consecutive W rows from LDS), K in LDS-staged chunks of 16.  Once per codeword (the
// MLP is < 2 % of a hidden-64 decode's MACs), so plain FMA, no MFMA.
namespace npd {
namespace gru {
constexpr int MK = 16;

__device__ __forceinline__ float mlp_act(float x, int act) {
    switch (act) {
        case 1: return x > 0.0f ? x : 0.0f;                                           // relu
        case 2: return 1.0507009873554805f * (x > 0.0f ? x : 1.6732632423543772f * expm1f(x));  // selu
        case 3: return x > 0.0f ? x : expm1f(x);                                      // elu (alpha 1)
        case 4: return tanhf(x);
        case 5: return 1.0f / (1.0f + expf(-x));                                      // sigmoid
        default: return x;                                                            // linear / unknown
    }
}

__global__ __launch_bounds__(256) void mlp_layer_kernel(const float* __restrict__ x, const float* __restrict__ W,
                                                        const float* __restrict__ bias, float* __restrict__ out,
                                                        int64_t B, int K, int Nout, int act) {
    __shared__ float xs[64][MK + 1];
    __shared__ float ws[64][MK + 1];
    const int tid = threadIdx.x;
    const int ty = tid >> 4, tx = tid & 15;
    const int64_t m0 = (int64_t)blockIdx.y * 64;
    const int j0 = blockIdx.x * 64;
    float acc[4][4] = {};
    for (int k0 = 0; k0 < K; k0 += MK) {
        for (int e = tid; e < 64 * MK; e += 256) {
            const int r = e / MK, k = e % MK;
            const int64_t m = m0 + r;
            const int j = j0 + r;
            xs[r][k] = (m < B && k0 + k < K) ? x[m * K + k0 + k] : 0.0f;
            ws[r][k] = (j < Nout && k0 + k < K) ? W[(int64_t)j * K + k0 + k] : 0.0f;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < MK; ++k)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int c = 0; c < 4; ++c) acc[i][c] = fmaf(xs[ty + 16 * i][k], ws[tx + 16 * c][k], acc[i][c]);
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int64_t m = m0 + ty + 16 * i;
        if (m >= B) continue;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int j = j0 + tx + 16 * c;
            if (j < Nout) out[m * Nout + j] = mlp_act(acc[i][c] + bias[j], act);
        }
    }
}
}  // namespace gru
}  // namespace npd

extern "C" int npd_ymlp_layer(const float* x, const float* W, const float* bias, float* out, int64_t B, int K, int Nout,
                              int act, void* stream) {
    NPD_ARG(B >= 0 && K > 0 && Nout > 0, "npd_ymlp_layer: bad sizes");
    if (B == 0) return NPD_OK;
    NPD_ARG(x != nullptr && W != nullptr && bias != nullptr && out != nullptr, "npd_ymlp_layer: null pointer");
    NPD_ARG(act >= 0 && act <= 5, "npd_ymlp_layer: act must be 0 (linear), 1 relu, 2 selu, 3 elu, 4 tanh, 5 sigmoid");
    NPD_ARG(B <= (int64_t)65535 * 64, "npd_ymlp_layer: B too large for one launch (split the batch)");
    dim3 grid((unsigned)((Nout + 63) / 64), (unsigned)((B + 63) / 64));
    hipLaunchKernelGGL(gru::mlp_layer_kernel, grid, dim3(256), 0, (hipStream_t)stream, x, W, bias, out, B, K, Nout, act);
    return launch_check("mlp_layer_kernel launch");
}
