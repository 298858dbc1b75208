// npd_sc_fast.hip -- the hot path: Polar SC min-sum decode for N <= 64, msg_hat + fused counters.
//
// Same arithmetic as npd_sc.hip (PolarCode.sc_decode_new, polar.py:465-484; bit-exact), restructured
// for HBM streaming at one wave per SIMD:
//   * software pipeline across tiles: while tile t is decoded from VGPRs, the 64 x N fp32 words of
//     tile t+1 are already in flight as coalesced global_load_dwordx4 into registers (no LDS-DMA, so
//     the compiler never has to drain them before an LDS access);
//   * tile t+1 is transposed to one-row-per-lane through an XOR-swizzled LDS image
//     (ds_write_b128 / ds_read_b128, conflict-free) at the top of its iteration;
//   * decisions of information positions are written as int8 in SLOT order (rank of the position),
//     so msg_hat rows are contiguous bytes: the error count compares 4 slots per dword against the
//     Philox message bits, and msg_hat leaves as coalesced 16-B stores.
#include "npd_common.hpp"

#include <cstdlib>

// Tuning knobs (compile-time; defaults are the measured best on MI355X):
#ifndef NPD_SCF_WPE
#define NPD_SCF_WPE 2
#endif
#ifndef NPD_SCF_WPB
#define NPD_SCF_WPB 8  // waves per workgroup (each with its own LDS tile; they share only the counter reduction)
#endif

namespace npd {
namespace scf {

constexpr int kMaxSeg = 16;  // SNR points of one sweep launch

// A launch decodes n_seg segments of B codewords each (the SNR points of a Monte-Carlo sweep), stored
// back to back: y (n_seg, B, N), msg (n_seg, B, K), counters (n_seg, 2).  n_seg = 1 is the plain call.
struct Args {
    const float* y;
    float* msg;                      // (n_seg, B, K) or null
    unsigned long long* counters;    // (n_seg, 2) {bit errors, block errors} or null
    uint64_t seed;
    uint64_t cw_offset;
    int64_t B;
    int64_t ntiles;                  // tiles per segment
    float scale[kMaxSeg];
    float sigma[kMaxSeg];            // GEN: channel sigma of each segment
    uint32_t snr_index0;             // GEN: Philox noise stream of segment s = kStreamNoise + snr_index0 + s
    int n_seg;
    uint32_t count;
    uint32_t ilv;                    // tile order: 0 = a workgroup's waves take adjacent tiles, 1 = interleaved
};

__device__ __forceinline__ float rmul(float a, float b) {
    float r = a * b;
    asm("" : "+v"(r));  // keep fl32(scale*y) rounded (no fma contraction), as polar.py:468
    return r;
}

// sign(a) sign(b) min(|a|, |b|) in two VALU ops: med3(|a|, -|a|, b) = clamp(b, -|a|, |a|) has the
// magnitude min(|a|, |b|) and the sign of b; xor in the sign of a (v_med3_f32 + v_bitop3_b32).
// Equal in value to the reference's product form (zeros may differ only in their sign bit, which
// no later step reads: sign(+-0) = 0, |+-0| = 0, u * (+-0) + b = b).
__device__ __forceinline__ float f_minsum(float a, float b) {
    const float m = __builtin_amdgcn_fmed3f(__builtin_fabsf(a), -__builtin_fabsf(a), b);
    return bitsf(__builtin_amdgcn_bitop3_b32(fbits(m), fbits(a), 0x80000000u, 0x78));  // m ^ (a & 0x80000000)
}

__device__ __forceinline__ float sgn_bits(float x) {
    const float s = bitsf((fbits(x) & 0x80000000u) | 0x3f800000u);
    return (x == 0.0f) ? 0.0f : s;
}

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

template <int N>
struct Lane {
    float lv[2 * N];   // level d at lv[2^d .. 2^(d+1)); input level at lv[N .. 2N)
    float beta[N];
    char* lds;
    uint32_t u_row;    // byte address of this lane's decision row (slot order)
    uint32_t slot;     // wave-uniform running rank of the next information position
    uint32_t fz[(N + 31) / 32];  // frozen-position bits (re-materialised each tile, see below)
    float infty;
};

template <int N, int I>
__device__ __forceinline__ void leaf(Lane<N>& c, const CodeParams& p, float L) {
    const bool frozen = (c.fz[I >> 5] >> (I & 31)) & 1u;
    // prior selected on the scalar unit (frozen and infty are wave-uniform): one v_add_f32
    const uint32_t pbits = __builtin_amdgcn_readfirstlane(frozen ? fbits(c.infty) : 0u);
    const float lf = L + bitsf(pbits);  // polar.py:438/446
    const float u = sgn_bits(lf);                     // polar.py:479
    if (!frozen) {
        *reinterpret_cast<int8_t*>(c.lds + c.u_row + c.slot) = (int8_t)(int)u;
        ++c.slot;
    }
    c.beta[I] = u;
}

template <int N, int D, int S0>
__device__ __forceinline__ void node(Lane<N>& c, const CodeParams& p) {
    if constexpr (D == 0) {
        leaf<N, S0>(c, p, c.lv[1]);
    } else {
        constexpr int h = 1 << (D - 1);
#pragma unroll
        for (int j = 0; j < h; ++j) c.lv[h + j] = f_minsum(c.lv[2 * h + j], c.lv[3 * h + j]);
        node<N, D - 1, S0>(c, p);
        if constexpr (h >= 2) {
            // g and the partial-sum products as packed fp32 (v_pk_fma_f32 / v_pk_mul_f32: two lanes' worth
            // per instruction).  u * a is exact (u in {-1, 0, 1}), so the fused form equals mul + add.
#pragma unroll
            for (int j = 0; j < h; j += 2) {
                const f2 u2 = {c.beta[S0 + j], c.beta[S0 + j + 1]};
                const f2 a2 = {c.lv[2 * h + j], c.lv[2 * h + j + 1]};
                const f2 b2 = {c.lv[3 * h + j], c.lv[3 * h + j + 1]};
                const f2 r = __builtin_elementwise_fma(u2, a2, b2);
                c.lv[h + j] = r.x;
                c.lv[h + j + 1] = r.y;
            }
        } else {
#pragma unroll
            for (int j = 0; j < h; ++j) c.lv[h + j] = c.beta[S0 + j] * c.lv[2 * h + j] + c.lv[3 * h + j];
        }
        node<N, D - 1, S0 + h>(c, p);
        if constexpr ((1 << D) < N) {
            if constexpr (h >= 2) {
#pragma unroll
                for (int j = 0; j < h; j += 2) {
                    const f2 x = {c.beta[S0 + j], c.beta[S0 + j + 1]};
                    const f2 y = {c.beta[S0 + h + j], c.beta[S0 + h + j + 1]};
                    const f2 r = x * y;
                    c.beta[S0 + j] = r.x;
                    c.beta[S0 + j + 1] = r.y;
                }
            } else {
#pragma unroll
                for (int j = 0; j < h; ++j) c.beta[S0 + j] = c.beta[S0 + j] * c.beta[S0 + h + j];
            }
        }
    }
}


// ------------------------------------------------------------------------------------- specialised codes
// For the reference's standard Polar codes the frozen set is a compile-time constant, so the decoder is
// unrolled against it: leaf tests, slot offsets and subtree classes are resolved at compile time, and
// three subtree classes are decoded in closed form where that is provably identical to the step-by-step
// SC (polar.py:465-484):
//  * rate-0 (all frozen) and repetition (only the last leaf informative): if sum |a_j| < 999 over the
//    subtree's input LLRs a, every leaf LLR inside has magnitude < 1000 (g adds magnitudes, f takes a
//    minimum, all partial sums are +1), so every frozen leaf decides sign(L + 1000) = +1; the partial sums
//    are +1 (rate-0) and the repetition node's informative leaf sees the SC-order pairwise sum of a;
//  * rate-1 (all informative): if no a_j is 0, SC's partial sums equal sign(a) (by induction: f keeps
//    |.| > 0, g adds two terms of equal sign) and the decisions are their Plotkin transform.
// A lane whose inputs break a condition flags the tile; the whole tile is then decoded again by the
// step-by-step path (reloaded from the LDS image), so results never depend on the shortcut.
namespace spec {

template <int N, uint64_t M>
struct CT {
    static constexpr bool frozen(int i) { return ((M >> i) & 1ull) != 0; }
    static constexpr int rank(int i) {
        int r = 0;
        for (int j = 0; j < i; ++j) r += frozen(j) ? 0 : 1;
        return r;
    }
    static constexpr int type(int D, int S0) {
        int k = 0;
        for (int i = S0; i < S0 + (1 << D); ++i) k += frozen(i) ? 0 : 1;
        if (k == 0) return kNodeRate0;
        if (k == (1 << D)) return kNodeRate1;
        if (k == 1 && !frozen(S0 + (1 << D) - 1)) return kNodeRep;
        return kNodeMixed;
    }
};

template <int N, uint64_t M, int D, int S0>
__device__ __forceinline__ void snode(Lane<N>& c, uint32_t& bad) {
    using T = CT<N, M>;
    constexpr int SZ = 1 << D;
    if constexpr (D == 0) {
        const float L = c.lv[1];
        if constexpr (T::frozen(S0)) {
            c.beta[S0] = sgn_bits(L + c.infty);  // polar.py:438/446, 479
        } else {
            const float u = sgn_bits(L);
            *reinterpret_cast<int8_t*>(c.lds + c.u_row + T::rank(S0)) = (int8_t)(int)u;
            c.beta[S0] = u;
        }
    } else if constexpr (T::type(D, S0) == kNodeRate0 || T::type(D, S0) == kNodeRep) {
        float sa = 0.0f;
#pragma unroll
        for (int j = 0; j < SZ; ++j) sa += __builtin_fabsf(c.lv[SZ + j]);
        bad |= (sa < 999.0f) ? 0u : 1u;
        if constexpr (T::type(D, S0) == kNodeRate0) {
#pragma unroll
            for (int j = 0; j < SZ; ++j) c.beta[S0 + j] = 1.0f;
        } else {
            float t[SZ];
#pragma unroll
            for (int j = 0; j < SZ; ++j) t[j] = c.lv[SZ + j];
#pragma unroll
            for (int h = SZ / 2; h >= 1; h /= 2)
#pragma unroll
                for (int j = 0; j < h; ++j) t[j] = t[j] + t[h + j];  // g-updates with u = +1
            const float u = sgn_bits(t[0]);
            *reinterpret_cast<int8_t*>(c.lds + c.u_row + T::rank(S0 + SZ - 1)) = (int8_t)(int)u;
#pragma unroll
            for (int j = 0; j < SZ; ++j) c.beta[S0 + j] = u;
        }
    } else if constexpr (T::type(D, S0) == kNodeRate1) {
        float m = __builtin_fabsf(c.lv[SZ]);
#pragma unroll
        for (int j = 1; j < SZ; ++j) m = __builtin_fminf(m, __builtin_fabsf(c.lv[SZ + j]));
        bad |= (m > 0.0f) ? 0u : 1u;
        float b[SZ];
#pragma unroll
        for (int j = 0; j < SZ; ++j) {
            b[j] = bitsf((fbits(c.lv[SZ + j]) & 0x80000000u) | 0x3f800000u);
            c.beta[S0 + j] = b[j];
        }
#pragma unroll
        for (int st = 1; st < SZ; st *= 2)
#pragma unroll
            for (int i = 0; i < SZ; i += 2 * st)
#pragma unroll
                for (int j = 0; j < st; ++j) b[i + j] = b[i + j] * b[i + st + j];
#pragma unroll
        for (int j = 0; j < SZ; ++j)
            *reinterpret_cast<int8_t*>(c.lds + c.u_row + T::rank(S0) + j) = (int8_t)(int)b[j];
    } else {
        constexpr int h = SZ / 2;
#pragma unroll
        for (int j = 0; j < h; ++j) c.lv[h + j] = f_minsum(c.lv[2 * h + j], c.lv[3 * h + j]);
        snode<N, M, D - 1, S0>(c, bad);
#pragma unroll
        for (int j = 0; j < h; ++j) c.lv[h + j] = c.beta[S0 + j] * c.lv[2 * h + j] + c.lv[3 * h + j];
        snode<N, M, D - 1, S0 + h>(c, bad);
        if constexpr (SZ < N) {
#pragma unroll
            for (int j = 0; j < h; ++j) c.beta[S0 + j] = c.beta[S0 + j] * c.beta[S0 + h + j];
        }
    }
}

}  // namespace spec

template <int N>
constexpr int log2c() {
    int n = 0;
    while ((1 << n) < N) ++n;
    return n;
}

template <int C>
__device__ __forceinline__ int swz(int r) {
    if constexpr (C >= 16) return r & 15;
    else return (r / (16 / C)) % C;
}

// number of nonzero bytes in x
__device__ __forceinline__ uint32_t nz_bytes(uint32_t x) {
    const uint32_t t = ((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x;
    return (uint32_t)__builtin_popcount(t & 0x80808080u);
}

// msg_hat of one finished tile: its rows*K floats are contiguous in HBM; decisions are int8 in slot order
template <int N>
__device__ __forceinline__ void store_msg(const char* lds, uint32_t kU, float* msg, int64_t row0, int rows, int K,
                                          int lane, int NB) {
    float* dst = msg + row0 * (int64_t)K;
    const int total = rows * K;
    if ((K & 3) == 0) {
        // batches of 4: the LDS reads first, then the conversions and 16-B stores (one wait per batch)
        int r = (4 * lane) / K, col = (4 * lane) % K;
        const int dr = 256 / K, dc = 256 % K;
        for (int f0 = 4 * lane; f0 < total; f0 += 4 * 256) {
            uint32_t w[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                w[i] = (f0 + 256 * i < total) ? *reinterpret_cast<const uint32_t*>(lds + kU + (uint32_t)(r * NB + col))
                                              : 0u;
                r += dr;
                col += dc;
                if (col >= K) {
                    col -= K;
                    ++r;
                }
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int f = f0 + 256 * i;
                if (f < total) {
                    f4 o;
                    o.x = (float)(int8_t)(w[i] & 0xFFu);
                    o.y = (float)(int8_t)((w[i] >> 8) & 0xFFu);
                    o.z = (float)(int8_t)((w[i] >> 16) & 0xFFu);
                    o.w = (float)(int8_t)(w[i] >> 24);
                    *reinterpret_cast<f4*>(dst + f) = o;
                }
            }
        }
    } else {
        int r = lane / K, col = lane % K;
        const int dr = kWave / K, dc = kWave % K;
        for (int f = lane; f < total; f += kWave) {
            dst[f] = (float)*reinterpret_cast<const int8_t*>(lds + kU + (uint32_t)(r * NB + col));
            r += dr;
            col += dc;
            if (col >= K) {
                col -= K;
                ++r;
            }
        }
    }
}

// chunk q of tile t for this lane = float4 index t*64*C + lane + 64*q.  Full tiles (all but possibly the
// last) address from a wave-uniform base (SGPR) plus the lane offset: no per-chunk 64-bit clamps.
template <int C>
__device__ __forceinline__ void load_tile(f4 (&nx)[C], const f4* __restrict__ y4, int64_t t, int lane, int64_t B,
                                          int64_t last4) {
    const f4* base = y4 + t * (int64_t)(kWave * C);
    if ((t + 1) * kWave <= B) {
#pragma unroll
        for (int q = 0; q < C; ++q) {
            nx[q] = base[lane + kWave * q];
        }
    } else {
#pragma unroll
        for (int q = 0; q < C; ++q) {
            const int64_t gi = t * (int64_t)(kWave * C) + lane + kWave * q;
            nx[q] = y4[gi < last4 ? gi : last4];
        }
    }
}

template <int N>
__device__ __forceinline__ void frozen_words_init(Lane<N>& c, const CodeParams& p) {
#pragma unroll
    for (int w = 0; w < (N + 31) / 32; ++w) {
        uint32_t fw = p.frozen[w];
        asm volatile("" : "+s"(fw));
        c.fz[w] = fw;
    }
}

// decision-row stride: an odd number of dwords holding the K slot bytes (conflict-free dword reads)
__host__ __device__ constexpr int row_stride(int K) { return 4 * ((((K > 0 ? K : 1) + 3) / 4) | 1); }

// ---- GEN (fused Monte-Carlo): the received word of this lane's codeword is generated in registers,
// value for value what npd_mc_generate writes (npd_gen.hip): message bits (Philox block 0 of the
// message stream) scattered to the information positions, Plotkin butterfly as XOR on bit words, then
// per 16-B chunk j the Philox noise block (cw, j) -> 4 Box-Muller normals -> y = x + fl32(sigma z).
template <int N, uint64_t MASK, bool SPEC>
__device__ __forceinline__ void codeword_bits(const uint32_t (&mw)[4], const uint32_t* fz, uint32_t (&U)[(N + 31) / 32]) {
    constexpr int NW = (N + 31) / 32;
#pragma unroll
    for (int w = 0; w < NW; ++w) U[w] = 0u;
    int kk = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const bool frozen = SPEC ? (((MASK >> i) & 1ull) != 0) : (((fz[i >> 5] >> (i & 31)) & 1u) != 0);
        if (!frozen) {
            U[i >> 5] |= ((mw[kk >> 5] >> (kk & 31)) & 1u) << (i & 31);
            ++kk;
        }
    }
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
}

template <int N>
__device__ __forceinline__ void gen_llrs(float* lv, const uint32_t (&U)[(N + 31) / 32], uint64_t seed, uint32_t stream,
                                         uint64_t cw, float sigma, float scale) {
#pragma unroll
    for (int j = 0; j < N / 4; ++j) {
        const u32x4 o = philox_block(seed, stream, cw, (uint32_t)j);
        float z[4];
        normals4(o, z);
        const uint32_t bits = (U[(4 * j) >> 5] >> ((4 * j) & 31)) & 0xFu;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float xv = ((bits >> e) & 1u) ? -1.0f : 1.0f;
            lv[4 * j + e] = rmul(scale, __fadd_rn(xv, __fmul_rn(sigma, z[e])));
        }
    }
}

// GEN (nothing staged, ~108 VGPRs): two 8-wave workgroups per CU = 4 waves per SIMD hide the Philox /
// Box-Muller dependency chains; the streaming decoder keeps one workgroup (LDS-bound, 2 waves per SIMD)
template <int N, uint64_t MASK = 0, bool SPEC = false, bool GEN = false>
__global__ __launch_bounds__(64 * NPD_SCF_WPB, GEN ? 2 : NPD_SCF_WPE * 4 / NPD_SCF_WPB) void sc_fast_kernel(
    const CodeParams p, const Args a) {
    constexpr int KC = N - __builtin_popcountll(MASK);  // information bits of a specialised code
    extern __shared__ __attribute__((aligned(16))) char lds_all[];
    constexpr int n = log2c<N>();
    constexpr int C = N / 4;                 // 16-B chunks per row (and per lane per tile)
    const int K = p.K;
    const int NB = SPEC ? row_stride(KC) : row_stride(K);
    const int wpb = blockDim.x >> 6;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
    const int lane = threadIdx.x & 63;
    // per-wave LDS: the staged tile (64 rows x N fp32) then 64 decision rows of NB bytes
    constexpr uint32_t kStageBytes = GEN ? 0u : (uint32_t)(kWave * N * 4);  // GEN generates y in registers
    const uint32_t per_wave = kStageBytes + (uint32_t)(kWave * NB);
    char* lds = lds_all + wave * per_wave;
    constexpr uint32_t kStage = 0;
    constexpr uint32_t kU = kStageBytes;

    Lane<N> c;
    c.lds = lds;
    c.u_row = kU + (uint32_t)(lane * NB);
    const int sw = swz<C>(lane);

    uint32_t err_bits = 0, err_blocks = 0;
    // per-wave partial counts per segment, flushed when the wave moves to another segment
    uint32_t* red = reinterpret_cast<uint32_t*>(lds_all + wpb * per_wave + N);
    if (a.count && lane < 2 * kMaxSeg) red[wave * 2 * kMaxSeg + lane] = 0u;
    const int64_t segC = a.B * C;  // float4s per segment

    // prefetch registers: chunk q of tile t for this lane = float4 index t*64*C + lane + 64*q
    f4 nx[C];
    int64_t pend_row0 = 0;  // previous tile: its msg_hat stores are issued one iteration late
    int pend_rows = 0, pend_seg = 0;
    // position (seg, t) of this wave's tiles: global tile index g = seg * ntiles + t, stride gstride
    int64_t gstride = (int64_t)gridDim.x * wpb;
    asm volatile("" : "+s"(gstride));  // keep the grid stride in SGPRs (otherwise re-read every tile)
    const int64_t total = a.ntiles * a.n_seg;
    // first tile of this wave: adjacent tiles go to the waves of one workgroup (ilv = 0) or to consecutive
    // workgroups, i.e. round-robin over the XCDs (ilv = 1); either way the waves partition the tiles
    int64_t g = a.ilv ? (int64_t)wave * gridDim.x + blockIdx.x : (int64_t)blockIdx.x * wpb + wave;
    int seg = (int)(g / (a.ntiles > 0 ? a.ntiles : 1));
    int64_t t = g - (int64_t)seg * a.ntiles;
    int cur_seg = seg;
    if (!GEN && g < total)
        load_tile<C>(nx, reinterpret_cast<const f4*>(a.y) + seg * segC, t, lane, a.B, segC - 1);
    auto flush = [&](int sg) {
        const uint32_t eb = wave_sum_u32(err_bits);
        const uint32_t bl = wave_sum_u32(err_blocks);
        if (lane == 0) {
            red[wave * 2 * kMaxSeg + 2 * sg] += eb;
            red[wave * 2 * kMaxSeg + 2 * sg + 1] += bl;
        }
        err_bits = 0;
        err_blocks = 0;
    };
    for (; g < total; g += gstride) {
        if (a.count && seg != cur_seg) {
            flush(cur_seg);
            cur_seg = seg;
        }
        float scale = a.scale[seg];
        asm volatile("" : "+s"(scale));
        const int64_t last4 = segC - 1;  // last valid float4 of this segment
        // next tile of this wave
        int64_t tn = t + gstride;
        int segn = seg;
        while (tn >= a.ntiles && segn < a.n_seg) {
            tn -= a.ntiles;
            ++segn;
        }
        const int64_t row0 = t * kWave;
        const int rows = (int)((a.B - row0) < kWave ? (a.B - row0) : kWave);
        // ---- this tile's message bits (Philox, pure VALU) first: it fills the wait for the tile's data.
        // The seed is made opaque per tile so the key schedule is recomputed with scalar adds here
        // instead of being hoisted into 20 loop-invariant SGPRs (which spill to VGPR lanes).
        uint32_t mw[4] = {0u, 0u, 0u, 0u};
        if (GEN || a.count) {
            uint64_t sd = a.seed;
            asm volatile("" : "+s"(sd));
            const u32x4 o = philox_block(sd, kStreamMsg, a.cw_offset + (uint64_t)(row0 + lane), 0u);
            mw[0] = o.x;
            mw[1] = o.y;
            mw[2] = o.z;
            mw[3] = o.w;
        }
        if constexpr (GEN && !SPEC) frozen_words_init(c, p);
        uint32_t Ubits[(N + 31) / 32];
        if constexpr (GEN) {
            codeword_bits<N, MASK, SPEC>(mw, c.fz, Ubits);
            // previous tile's msg_hat before this tile's leaves overwrite the decision rows
            if (a.msg && pend_rows > 0) store_msg<N>(lds, kU, a.msg + pend_seg * a.B * K, pend_row0, pend_rows, K, lane, NB);
            uint64_t sd = a.seed;
            asm volatile("" : "+s"(sd));
            gen_llrs<N>(c.lv + N, Ubits, sd, kStreamNoise + a.snr_index0 + (uint32_t)seg, a.cw_offset + (uint64_t)(row0 + lane),
                        a.sigma[seg], scale);
        } else {
        // ---- transpose the tile through LDS: chunk (lane + 64q) -> row r = (lane + 64q)/C, col chunk
#pragma unroll
        for (int q = 0; q < C; ++q) {
            const int pch = lane + kWave * q;
            const int r = pch / C, cc = pch % C;
            *reinterpret_cast<f4*>(lds + kStage + 16u * (uint32_t)(r * C + (cc ^ swz<C>(r)))) = nx[q];
        }
        // ---- prefetch the next tile as soon as its registers are free (lands while this one is decoded)
        if (g + gstride < total)
            load_tile<C>(nx, reinterpret_cast<const f4*>(a.y) + segn * segC, tn, lane, a.B, last4);
        // ---- previous tile's msg_hat (its decision rows are read before this tile's leaves overwrite them;
        // done before this tile's LLRs occupy registers)
        if (a.msg && pend_rows > 0)
            store_msg<N>(lds, kU, a.msg + pend_seg * a.B * K, pend_row0, pend_rows, K, lane, NB);
        {
#pragma unroll
            for (int q = 0; q < C; ++q) {
                const f4 v = *reinterpret_cast<const f4*>(lds + kStage + 16u * (uint32_t)(lane * C + (q ^ sw)));
                c.lv[N + 4 * q + 0] = rmul(scale, v.x);
                c.lv[N + 4 * q + 1] = rmul(scale, v.y);
                c.lv[N + 4 * q + 2] = rmul(scale, v.z);
                c.lv[N + 4 * q + 3] = rmul(scale, v.w);
            }
        }
        }  // !GEN
        // ---- decode.  The per-leaf frozen tests are loop-invariant; left alone the compiler hoists all
        // of them out of the tile loop and spills the resulting 64 SGPR pairs to VGPR lanes.  Making the
        // frozen words opaque per tile keeps each test a single s_bitcmp next to its leaf.
        auto frozen_words = [&] {
#pragma unroll
            for (int w = 0; w < (N + 31) / 32; ++w) {
                uint32_t fw = p.frozen[w];
                asm volatile("" : "+s"(fw));
                c.fz[w] = fw;
            }
        };
        if constexpr (!SPEC && !GEN) frozen_words();
        {
            float inf = p.infty;
            asm volatile("" : "+s"(inf));
            c.infty = inf;
        }
        c.slot = 0;
        if constexpr (SPEC) {
            uint32_t bad = 0;
            spec::snode<N, MASK, n, 0>(c, bad);
            if (__ballot(bad != 0u) != 0ull) {
                // a shortcut's precondition failed on some lane (huge or zero LLRs): decode the tile again
                // step by step from the LDS image of its received words (GEN: regenerated)
                if constexpr (GEN) {
                    uint64_t sd = a.seed;
                    asm volatile("" : "+s"(sd));
                    gen_llrs<N>(c.lv + N, Ubits, sd, kStreamNoise + a.snr_index0 + (uint32_t)seg,
                                a.cw_offset + (uint64_t)(row0 + lane), a.sigma[seg], scale);
                } else {
#pragma unroll
                for (int q = 0; q < C; ++q) {
                    const f4 v = *reinterpret_cast<const f4*>(lds + kStage + 16u * (uint32_t)(lane * C + (q ^ sw)));
                    c.lv[N + 4 * q + 0] = rmul(scale, v.x);
                    c.lv[N + 4 * q + 1] = rmul(scale, v.y);
                    c.lv[N + 4 * q + 2] = rmul(scale, v.z);
                    c.lv[N + 4 * q + 3] = rmul(scale, v.w);
                }
                }
                c.slot = 0;
                frozen_words();
                node<N, n, 0>(c, p);
            }
        } else {
            node<N, n, 0>(c, p);
        }

        // ---- error count: 4 slots per dword vs the Philox message bits (errors_ber/bler semantics)
        if (a.count) {
            // all decision dwords first (reads past slot K land in the next row or the slack after the last
            // wave's rows and are masked out), then branch-free masking: slots >= K contribute nothing
            uint32_t dec[N / 4];
#pragma unroll
            for (int w = 0; w < N / 4; ++w)
                dec[w] = *reinterpret_cast<const uint32_t*>(lds + c.u_row + 4 * w);
            uint32_t e = 0;
#pragma unroll
            for (int w = 0; w < N / 4; ++w) {
                if (SPEC && 4 * w >= KC) continue;
                const uint32_t nib = (mw[(4 * w) >> 5] >> ((4 * w) & 31)) & 0xFu;
                const uint32_t x = (nib * 0x00204081u) & 0x01010101u;  // bit i -> byte i
                const uint32_t expect = 0x01010101u | ((x << 8) - x);  // +1 -> 0x01, -1 -> 0xFF
                const int valid = (SPEC ? KC : K) - 4 * w;                 // slots in this dword
                const uint32_t vmask = valid >= 4 ? 0xFFFFFFFFu : (valid <= 0 ? 0u : ((1u << (8 * valid)) - 1u));
                e += nz_bytes((dec[w] ^ expect) & vmask);
            }
            if (lane < rows) {
                err_bits += e;
                err_blocks += e ? 1u : 0u;
            }
        }

        pend_row0 = row0;
        pend_rows = rows;
        pend_seg = seg;
        seg = segn;
        t = tn;
    }
    // the last tile's msg_hat
    if (a.msg && pend_rows > 0) store_msg<N>(lds, kU, a.msg + pend_seg * a.B * K, pend_row0, pend_rows, K, lane, NB);

    if (a.count) {
        // one pair of device atomics per workgroup and segment: same-address atomics from every wave
        // serialise at the memory side (~20 us per launch at one pair per wave)
        flush(cur_seg);
        __syncthreads();
        if ((int)threadIdx.x < 2 * a.n_seg) {
            unsigned long long sum = 0;
            for (int w = 0; w < wpb; ++w) sum += red[w * 2 * kMaxSeg + threadIdx.x];
            if (sum) atomicAdd(a.counters + threadIdx.x, sum);
        }
    }
}

template <int N, uint64_t MASK = 0, bool SPEC = false, bool GEN = false>
static int launch(const CodeParams& p, Args a, hipStream_t s) {
    constexpr int KC = N - __builtin_popcountll(MASK);
    const int NB = row_stride(SPEC ? KC : p.K);
    const size_t per_wave = (GEN ? (size_t)0 : (size_t)kWave * N * 4) + (size_t)kWave * NB;
    // as many waves per workgroup as fit (up to NPD_SCF_WPB): fewer workgroups -> fewer counter atomics
    int wpb = NPD_SCF_WPB;
    if (const char* e = getenv("NPD_SCF_WPB")) {  // A/B: waves per workgroup (1..8)
        const int v = atoi(e);
        if (v >= 1 && v <= NPD_SCF_WPB) wpb = v;
    }
    const size_t red = (size_t)8 * kMaxSeg;  // per wave: n_seg x {bits, blocks} uint32
    while (wpb > 1 && (size_t)wpb * (per_wave + red) + N > 160 * 1024) --wpb;
    const size_t lds = (size_t)wpb * (per_wave + red) + N;
    a.ntiles = (a.B + kWave - 1) / kWave;
    auto kern = sc_fast_kernel<N, MASK, SPEC, GEN>;
    static bool attr = false;
    if (!attr) {
        NPD_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        attr = true;
    }
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, kWave * wpb, lds) != hipSuccess || occ <= 0) {
        (void)hipGetLastError();
        occ = 1;
    }
    const int64_t groups = (a.ntiles * a.n_seg + wpb - 1) / wpb;
    const int grid = grid_for(groups, occ, device_cu_count());
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kWave * wpb), lds, s, p, a);
    return launch_check("sc_fast_kernel launch");
}

}  // namespace scf

// (N, frozen mask) of the specialised codes: PolarCode 'polar' profile (run_models.py:630-639), K = N/2
#define NPD_SPEC_CODES(X) X(64, 0x1013f037f7fff) X(32, 0x117177f) X(16, 0x17f) X(8, 0x17)

// tile order (Args::ilv).  Streaming decode: interleaved -- adjacent 16 KiB tiles on different XCDs
// measured 0.408 -> 0.398 ms per 5 x 2^20 (membench, same geometry: 5.24 -> 5.57 TB/s); the VALU-bound
// fused Monte-Carlo kernel is 1 % faster with a workgroup's waves on adjacent tiles.  NPD_SCF_ILV=0/1
// overrides both (A/B).
// The switches are read per call (a getenv per launch), so a test can run both sides in one process.
static uint32_t tile_interleave(bool gen) {
    const char* e = getenv("NPD_SCF_ILV");
    const int v = (e && *e) ? (e[0] == '1' ? 1 : 0) : -1;
    return v >= 0 ? (uint32_t)v : (gen ? 0u : 1u);
}

static bool spec_disabled() {
    const char* e = getenv("NPD_SC_NOSPEC");
    return e && e[0] == '1';
}

// eligible: Polar, 8 <= N <= 64, K <= 128 (one Philox block of message bits), y 16-B aligned
bool sc_fast_eligible(const CodeParams& p, const void* y) {
    return !p.pac && p.N >= 8 && p.N <= 64 && p.K <= 128 && (((uintptr_t)y) & 15) == 0;
}

// fused Monte-Carlo sweep: same eligibility as the decode path minus the y pointer
int sc_fast_run_gen(const CodeParams& p, const float* sigma, const float* llr_scale, int n_seg, uint32_t snr_index0,
                    float* msg, unsigned long long* counters, uint64_t seed, uint64_t cw_offset, int64_t B,
                    hipStream_t s) {
    if (n_seg < 1 || n_seg > scf::kMaxSeg) return fail(NPD_EINVAL, "sc_mc_sweep_fused: 1 <= segments <= 16");
    if (p.pac || p.N < 8 || p.N > 64 || p.K > 128)
        return fail(NPD_ENOTSUP, "sc_mc_sweep_fused: Polar codes with 8 <= N <= 64 (use npd_mc_generate + "
                                 "npd_sc_decode_mc otherwise)");
    scf::Args a{};
    a.y = nullptr;
    a.msg = msg;
    a.counters = counters;
    a.seed = seed;
    a.cw_offset = cw_offset;
    a.B = B;
    a.n_seg = n_seg;
    a.snr_index0 = snr_index0;
    for (int i = 0; i < n_seg; ++i) {
        a.scale[i] = llr_scale[i];
        a.sigma[i] = sigma[i];
    }
    a.count = counters ? 1u : 0u;
    a.ilv = tile_interleave(true);
    if (!spec_disabled()) {
        uint64_t m = 0;
        for (int i = 0; i < p.N; ++i)
            if ((p.frozen[i >> 5] >> (i & 31)) & 1u) m |= 1ull << i;
#define NPD_SPEC(NN, MM) \
        if (p.N == NN && m == MM##ull) return scf::launch<NN, MM##ull, true, true>(p, a, s);
        NPD_SPEC_CODES(NPD_SPEC)
#undef NPD_SPEC
    }
    switch (p.N) {
        case 8: return scf::launch<8, 0, false, true>(p, a, s);
        case 16: return scf::launch<16, 0, false, true>(p, a, s);
        case 32: return scf::launch<32, 0, false, true>(p, a, s);
        default: return scf::launch<64, 0, false, true>(p, a, s);
    }
}

int sc_fast_run(const CodeParams& p, const float* y, const float* llr_scale, int n_seg, float* msg,
                unsigned long long* counters, uint64_t seed, uint64_t cw_offset, int64_t B, hipStream_t s) {
    if (n_seg < 1 || n_seg > scf::kMaxSeg) return fail(NPD_EINVAL, "sc_fast: 1 <= segments <= 16");
    scf::Args a{};
    a.y = y;
    a.msg = msg;
    a.counters = counters;
    a.seed = seed;
    a.cw_offset = cw_offset;
    a.B = B;
    a.n_seg = n_seg;
    for (int i = 0; i < n_seg; ++i) a.scale[i] = llr_scale[i];
    a.count = counters ? 1u : 0u;
    a.ilv = tile_interleave(false);
    // the reference's standard codes ('polar' rate profile, K = N/2) have specialised decoders
    if (!spec_disabled() && p.N <= 64) {
        uint64_t m = 0;
        for (int i = 0; i < p.N; ++i)
            if ((p.frozen[i >> 5] >> (i & 31)) & 1u) m |= 1ull << i;
#define NPD_SPEC(NN, MM) \
        if (p.N == NN && m == MM##ull) return scf::launch<NN, MM##ull, true>(p, a, s);
        NPD_SPEC_CODES(NPD_SPEC)
#undef NPD_SPEC
    }
    switch (p.N) {
        case 8: return scf::launch<8>(p, a, s);
        case 16: return scf::launch<16>(p, a, s);
        case 32: return scf::launch<32>(p, a, s);
        case 64: return scf::launch<64>(p, a, s);
        default: return fail(NPD_EINVAL, "sc_fast: unsupported N");
    }
}

}  // namespace npd
