// npd_sc.hip -- successive-cancellation min-sum decoding (Polar and PAC) for gfx950.
//
// Replaces PolarCode.sc_decode_new (polar.py:361-484) and PAC.pac_sc_decode (pac_code.py:233-345,
// 534-573).  The reference re-walks the code tree for every leaf with torch.cat/clone on (B, n+1, N)
// arrays; here one lane owns one codeword and runs the whole SC schedule fully unrolled at compile
// time, so every LLR and partial sum lives at a fixed register (or LDS row) address.
//
// Data path per wave (64 codewords = one "tile"):
//   HBM y tile (64 x N fp32, contiguous) --global_load_lds_dwordx4, 1 KiB per instruction,
//   XOR-swizzled chunk order--> LDS staging --ds_read_b128, conflict-free--> VGPRs (LLR levels with
//   node size <= R) / LDS rows (levels with node size > R) --> decisions written per leaf into an
//   LDS row (stride N+1 floats, conflict-free) --> coalesced dword stores of msg_hat / leaf / u_hat.
//
// Arithmetic is exactly the reference's fp32 sequence:
//   L = fl32(llr_scale * y);  f(a,b) = min(|a|,|b|)*sign(a)*sign(b) (utils.py:272-275) -- computed as
//   min(|a|,|b|) with the xor of the sign bits (identical value, +-0 aside);  g = u*a + b (u in
//   {-1,0,1}, so the product is exact and fma == mul+add);  leaf = L + prior (polar.py:438, 446);
//   u = sign(leaf) (polar.py:479).  Partial sums of finished R-blocks are kept as sign/zero bit masks.
#include <stdlib.h>

#include "npd_common.hpp"

#ifndef NPD_SC_WPE
#define NPD_SC_WPE 2  // waves per SIMD requested for the register-resident (N <= 64) kernels
#endif
#ifndef NPD_SC_STAGE_ROOT
#define NPD_SC_STAGE_ROOT 1  // N = 128: root level through a coalesced 8 KB LDS stage (0: per-lane row reads)
#endif

namespace npd {
namespace sc {

enum Flags : uint32_t {
    kLeaf = 1u << 0,   // write leaf LLRs (B,N)
    kMsg = 1u << 1,    // write msg_hat (B,K)
    kUhat = 1u << 2,   // write u_hat (B,N) (PAC)
    kGt = 1u << 3,     // genie decisions from gt (B,N)
    kCount = 1u << 4,  // count errors against the Philox message stream
};

constexpr int kMaxSeg = 16;  // SNR points of one fused Monte-Carlo sweep launch
constexpr int kRootModeDefault = 1;  // Spec::root of the streaming PAC(128,64) RM decode (measured best)

struct Args {
    const float* y;
    float* leaf;
    float* msg;
    float* uhat;
    const float* gt;
    unsigned long long* counters;
    uint64_t seed;
    uint64_t cw_offset;
    int64_t B;
    int64_t ntiles;
    float scale;
    uint32_t flags;
    // byte offsets inside the dynamic LDS block of the (single-wave) workgroup
    uint32_t off_stage, off_u, off_v, off_leaf, off_gt, off_info, off_lvl;
    // segments: n_seg runs of B codewords decoded back to back (msg_hat and counters per segment).  GEN
    // (fused Monte-Carlo sweep, npd_sc_mc_sweep_fused): segment s is generated in registers at seg_sigma[s] on
    // noise stream kStreamNoise + snr_index0 + s and decoded with seg_scale[s]; y is not read.
    int n_seg;
    uint32_t snr_index0;
    float seg_scale[kMaxSeg];
    float seg_sigma[kMaxSeg];
};

// ------------------------------------------------------------------------------ small helpers
// The reference rounds L = fl32(scale*y) before any add (polar.py:468).  hipcc contracts fmul+fadd
// into fma by default, even for __fmul_rn; an empty asm makes the rounded product opaque.
__device__ __forceinline__ float rmul(float a, float b) {
    float r = a * b;
    asm("" : "+v"(r));
    return r;
}

// sign(a) sign(b) min(|a|, |b|) in two VALU ops: med3(|a|, -|a|, b) = clamp(b, -|a|, |a|) has the magnitude
// min(|a|, |b|) and the sign of b; xor in the sign of a (v_med3_f32 + v_bitop3_b32).  Equal in value to the
// reference's product form (a zero may differ only in its sign bit, which no later step reads).
__device__ __forceinline__ float f_minsum(float a, float b) {
    const float m = __builtin_amdgcn_fmed3f(__builtin_fabsf(a), -__builtin_fabsf(a), b);
    return bitsf(__builtin_amdgcn_bitop3_b32(fbits(m), fbits(a), 0x80000000u, 0x78));  // m ^ (a & 0x80000000)
}

// fl32(s * v) for 4 values in two packed multiplies (each product rounded, never contracted: see rmul)
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float4 rmul4(float s, float4 v) {
    f2v lo = {v.x, v.y}, hi = {v.z, v.w};
    const f2v ss = {s, s};
    lo = lo * ss;
    hi = hi * ss;
    asm("" : "+v"(lo), "+v"(hi));
    return make_float4(lo.x, lo.y, hi.x, hi.y);
}

// sign(x) in {-1, 0, +1} (torch.sign): copy the sign bit onto 1.0, 0 for +-0
__device__ __forceinline__ float sgn_bits(float x) {
    const float s = bitsf((fbits(x) & 0x80000000u) | 0x3f800000u);
    return (x == 0.0f) ? 0.0f : s;
}

// g with the left partial sum given as sign/zero bits of one position
__device__ __forceinline__ float g_bits(uint32_t sw, uint32_t zw, int bit, float a, float b) {
    const float s = bitsf(fbits(a) ^ ((sw << (31 - bit)) & 0x80000000u)) + b;
    return ((zw >> bit) & 1u) ? b : s;
}

template <int C>
__device__ __forceinline__ int swz(int r) {
    if constexpr (C >= 16) return r & 15;
    else return (r / (16 / C)) % C;
}

template <int N>
struct Geo {
    static constexpr int C = N / 4;             // 16-B chunks per row
    static constexpr int NP = N + 1;            // padded row stride (floats) for per-lane float rows
    static constexpr int NB = 4 * ((N / 4) | 1);  // byte-row stride: an odd number of dwords (conflict-free)
};

// ------------------------------------------------------------------------------ frozen set
// NoSpec: the frozen set is read at run time (CodeParams).  Spec<M0, M1>: known at compile time (the
// reference's standard PAC(128,64) 'RM' profile) -- every frozen test is static, and in msg-only PAC decoding
// a rate-0 subtree needs no LLRs at all: its decisions are the convolution's output for v = +1
// (pac_code.py:545-551), whatever the channel says, so the f/g steps feeding it are skipped.
struct NoSpec {
    static constexpr bool on = false;
    static constexpr int root = 0;
    static constexpr bool frozen(int) { return false; }
    static constexpr bool rate0(int, int) { return false; }
    static constexpr int slot(int) { return 0; }
};
// ROOT (msg-only N = 128 decode, see RootStage): 0 = root level through the LDS stage at each root step (the
// g step re-reads y; 2 waves per SIMD), 1 = the whole row staged once and held in registers (1 wave per SIMD)
template <uint64_t M0, uint64_t M1, int ROOT = 0>
struct Spec {
    static constexpr bool on = true;
    static constexpr int root = ROOT;
    static constexpr bool frozen(int i) { return (((i < 64) ? (M0 >> i) : (M1 >> (i - 64))) & 1ull) != 0; }
    static constexpr bool rate0(int s0, int len) {
        for (int i = s0; i < s0 + len; ++i)
            if (!frozen(i)) return false;
        return true;
    }
    static constexpr int slot(int i) {  // message slot of information position i
        int k = 0;
        for (int t = 0; t < i; ++t) k += frozen(t) ? 0 : 1;
        return k;
    }
};
// PAC(128,64), 'RM' rate profile (popcount(i) < 4 frozen; pac_code.py:121-174)
using SpecPacRm128 = Spec<0x117177f177f7fffull, 0x101170117177full>;
template <int ROOT>
using SpecPacRm128R = Spec<0x117177f177f7fffull, 0x101170117177full, ROOT>;

// N = 128 streaming decode: the root level reaches the lanes through LDS-DMA (coalesced 1 KiB instructions)
// instead of per-lane row reads (64 cache-line lookups per instruction: PMC TA busy 0.57, TD busy 0.70).
//   on:    32-column chunks through one or two 8 KB slots at each root step (dma_chunk / root_pass); the g step
//          reads y again (L2 misses: 2x the y bytes cross the fabric), 2 waves per SIMD
//   regs:  (Spec::root == 1, msg-only PAC on a compile-time frozen set) the whole 32 KB tile is staged once and
//          the row held in 128 VGPRs across the left subtree (1 wave per SIMD, LDS 34 KB per wave), the next
//          tile's DMA landing meanwhile: y crosses once (PMC: 805.7 MB per 2^20 words = algorithmic)
//   vbits: the v decisions kept as sign / zero bit words in registers instead of LDS rows
template <int N, int R, bool PAC, bool FULL, class SP, bool GEN>
struct RootStage {
    static constexpr bool on = NPD_SC_STAGE_ROOT && !GEN && R < N && N == 128;
    static constexpr bool vbits = on && PAC && !FULL && SP::on;  // v decisions as sign / zero bit words
    static constexpr int slots = vbits ? 2 : 1;
    static constexpr bool regs = SP::root == 1 && vbits;  // whole tile staged, row held in registers
    static constexpr uint32_t kSlot = 64u * 32u * 4u;
    static constexpr uint32_t kBytes = regs ? 64u * N * 4u : (on ? kSlot * slots : 0u);
};

// ------------------------------------------------------------------------------ per-lane context
template <int N, int R, bool PAC, bool FULL, class SP, bool GEN>
struct Ctx {
    static constexpr int NW = (N + 31) / 32;
    float lv[2 * R];      // register LLR levels: level d (2^d <= R) at lv[2^d .. 2^(d+1))
    float beta[R];        // partial sums of the current R-block
    uint32_t S[NW], Z[NW];  // sign / zero bits of partial sums of completed R-blocks (N > R only)
    uint32_t st;          // PAC conv state (bit t = 1 iff state[t] == -1)
    int k;                // information leaves decided so far = slot of the next msg decision (v for PAC)
    uint32_t fz[NW];      // frozen-set words, re-read per tile (see the tile loop)
    // LDS row bases (bytes) of this lane
    char* lds;
    uint32_t stage_row;   // staging chunk base for this lane's row (chunk index r*C)
    int sw;               // this lane's swizzle
    uint32_t u_row, v_row;            // decision rows (int8 per position, stride NB bytes)
    uint32_t leaf_row, gt_row;        // float rows (R == N only; stride N+1 floats)
    float* leaf_g;                    // R < N: this lane's leaf-LLR output row in HBM (or null)
    const float* gt_g;                // R < N: this lane's genie row in HBM (or null)
    uint32_t lvl_row[9];  // per-level LDS rows for upper levels (node size > R, < N)
    float scale;
    uint32_t flags;
    const float4* yrow;   // N > R: this lane's received word in HBM (the root level is read from it directly)
    int64_t row0;         // kStageRoot: this tile's first row
    // GEN: this lane's codeword bits (bit i set iff x_i = -1) and its noise stream
    uint32_t U[NW];
    uint32_t VS[NW], VZ[NW];  // RootStage::vbits: v decisions by message slot, sign / zero bits
    float4 yr[(N + 3) / 4];   // RootStage::regs: this lane's received word
    uint64_t gseed, gcw;
    uint32_t gstream;
    float gsigma;
};

// GEN: chunk q (elements 4q .. 4q+3) of this lane's received word, value for value what npd_mc_generate writes
// (npd_gen.hip): Philox noise block (cw, q) -> 4 Box-Muller normals -> y = x + fl32(sigma z)
template <int N, int R, bool PAC, bool FULL, class SP, bool GEN>
__device__ __forceinline__ float4 gen_chunk(const Ctx<N, R, PAC, FULL, SP, GEN>& c, uint64_t cw, int q) {
    const u32x4 o = philox_block(c.gseed, c.gstream, cw, (uint32_t)q);
    float z[4];
    normals4(o, z);
    const uint32_t bits = (c.U[(4 * q) >> 5] >> ((4 * q) & 31)) & 0xFu;
    float4 y;
    y.x = __fadd_rn((bits & 1u) ? -1.0f : 1.0f, __fmul_rn(c.gsigma, z[0]));
    y.y = __fadd_rn((bits & 2u) ? -1.0f : 1.0f, __fmul_rn(c.gsigma, z[1]));
    y.z = __fadd_rn((bits & 4u) ? -1.0f : 1.0f, __fmul_rn(c.gsigma, z[2]));
    y.w = __fadd_rn((bits & 8u) ? -1.0f : 1.0f, __fmul_rn(c.gsigma, z[3]));
    return y;
}

// GEN: message bits (Philox message block(s) of the codeword) -> v at the information positions -> PAC
// convolution -> Plotkin transform, all on bit words (npd_gen.hip mc_generate_kernel, same bits)
template <int N, int R, bool PAC, bool FULL, class SP, bool GEN>
__device__ __forceinline__ void gen_codeword(Ctx<N, R, PAC, FULL, SP, GEN>& c, const CodeParams& p) {
    constexpr int NW = Ctx<N, R, PAC, FULL, SP, GEN>::NW;
    constexpr int MB = (N + 127) / 128;
    uint32_t m[4 * MB];
#pragma unroll
    for (int blk = 0; blk < MB; ++blk) {
        if (blk * 128 < p.K) {
            const u32x4 o = philox_block(c.gseed, kStreamMsg, c.gcw, (uint32_t)blk);
            m[4 * blk + 0] = o.x; m[4 * blk + 1] = o.y; m[4 * blk + 2] = o.z; m[4 * blk + 3] = o.w;
        } else {
            m[4 * blk + 0] = m[4 * blk + 1] = m[4 * blk + 2] = m[4 * blk + 3] = 0u;
        }
    }
#pragma unroll
    for (int w = 0; w < NW; ++w) c.U[w] = 0u;
    // scatter: the k-th information position (ascending) takes message bit k; the current message word is
    // consumed by shifting (no run-time indexing into m), the next one selected every 32 bits
    uint32_t cur = m[0];
    int kk = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const bool frozen = SP::on ? SP::frozen(i) : (((c.fz[i >> 5] >> (i & 31)) & 1u) != 0);
        if (!frozen) {
            c.U[i >> 5] |= (cur & 1u) << (i & 31);
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
    if constexpr (PAC) {
        // u_i = v_i xor parity(state & taps), state bit t = v_{i-1-t} (pac_code.py:181-208): u = v xor the
        // shifts of v by t + 1 for every tap t, on the whole bit vector (zeros shifted in = the +1 start state)
        uint32_t v[NW];
#pragma unroll
        for (int w = 0; w < NW; ++w) v[w] = c.U[w];
        uint32_t taps = p.tapmask;
        asm volatile("" : "+s"(taps));
        for (int t = 0; t < 31; ++t) {
            if (!((taps >> t) & 1u)) continue;
            const int sh = t + 1;
#pragma unroll
            for (int w = NW - 1; w >= 0; --w) {
                const uint32_t lo = (w > 0) ? (v[w - 1] >> (32 - sh)) : 0u;
                c.U[w] ^= (v[w] << sh) | (sh < 32 ? lo : 0u);
            }
        }
    }
#pragma unroll
    for (int h = 1; h < 32 && h < N; h <<= 1) {
        uint32_t msk = 0;
        for (int i = 0; i < 32; ++i)
            if (((i / h) & 1) == 0) msk |= 1u << i;
#pragma unroll
        for (int w = 0; w < NW; ++w) c.U[w] ^= (c.U[w] >> h) & msk;
    }
#pragma unroll
    for (int hw = 1; hw < NW; hw <<= 1)
#pragma unroll
        for (int w = 0; w < NW; ++w)
            if (((w / hw) & 1) == 0) c.U[w] ^= c.U[w + hw];
}

template <int N>
__device__ __forceinline__ float4 stage_chunk(char* lds, uint32_t off_stage, uint32_t row_chunk, int sw, int c) {
    const uint32_t addr = off_stage + ((row_chunk + (uint32_t)(c ^ sw)) << 4);
    return *reinterpret_cast<const float4*>(lds + addr);
}

__device__ __forceinline__ void lds_wr(char* lds, uint32_t byte, float v) { *reinterpret_cast<float*>(lds + byte) = v; }
__device__ __forceinline__ float lds_rd(const char* lds, uint32_t byte) { return *reinterpret_cast<const float*>(lds + byte); }
__device__ __forceinline__ void lds_wr8(char* lds, uint32_t byte, float v) {
    *reinterpret_cast<int8_t*>(lds + byte) = (int8_t)(int)v;  // v in {-1, 0, 1}
}
__device__ __forceinline__ float lds_rd8(const char* lds, uint32_t byte) {
    return (float)*reinterpret_cast<const int8_t*>(lds + byte);
}

// ------------------------------------------------------------------------------ leaf
template <int N, int R, bool PAC, bool FULL, class SP, bool GEN, int I>
__device__ __forceinline__ void write_leaf(Ctx<N, R, PAC, FULL, SP, GEN>& c, float v) {
    if constexpr (FULL) {
        if (c.flags & kLeaf) {
            if constexpr (R == N) lds_wr(c.lds, c.leaf_row + 4 * I, v);
            else c.leaf_g[I] = v;
        }
    }
}

template <int N, int R, bool PAC, bool FULL, class SP, bool GEN, int I>
__device__ __forceinline__ float genie(const Ctx<N, R, PAC, FULL, SP, GEN>& c) {
    if constexpr (R == N) return lds_rd(c.lds, c.gt_row + 4 * I);
    else return c.gt_g[I];
}

template <int N, int R, bool PAC, bool FULL, class SP, bool GEN, int I>
__device__ __forceinline__ void leaf(Ctx<N, R, PAC, FULL, SP, GEN>& c, const CodeParams& p, const Args& a, float L) {
    const bool frozen = SP::on ? SP::frozen(I) : (((c.fz[I >> 5] >> (I & 31)) & 1u) != 0);
    const bool use_gt = FULL && (c.flags & kGt);
    float u;
    if constexpr (!PAC) {
        // polar.py:438/446: leaf = L + prior; prior = infty on frozen positions, 0 elsewhere
        const float lf = L + (frozen ? p.infty : 0.0f);
        write_leaf<N, R, PAC, FULL, SP, GEN, I>(c, lf);
        u = use_gt ? genie<N, R, PAC, FULL, SP, GEN, I>(c) : sgn_bits(lf);
    } else if constexpr (!FULL) {
        // msg-only PAC leaf on integer bits: conv(+1) = (-1)^parity(st & taps) (pac_code.py:188-193); a frozen
        // leaf decides it (pac_code.py:545-551); an information leaf decides u = sign(L) and v = +1 when u equals
        // conv(+1), -1 when it is the opposite, 0 when L = 0 (state unchanged) (pac_code.py:553-568) -- so v's
        // sign is sign(L) xor the parity, and no float compares are needed
        // (the state word is not masked to the register length here: only its bits under the taps are read)
        const uint32_t cnt = (uint32_t)__builtin_popcount(c.st & p.tapmask);
        if (frozen) {
            u = bitsf(0x3f800000u | (cnt << 31));
            c.st = c.st << 1;
        } else {
            const uint32_t Lb = fbits(L);
            const bool nz = (Lb << 1) != 0u;
            const uint32_t negb = ((Lb >> 31) ^ cnt) & 1u;
            u = nz ? bitsf((Lb & 0x80000000u) | 0x3f800000u) : 0.0f;
            const uint32_t sh = (c.st << 1) | negb;
            c.st = nz ? sh : c.st;
            if constexpr (RootStage<N, R, PAC, FULL, SP, GEN>::vbits) {
                // bits folded in at the leaf (opaque words: the 64 decisions do not stay live to the tile end)
                constexpr int k = SP::slot(I);
                c.VS[k >> 5] |= negb << (k & 31);
                c.VZ[k >> 5] |= (nz ? 0u : 1u) << (k & 31);
                asm volatile("" : "+v"(c.VS[k >> 5]), "+v"(c.VZ[k >> 5]));
            } else {
                lds_wr8(c.lds, c.v_row + (uint32_t)c.k, nz ? (negb ? -1.0f : 1.0f) : 0.0f);
            }
            ++c.k;
        }
    } else {
        write_leaf<N, R, PAC, FULL, SP, GEN, I>(c, L);
        const float u0 = (__builtin_popcount(c.st & p.tapmask) & 1) ? -1.0f : 1.0f;  // conv(+1) (pac_code.py:188-193)
        float v;
        if (frozen) {  // pac_code.py:545-551
            v = 1.0f;
            if (use_gt) {
                u = genie<N, R, PAC, FULL, SP, GEN, I>(c);
            } else {
                u = u0;
                c.st = (c.st << 1) & p.smask;
            }
        } else {  // pac_code.py:553-568, branch-free: u == u0 -> v = 1, u == -u0 -> v = -1, u == 0 -> v = 0
            u = use_gt ? genie<N, R, PAC, FULL, SP, GEN, I>(c) : sgn_bits(L);
            const bool eq = (u == u0), neg = (u == -u0);
            v = eq ? 1.0f : (neg ? -1.0f : 0.0f);
            const uint32_t sh = ((c.st << 1) | (neg ? 1u : 0u)) & p.smask;
            c.st = (eq || neg) ? sh : c.st;
        }
        // v is read at information positions only (msg_hat, counts): stored in slot (message) order, so
        // msg_hat leaves as 16-B rows
        if (!frozen) {
            lds_wr8(c.lds, c.v_row + (uint32_t)c.k, v);
            ++c.k;
        }
    }
    // PAC: u rows by position feed u_hat (FULL only).  Polar: the u decisions of information positions
    // feed only msg_hat and the counts -> slot (message) order, like PAC's v rows
    if constexpr (PAC) {
        if (FULL) lds_wr8(c.lds, c.u_row + I, u);
    } else if (!frozen) {
        lds_wr8(c.lds, c.u_row + (uint32_t)c.k, u);
        ++c.k;
    }
    c.beta[I % R] = u;
}

// ------------------------------------------------------------------------------ register levels
// node at depth D (2^D <= R) covering absolute leaves [S0, S0 + 2^D); its LLRs at lv[2^D ..]
template <int N, int R, bool PAC, bool FULL, class SP, bool GEN, int D, int S0>
__device__ __forceinline__ void node_reg(Ctx<N, R, PAC, FULL, SP, GEN>& c, const CodeParams& p, const Args& a) {
    if constexpr (D == 0) {
        leaf<N, R, PAC, FULL, SP, GEN, S0>(c, p, a, c.lv[1]);
    } else {
        constexpr int h = 1 << (D - 1);
        constexpr int bs = S0 % R;  // local beta base
        // a child whose leaves are all frozen needs no LLRs (msg-only PAC with a static frozen set)
        constexpr bool skipL = SP::on && PAC && !FULL && SP::rate0(S0, h);
        constexpr bool skipR = SP::on && PAC && !FULL && SP::rate0(S0 + h, h);
        if constexpr (!skipL) {
#pragma unroll
            for (int j = 0; j < h; ++j) c.lv[h + j] = f_minsum(c.lv[2 * h + j], c.lv[3 * h + j]);
        }
        node_reg<N, R, PAC, FULL, SP, GEN, D - 1, S0>(c, p, a);
        if constexpr (!skipR) {
#pragma unroll
            for (int j = 0; j < h; ++j) c.lv[h + j] = c.beta[bs + j] * c.lv[2 * h + j] + c.lv[3 * h + j];
        }
        node_reg<N, R, PAC, FULL, SP, GEN, D - 1, S0 + h>(c, p, a);
        if constexpr ((1 << D) < N) {  // the root's combined partial sums are never used
#pragma unroll
            for (int j = 0; j < h; ++j) c.beta[bs + j] = c.beta[bs + j] * c.beta[bs + h + j];
        }
    }
}

// pack the float partial sums of a finished R-block starting at absolute position S0 into bits
template <int N, int R, bool PAC, bool FULL, class SP, bool GEN, int S0>
__device__ __forceinline__ void pack_block(Ctx<N, R, PAC, FULL, SP, GEN>& c) {
#pragma unroll
    for (int j = 0; j < R; ++j) {
        const int pos = S0 + j;
        // b in {+-1, +-0}: sign = bit 31, zero = NOT exponent bit 23 (1.0f = 0x3f800000).  Integer ops,
        // no compares: compares make 64-bit lane masks that the scheduler parks in VGPR lanes.  A -0's
        // sign bit is harmless: g_bits returns b outright when the zero bit is set.
        const uint32_t bb = fbits(c.beta[j]);
        const uint32_t sb = bb >> 31;
        const uint32_t zb = (~bb >> 23) & 1u;
        if ((pos & 31) == 0) {
            c.S[pos >> 5] = sb;
            c.Z[pos >> 5] = zb;
        } else {
            c.S[pos >> 5] |= sb << (pos & 31);
            c.Z[pos >> 5] |= zb << (pos & 31);
        }
    }
}

// ------------------------------------------------------------------------------ upper levels
// value j of the level-D LLR vector of the current node (D = n: staging input scaled; else LDS row)
template <int N, int R, bool PAC, bool FULL, class SP, bool GEN, int D>
__device__ __forceinline__ float up_get(const Ctx<N, R, PAC, FULL, SP, GEN>& c, const Args& a, int j) {
    (void)a;
    if constexpr ((1 << D) == N) {
        // staging: element j of the row is in chunk j/4, sub j%4
        const uint32_t addr = a.off_stage + ((c.stage_row + (uint32_t)((j >> 2) ^ c.sw)) << 4) + 4 * (j & 3);
        return rmul(c.scale, lds_rd(c.lds, addr));
    } else {
        return lds_rd(c.lds, c.lvl_row[D] + 4 * j);
    }
}

template <int N, int R, bool PAC, bool FULL, class SP, bool GEN, int D>
__device__ __forceinline__ void up_put(Ctx<N, R, PAC, FULL, SP, GEN>& c, int j, float v) {
    if constexpr ((1 << D) == R) c.lv[R + j] = v;
    else lds_wr(c.lds, c.lvl_row[D] + 4 * j, v);
}

// ------------------------------------------------------------------------------ tile staging
// the 64 x N fp32 y tile starting at row0 -> LDS staging buffer: C x 1 KiB global_load_lds (asynchronous;
// consumers wait with s_waitcnt vmcnt(0)), swizzled source addresses
template <int N>
__device__ __forceinline__ void stage_tile(char* lds, const Args& a, int64_t row0, int lane) {
    constexpr int C = N / 4;
#pragma unroll
    for (int k = 0; k < C; ++k) {
        const int pch = k * kWave + lane;
        const int r = pch / C;
        const int q = pch % C;
        const int cc = q ^ swz<C>(r);
        int64_t grow = row0 + r;
        if (grow >= a.B) grow = a.B - 1;
        const float* src = a.y + grow * N + cc * 4;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)(lds + a.off_stage + k * 1024), 16, 0, 0);
    }
}

// N = 128 streaming decode: the root level reaches the lanes through an LDS stage per wave instead of per-lane
// row reads.  A per-lane 16-B read of 64 different rows costs the texture path 64 cache-line lookups per
// instruction (PMC, per-lane version: TA busy 0.57 and TD busy 0.70 of the kernel, mostly stalled on the L1);
// one 1 KiB LDS-DMA here covers 8 whole 128-B lines.  A root step (f or g) walks 4 chunks of 32 columns: A0
// A1 (first half of the row) and B0 B1 (second half).  Chunk slots of 8 KB: one slot (A0 arrives prefetched,
// B0 A1 B1 in turn) or, with the v decisions kept as bits in registers (msg-only PAC on a compile-time frozen
// set: the LDS then holds no decision rows), two slots (A0 B0 prefetched, A1 B1 fetched together).

// LDS-DMA of columns col0 .. col0+31 of rows row0 .. row0+63 into the slot at byte `base`: 64 rows x 8 chunks of
// 16 B, chunk (r, q) at slot r*8 + q holding source chunk q ^ swz<8>(r) (stage_tile's swizzle: the row-per-lane
// ds_read_b128 is conflict-free).  Asynchronous; read_slot waits.
template <int N>
__device__ __forceinline__ void dma_chunk(char* lds, uint32_t base, const Args& a, int64_t row0, int col0, int lane) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every lane's reads of the slot are done
    // opaque per call, so the 8 row addresses are not kept live between the calls of a tile
    asm volatile("" : "+s"(row0));
    // a buffer descriptor over the tile's rows (wave-uniform): 32-bit offsets, and rows past B read as zeros
    // (tail lanes decode them; their results are neither counted nor stored)
    const int64_t nrows = (a.B - row0) < kWave ? (a.B - row0) : kWave;
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)(a.y + row0 * N), 0, (int)(nrows * N * 4), 0x00020000);
    // row r = 8k + lane/8, chunk (lane & 7) ^ swz<8>(r) = (lane & 7) ^ (lane >> 4) ^ 4 (k & 1)
    const int c0 = (lane & 7) ^ (lane >> 4);
    const uint32_t v0 = (uint32_t)(((lane >> 3) * N + col0 + (c0 << 2)) * 4);
    const uint32_t v1 = (uint32_t)(((lane >> 3) * N + col0 + ((c0 ^ 4) << 2)) * 4);
#pragma unroll
    for (int k = 0; k < 8; ++k)
        // the row offset goes in voffset, not soffset: the descriptor's range check covers voffset + the
        // immediate only, so rows past B must be addressed through voffset to read as zeros
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)(lds + base + k * 1024), 16,
                                                 ((k & 1) ? v1 : v0) + (uint32_t)(8 * k * N * 4), 0, 0, 0);
}

// this lane's 32 values of the slot at `base` (waits for every outstanding DMA)
__device__ __forceinline__ void read_slot(const char* lds, uint32_t base, int lane, float4 (&v)[8]) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int sw = swz<8>(lane);
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = *reinterpret_cast<const float4*>(lds + base + ((uint32_t)(lane * 8 + (q ^ sw)) << 4));
}

// one root step: emit(j0, A, B) gets this lane's columns j0 .. j0+31 of both halves of its row.  Chunk 0 (and
// with two slots B0) is in the stage; afterwards the same for rows pf_row0 is prefetched (pf_row0 < 0: none)
template <int N, int SLOTS, class Emit>
__device__ __forceinline__ void root_pass(char* lds, const Args& a, int64_t row0, int64_t pf_row0, int lane, Emit&& emit) {
    constexpr uint32_t kSlot = 64u * 32u * 4u;
    const uint32_t s0 = a.off_stage, s1 = a.off_stage + (SLOTS == 2 ? kSlot : 0u);
    float4 A[8], B[8];
    if constexpr (SLOTS == 2) {
        read_slot(lds, s0, lane, A);
        read_slot(lds, s1, lane, B);
        dma_chunk<N>(lds, s0, a, row0, 32, lane);
        dma_chunk<N>(lds, s1, a, row0, 96, lane);
        emit(0, A, B);
        __builtin_amdgcn_sched_barrier(0);  // emit(0) before the next reads: A0 B0 and A1 B1 never live together
        read_slot(lds, s0, lane, A);
        read_slot(lds, s1, lane, B);
        if (pf_row0 >= 0) {
            dma_chunk<N>(lds, s0, a, pf_row0, 0, lane);
            dma_chunk<N>(lds, s1, a, pf_row0, 64, lane);
        }
    } else {
        read_slot(lds, s0, lane, A);
        dma_chunk<N>(lds, s0, a, row0, 64, lane);
        read_slot(lds, s0, lane, B);
        dma_chunk<N>(lds, s0, a, row0, 32, lane);
        emit(0, A, B);
        __builtin_amdgcn_sched_barrier(0);
        read_slot(lds, s0, lane, A);
        dma_chunk<N>(lds, s0, a, row0, 96, lane);
        read_slot(lds, s0, lane, B);
        if (pf_row0 >= 0) dma_chunk<N>(lds, s0, a, pf_row0, 0, lane);
    }
    emit(32, A, B);
}

// g at the root for position pos of the left half.  N = 2R: the left half is one register block whose combined
// partial sums are still in c.beta (nothing has overwritten them yet), so g = u a + b as in the register levels
// (u in {-1, 0, 1}: the product is exact, one rounding); otherwise from the packed sign / zero bits.
template <int N, int R, bool PAC, bool FULL, class SP, bool GEN>
__device__ __forceinline__ float root_g(const Ctx<N, R, PAC, FULL, SP, GEN>& c, int pos, float a, float b) {
    if constexpr (N == 2 * R) return c.beta[pos] * a + b;
    else return g_bits(c.S[pos >> 5], c.Z[pos >> 5], pos & 31, a, b);
}

// RootStage::regs: the whole 64 x N tile by LDS-DMA through a buffer descriptor (32-bit offsets; rows past B
// read as zeros), in stage_tile's swizzled layout (chunk (r, q) at slot r*C + q holds source chunk q ^ swz<C>(r))
template <int N>
__device__ __forceinline__ void stage_tile_buf(char* lds, const Args& a, int64_t row0, int lane) {
    constexpr int C = N / 4;
    static_assert(C == 32, "N = 128");
    asm volatile("" : "+s"(row0));
    const int64_t nrows = (a.B - row0) < kWave ? (a.B - row0) : kWave;
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)(a.y + row0 * N), 0, (int)(nrows * N * 4), 0x00020000);
    // instruction k: rows 2k + lane/32, chunk (lane & 31) ^ swz<32>(r), swz<32>(r) = r & 15 = 2 (k & 7) + lane/32
    const int hi = lane >> 5;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        const uint32_t vo = (uint32_t)((hi * N + 4 * ((lane & 31) ^ (2 * (k & 7) + hi))) * 4);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)(lds + a.off_stage + k * 1024), 16,
                                                 vo + (uint32_t)(2 * k * N * 4), 0, 0, 0);  // range-checked (dma_chunk)
    }
}

template <int N, int R, bool PAC, bool FULL, class SP, bool GEN, int D, int S0>
__device__ __forceinline__ void node_up(Ctx<N, R, PAC, FULL, SP, GEN>& c, const CodeParams& p, const Args& a) {
    if constexpr ((1 << D) == R) {
        node_reg<N, R, PAC, FULL, SP, GEN, D, S0>(c, p, a);
        // the packed bits feed g steps above the register levels other than the root's (N = 2R: root_g reads
        // c.beta, and no level lies between)
        if constexpr (N > 2 * R) pack_block<N, R, PAC, FULL, SP, GEN, S0>(c);
    } else {
        constexpr int h = 1 << (D - 1);
        if constexpr ((1 << D) == N && RootStage<N, R, PAC, FULL, SP, GEN>::regs) {
#pragma unroll
            for (int q = 0; q < h / 4; ++q) {
                const float4 A = c.yr[q], Bv = c.yr[q + h / 4];  // scaled at the tile start
                up_put<N, R, PAC, FULL, SP, GEN, D - 1>(c, 4 * q + 0, f_minsum(A.x, Bv.x));
                up_put<N, R, PAC, FULL, SP, GEN, D - 1>(c, 4 * q + 1, f_minsum(A.y, Bv.y));
                up_put<N, R, PAC, FULL, SP, GEN, D - 1>(c, 4 * q + 2, f_minsum(A.z, Bv.z));
                up_put<N, R, PAC, FULL, SP, GEN, D - 1>(c, 4 * q + 3, f_minsum(A.w, Bv.w));
            }
        } else if constexpr ((1 << D) == N && RootStage<N, R, PAC, FULL, SP, GEN>::on) {
            using RS = RootStage<N, R, PAC, FULL, SP, GEN>;
            root_pass<N, RS::slots>(c.lds, a, c.row0, c.row0, threadIdx.x, [&](int j0, const float4 (&A)[8], const float4 (&Bv)[8]) {
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int j = j0 + 4 * q;
                    const float4 As = rmul4(c.scale, A[q]), Bs = rmul4(c.scale, Bv[q]);
                    up_put<N, R, PAC, FULL, SP, GEN, D - 1>(c, j + 0, f_minsum(As.x, Bs.x));
                    up_put<N, R, PAC, FULL, SP, GEN, D - 1>(c, j + 1, f_minsum(As.y, Bs.y));
                    up_put<N, R, PAC, FULL, SP, GEN, D - 1>(c, j + 2, f_minsum(As.z, Bs.z));
                    up_put<N, R, PAC, FULL, SP, GEN, D - 1>(c, j + 3, f_minsum(As.w, Bs.w));
                }
            });  // then this tile's first chunk(s) again, for the g step
        } else if constexpr ((1 << D) == N) {
            // the root level straight from this lane's row in HBM (16-B loads), or generated (GEN)
#pragma unroll
            for (int q = 0; q < h / 4; ++q) {
                const float4 A = GEN ? gen_chunk(c, c.gcw, q) : c.yrow[q];
                const float4 Bv = GEN ? gen_chunk(c, c.gcw, q + h / 4) : c.yrow[q + h / 4];
                up_put<N, R, PAC, FULL, SP, GEN, D - 1>(c, 4 * q + 0, f_minsum(rmul(c.scale, A.x), rmul(c.scale, Bv.x)));
                up_put<N, R, PAC, FULL, SP, GEN, D - 1>(c, 4 * q + 1, f_minsum(rmul(c.scale, A.y), rmul(c.scale, Bv.y)));
                up_put<N, R, PAC, FULL, SP, GEN, D - 1>(c, 4 * q + 2, f_minsum(rmul(c.scale, A.z), rmul(c.scale, Bv.z)));
                up_put<N, R, PAC, FULL, SP, GEN, D - 1>(c, 4 * q + 3, f_minsum(rmul(c.scale, A.w), rmul(c.scale, Bv.w)));
            }
        } else {
#pragma unroll
            for (int j = 0; j < h; ++j)
                up_put<N, R, PAC, FULL, SP, GEN, D - 1>(c, j, f_minsum(up_get<N, R, PAC, FULL, SP, GEN, D>(c, a, j), up_get<N, R, PAC, FULL, SP, GEN, D>(c, a, j + h)));
        }
        node_up<N, R, PAC, FULL, SP, GEN, D - 1, S0>(c, p, a);
        if constexpr ((1 << D) == N && RootStage<N, R, PAC, FULL, SP, GEN>::regs) {
#pragma unroll
            for (int q = 0; q < h / 4; ++q) {
                const float4 As = c.yr[q], Bs = c.yr[q + h / 4];
                const float av[4] = {As.x, As.y, As.z, As.w};
                const float bv[4] = {Bs.x, Bs.y, Bs.z, Bs.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int pos = S0 + 4 * q + e;
                    up_put<N, R, PAC, FULL, SP, GEN, D - 1>(c, 4 * q + e, root_g(c, pos, av[e], bv[e]));
                }
            }
        } else if constexpr ((1 << D) == N && RootStage<N, R, PAC, FULL, SP, GEN>::on) {
            using RS = RootStage<N, R, PAC, FULL, SP, GEN>;
            const int64_t nrow0 = c.row0 + (int64_t)gridDim.x * kWave;  // grid-stride successor tile
            root_pass<N, RS::slots>(c.lds, a, c.row0, nrow0 < a.B ? nrow0 : -1, threadIdx.x,
                                    [&](int j0, const float4 (&A)[8], const float4 (&Bv)[8]) {
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const float4 As = rmul4(c.scale, A[q]), Bs = rmul4(c.scale, Bv[q]);
                    const float av[4] = {As.x, As.y, As.z, As.w};
                    const float bv[4] = {Bs.x, Bs.y, Bs.z, Bs.w};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int j = j0 + 4 * q + e;
                        const int pos = S0 + j;
                        up_put<N, R, PAC, FULL, SP, GEN, D - 1>(c, j, root_g(c, pos, av[e], bv[e]));
                    }
                }
            });
        } else if constexpr ((1 << D) == N) {
            // second read of the row (L2 / MALL).  The pointer is laundered through an empty asm so the
            // compiler cannot forward the f step's loads: keeping those N values live across the left
            // half would cost N VGPRs (N = 128: 384 instead of ~250 -> one wave per SIMD instead of two)
            // (GEN: generated again, from a laundered codeword index so the f step's values are not kept live)
            const float4* yr = c.yrow;
            asm volatile("" : "+v"(yr));
            uint64_t cw2 = c.gcw;
            if constexpr (GEN) asm volatile("" : "+v"(cw2));
#pragma unroll
            for (int q = 0; q < h / 4; ++q) {
                const float4 A = GEN ? gen_chunk(c, cw2, q) : yr[q];
                const float4 Bv = GEN ? gen_chunk(c, cw2, q + h / 4) : yr[q + h / 4];
                const float av[4] = {A.x, A.y, A.z, A.w};
                const float bv[4] = {Bv.x, Bv.y, Bv.z, Bv.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int pos = S0 + 4 * q + e;
                    up_put<N, R, PAC, FULL, SP, GEN, D - 1>(c, 4 * q + e,
                                             root_g(c, pos, rmul(c.scale, av[e]), rmul(c.scale, bv[e])));
                }
            }
        } else {
#pragma unroll
            for (int j = 0; j < h; ++j) {
                const int pos = S0 + j;
                up_put<N, R, PAC, FULL, SP, GEN, D - 1>(c, j, g_bits(c.S[pos >> 5], c.Z[pos >> 5], pos & 31, up_get<N, R, PAC, FULL, SP, GEN, D>(c, a, j),
                                                      up_get<N, R, PAC, FULL, SP, GEN, D>(c, a, j + h)));
            }
        }
        node_up<N, R, PAC, FULL, SP, GEN, D - 1, S0 + h>(c, p, a);
        if constexpr ((1 << D) < N) {
            // combine bit partial sums: left *= right  (h >= 64: whole words)
#pragma unroll
            for (int w = 0; w < h / 32; ++w) {
                c.S[(S0 >> 5) + w] ^= c.S[((S0 + h) >> 5) + w];
                c.Z[(S0 >> 5) + w] |= c.Z[((S0 + h) >> 5) + w];
            }
        }
    }
}

template <int N>
constexpr int log2c() {
    int n = 0;
    while ((1 << n) < N) ++n;
    return n;
}

// ------------------------------------------------------------------------------ output pass
// store W floats per row for the tile's `rows` valid rows: value(r, col) = lds[base + r*stride + 4*map(col)]
template <bool BYTES>
__device__ __forceinline__ void store_rows(const char* lds, uint32_t base, uint32_t stride_b, const int32_t* info_lds,
                                           int W, float* out, int64_t tile_row0, int rows, int lane) {
    if (out == nullptr || W == 0) return;
    float* dst = out + tile_row0 * (int64_t)W;
    const int total = rows * W;
    int r = lane / W, col = lane % W;
    const int dr = kWave / W, dc = kWave % W;
    for (int e = lane; e < total; e += kWave) {
        const int m = info_lds ? info_lds[col] : col;
        if constexpr (BYTES) dst[e] = lds_rd8(lds, base + (uint32_t)r * stride_b + (uint32_t)m);
        else dst[e] = lds_rd(lds, base + (uint32_t)r * stride_b + 4u * (uint32_t)m);
        r += dr;
        col += dc;
        if (col >= W) {
            col -= W;
            ++r;
        }
    }
}

// K int8 decisions per row in slot order -> fp32 msg_hat rows with 16-B stores (K % 4 == 0, 16-B aligned
// output): one ds_read_b32 of 4 slots per float4
__device__ __forceinline__ void store_slots(const char* lds, uint32_t base, uint32_t stride_b, int K, float* out,
                                            int64_t tile_row0, int rows, int lane) {
    const int K4 = K >> 2;
    float4* dst = reinterpret_cast<float4*>(out + tile_row0 * (int64_t)K);
    int r = lane / K4, c4 = lane - (lane / K4) * K4;  // stepped incrementally (no division per element)
    const int dr = kWave / K4, dc = kWave - (kWave / K4) * K4;
    for (int e = lane; e < rows * K4; e += kWave) {
        const uint32_t w = *reinterpret_cast<const uint32_t*>(lds + base + (uint32_t)r * stride_b + 4u * (uint32_t)c4);
        float4 v;
        v.x = (float)(int8_t)(w & 0xffu);
        v.y = (float)(int8_t)((w >> 8) & 0xffu);
        v.z = (float)(int8_t)((w >> 16) & 0xffu);
        v.w = (float)(int8_t)(w >> 24);
        dst[e] = v;
        r += dr;
        c4 += dc;
        if (c4 >= K4) {
            c4 -= K4;
            ++r;
        }
    }
}

// v decisions held as sign / zero bit words per lane (RootStage::vbits) -> fp32 msg_hat rows: the words go
// through LDS (NW x 2 dwords per row at `base`) so the stores are coalesced, 16 B per lane when K % 4 == 0
template <int NW>
__device__ __forceinline__ void store_vbits(char* lds, uint32_t base, const uint32_t (&vs)[NW], const uint32_t (&vz)[NW],
                                            int K, bool vec, float* out, int64_t tile_row0, int rows, int lane) {
    constexpr uint32_t kRow = 2u * NW * 4u;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        *reinterpret_cast<uint32_t*>(lds + base + (uint32_t)lane * kRow + 4u * w) = vs[w];
        *reinterpret_cast<uint32_t*>(lds + base + (uint32_t)lane * kRow + 4u * (NW + w)) = vz[w];
    }
    if (vec) {
        const int K4 = K >> 2;
        float4* dst = reinterpret_cast<float4*>(out + tile_row0 * (int64_t)K);
        // (row, column) of element e stepped incrementally: one division per tile, not per element
        int r = lane / K4, c4 = lane - (lane / K4) * K4;
        const int dr = kWave / K4, dc = kWave - (kWave / K4) * K4;
        for (int e = lane; e < rows * K4; e += kWave) {
            const int s = 4 * c4;
            const uint32_t row = base + (uint32_t)r * kRow;
            const uint32_t sb = *reinterpret_cast<const uint32_t*>(lds + row + 4u * (uint32_t)(s >> 5)) >> (s & 31);
            const uint32_t zb = *reinterpret_cast<const uint32_t*>(lds + row + 4u * (uint32_t)(NW + (s >> 5))) >> (s & 31);
            float4 v;
            v.x = (zb & 1u) ? 0.0f : ((sb & 1u) ? -1.0f : 1.0f);
            v.y = (zb & 2u) ? 0.0f : ((sb & 2u) ? -1.0f : 1.0f);
            v.z = (zb & 4u) ? 0.0f : ((sb & 4u) ? -1.0f : 1.0f);
            v.w = (zb & 8u) ? 0.0f : ((sb & 8u) ? -1.0f : 1.0f);
            dst[e] = v;
            r += dr;
            c4 += dc;
            if (c4 >= K4) {
                c4 -= K4;
                ++r;
            }
        }
    } else {
        float* dst = out + tile_row0 * (int64_t)K;
        for (int e = lane; e < rows * K; e += kWave) {
            const int r = e / K, s = e - r * K;
            const uint32_t row = base + (uint32_t)r * kRow;
            const uint32_t sb = *reinterpret_cast<const uint32_t*>(lds + row + 4u * (uint32_t)(s >> 5)) >> (s & 31);
            const uint32_t zb = *reinterpret_cast<const uint32_t*>(lds + row + 4u * (uint32_t)(NW + (s >> 5))) >> (s & 31);
            dst[e] = (zb & 1u) ? 0.0f : ((sb & 1u) ? -1.0f : 1.0f);
        }
    }
}

// ------------------------------------------------------------------------------ kernel
// <= 256 VGPRs so two waves share each SIMD (N = 256 is LDS-bound at 3 waves per CU anyway)
template <int N, int R, bool PAC, bool FULL, class SP, bool GEN>
__global__ __launch_bounds__(64, SP::root == 1 ? 1 : NPD_SC_WPE) void sc_decode_kernel(const CodeParams p, const Args a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    constexpr int n = log2c<N>();
    constexpr int C = Geo<N>::C;
    constexpr int NP = Geo<N>::NP;
    const int lane = threadIdx.x;

    Ctx<N, R, PAC, FULL, SP, GEN> c;
    c.lds = lds;
    c.scale = a.scale;
    c.flags = a.flags;
    c.sw = swz<C>(lane);
    c.stage_row = (uint32_t)(lane * C);
    constexpr int NB = Geo<N>::NB;
    c.u_row = a.off_u + (uint32_t)(lane * NB);
    c.v_row = a.off_v + (uint32_t)(lane * NB);
    c.leaf_row = a.off_leaf + (uint32_t)(lane * NP * 4);
    c.gt_row = a.off_gt + (uint32_t)(lane * NP * 4);
    c.leaf_g = nullptr;
    c.gt_g = nullptr;
    {
        uint32_t off = a.off_lvl;
#pragma unroll
        for (int d = 0; d < 9; ++d) {
            c.lvl_row[d] = 0;
            if ((1 << d) > R && (1 << d) < N) {
                c.lvl_row[d] = off + (uint32_t)(lane * ((1 << d) + 1) * 4);
                off += (uint32_t)(kWave * ((1 << d) + 1) * 4);
            }
        }
    }

    uint32_t err_bits = 0, err_blocks = 0;
    const bool count = (a.flags & kCount) != 0;
    const bool vec_msg = (p.K & 3) == 0 && (((uintptr_t)a.msg) & 15u) == 0;

    // tiles of all segments: g = seg * ntiles + t (one segment unless a sweep / GEN launch)
    const int64_t total = GEN ? a.ntiles * (int64_t)a.n_seg : a.ntiles;
    int cur_seg = 0;
    auto flush = [&](int sg) {
        const uint32_t eb = wave_sum_u32(err_bits);
        const uint32_t bl = wave_sum_u32(err_blocks);
        if (lane == 0 && (eb | bl)) {
            atomicAdd(a.counters + 2 * sg + 0, (unsigned long long)eb);
            atomicAdd(a.counters + 2 * sg + 1, (unsigned long long)bl);
        }
        err_bits = 0;
        err_blocks = 0;
    };
    using RS = RootStage<N, R, PAC, FULL, SP, GEN>;
    constexpr bool kStageRoot = RS::on;
    if constexpr (RS::regs) {  // the first tile (whole)
        if (blockIdx.x < total) stage_tile_buf<N>(lds, a, (int64_t)blockIdx.x * kWave, lane);
    } else if constexpr (kStageRoot) {  // the first tile's prefetched chunk(s)
        if (blockIdx.x < total) {
            dma_chunk<N>(lds, a.off_stage, a, (int64_t)blockIdx.x * kWave, 0, lane);
            if (RS::slots == 2) dma_chunk<N>(lds, a.off_stage + RS::kSlot, a, (int64_t)blockIdx.x * kWave, 64, lane);
        }
    }
    for (int64_t g = blockIdx.x; g < total; g += gridDim.x) {
        const int seg = GEN ? (int)(g / a.ntiles) : 0;
        const int64_t t = GEN ? g - (int64_t)seg * a.ntiles : g;
        const int64_t row0 = t * kWave;
        const int rows = (int)((a.B - row0) < kWave ? (a.B - row0) : kWave);
        if (GEN && count && seg != cur_seg) {
            flush(cur_seg);
            cur_seg = seg;
        }
        if constexpr (GEN) {
            c.scale = a.seg_scale[seg];
            c.gsigma = a.seg_sigma[seg];
            c.gstream = kStreamNoise + a.snr_index0 + (uint32_t)seg;
            c.gseed = a.seed;
            // tail lanes decode a duplicate of the last codeword (not counted), as the streaming path does
            c.gcw = a.cw_offset + (uint64_t)((row0 + lane) < a.B ? row0 + lane : a.B - 1);
        }

        // ---- N <= R: stage the y tile through LDS (coalesced, transposed to row-per-lane).  N > R: each
        // lane reads the root level of its own row straight from HBM at the root's f and g steps (no LDS
        // stage: the LDS then holds only decision rows, so occupancy is register-bound)
        if constexpr (GEN) {
        } else if constexpr (R == N) {
            stage_tile<N>(lds, a, row0, lane);
        } else if constexpr (RS::regs) {
            // the staged tile -> this lane's row in registers, then the next tile's DMA into the stage
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
            for (int q = 0; q < N / 4; ++q) c.yr[q] = stage_chunk<N>(lds, a.off_stage, c.stage_row, c.sw, q);
            // scaled once: the f and g steps both read fl32(scale * y)
#pragma unroll
            for (int q = 0; q < N / 4; ++q) c.yr[q] = rmul4(c.scale, c.yr[q]);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (row0 + (int64_t)gridDim.x * kWave < a.B) stage_tile_buf<N>(lds, a, row0 + (int64_t)gridDim.x * kWave, lane);
        } else if constexpr (kStageRoot) {
            c.row0 = row0;
        } else {
            const int64_t grow = (row0 + lane) < a.B ? row0 + lane : a.B - 1;
            c.yrow = reinterpret_cast<const float4*>(a.y + grow * N);
        }
        if constexpr (FULL && R < N) {
            int64_t grow = row0 + lane;
            if (grow >= a.B) grow = a.B - 1;
            c.gt_g = a.gt ? a.gt + grow * N : nullptr;
            // tail lanes decode a duplicate of the last row; their leaf writes go to a scratch-free
            // duplicate row only when in range
            c.leaf_g = (a.leaf && lane < rows) ? a.leaf + (row0 + lane) * N : nullptr;
            if (a.leaf && lane >= rows) c.flags &= ~kLeaf;
            else if (a.leaf) c.flags |= kLeaf;
        }
        if (FULL && R == N && (a.flags & kGt)) {
            for (int e = lane; e < kWave * N; e += kWave) {
                const int r = e / N, col = e % N;
                int64_t grow = row0 + r;
                if (grow >= a.B) grow = a.B - 1;
                lds_wr(lds, a.off_gt + (uint32_t)((r * NP + col) * 4), a.gt[grow * N + col]);
            }
        }
        if constexpr (!kStageRoot) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

        c.st = 0;
        c.k = 0;
        if constexpr (RS::vbits) {
#pragma unroll
            for (int w = 0; w < Ctx<N, R, PAC, FULL, SP, GEN>::NW; ++w) c.VS[w] = c.VZ[w] = 0u;
        }
        // The frozen words are loop-invariant, so LICM would hoist all N per-leaf frozen tests out of the
        // tile loop as 64-bit lane masks and spill them into VGPR lanes (two v_readlane per leaf, plus
        // scratch); an opaque per-tile copy keeps each test next to its leaf (one s_bitcmp).
#pragma unroll
        for (int w = 0; w < Ctx<N, R, PAC, FULL, SP, GEN>::NW; ++w) {
            c.fz[w] = p.frozen[w];
            asm volatile("" : "+s"(c.fz[w]));
        }
        if constexpr (GEN) gen_codeword(c, p);
        if constexpr (R == N) {
            // whole row into registers (GEN: generated in registers)
#pragma unroll
            for (int q = 0; q < C; ++q) {
                const float4 v = GEN ? gen_chunk(c, c.gcw, q) : stage_chunk<N>(lds, a.off_stage, c.stage_row, c.sw, q);
                c.lv[N + 4 * q + 0] = rmul(c.scale, v.x);
                c.lv[N + 4 * q + 1] = rmul(c.scale, v.y);
                c.lv[N + 4 * q + 2] = rmul(c.scale, v.z);
                c.lv[N + 4 * q + 3] = rmul(c.scale, v.w);
            }
            node_reg<N, R, PAC, FULL, SP, GEN, n, 0>(c, p, a);
        } else {
            node_up<N, R, PAC, FULL, SP, GEN, n, 0>(c, p, a);
        }

        // ---- error counting against the Philox message stream (utils.py:17-51 semantics)
        if (count) {
            const uint64_t cw = a.cw_offset + (uint64_t)(row0 + lane);
            const uint32_t dec_row = PAC ? c.v_row : c.u_row;
            uint32_t e = 0;
#pragma unroll
            for (int blk = 0; blk < (N + 127) / 128; ++blk) {
                if (blk * 128 < p.K) {
                    const u32x4 o = philox_block(a.seed, kStreamMsg, cw, (uint32_t)blk);
                    const uint32_t w4[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
                    for (int w = 0; w < 4; ++w) {
                        const int k0 = blk * 128 + w * 32;
                        const int kn = (p.K - k0) < 32 ? (p.K - k0) : 32;
                        const uint32_t bits = w4[w];
                        if constexpr (RS::vbits) {
                            // a slot counts if its sign differs from the message bit (bit 1 = -1) or it is 0
                            if (kn > 0) {
                                const uint32_t m = kn >= 32 ? 0xFFFFFFFFu : ((1u << kn) - 1u);
                                e += (uint32_t)__builtin_popcount(((c.VS[(k0 >> 5) & (Ctx<N, R, PAC, FULL, SP, GEN>::NW - 1)] ^ bits) |
                                                                   c.VZ[(k0 >> 5) & (Ctx<N, R, PAC, FULL, SP, GEN>::NW - 1)]) & m);
                            }
                        } else {
                            // slot-ordered decision bytes, 4 per dword, against the message nibbles: +1 ->
                            // 0x01, -1 -> 0xFF; a byte counts if it differs (0 decisions always do)
                            for (int q = 0; q < kn; q += 4) {
                                const uint32_t dw = *reinterpret_cast<const uint32_t*>(lds + dec_row + (uint32_t)(k0 + q));
                                const uint32_t nib = (bits >> q) & 0xFu;
                                const uint32_t x = (nib * 0x00204081u) & 0x01010101u;  // bit i -> byte i
                                const uint32_t expect = 0x01010101u | ((x << 8) - x);
                                const int valid = kn - q;
                                const uint32_t vmask = valid >= 4 ? 0xFFFFFFFFu : ((1u << (8 * valid)) - 1u);
                                const uint32_t d = (dw ^ expect) & vmask;
                                const uint32_t tb = ((d & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d;
                                e += (uint32_t)__builtin_popcount(tb & 0x80808080u);
                            }
                        }
                    }
                }
            }
            if (lane < rows) {
                err_bits += e;
                err_blocks += (e > 0) ? 1u : 0u;
            }
        }

        // ---- coalesced output stores
        if (RS::vbits && (a.flags & kMsg)) {
            store_vbits<Ctx<N, R, PAC, FULL, SP, GEN>::NW>(lds, a.off_v, c.VS, c.VZ, p.K, vec_msg, a.msg, row0, rows, lane);
        } else if (a.flags & kMsg) {
            const uint32_t slots = PAC ? a.off_v : a.off_u;  // decisions in message order
            float* msg = GEN ? a.msg + (int64_t)seg * a.B * p.K : a.msg;
            if (vec_msg)
                store_slots(lds, slots, NB, p.K, msg, row0, rows, lane);
            else
                store_rows<true>(lds, slots, NB, nullptr, p.K, msg, row0, rows, lane);
        }
        if constexpr (FULL && R == N) {
            if (a.flags & kLeaf) store_rows<false>(lds, a.off_leaf, NP * 4, nullptr, N, a.leaf, row0, rows, lane);
        }
        if (FULL && (a.flags & kUhat)) store_rows<true>(lds, a.off_u, NB, nullptr, N, a.uhat, row0, rows, lane);
    }

    if (count) flush(cur_seg);
}

// ------------------------------------------------------------------------------ host side
struct Layout {
    uint32_t off_stage, off_u, off_v, off_leaf, off_gt, off_info, off_lvl, total;
};

static uint32_t align16(uint32_t x) { return (x + 15u) & ~15u; }

template <int N, int R, class RS>
static Layout make_layout(bool pac, uint32_t flags) {
    Layout L{};
    const uint32_t stage = (uint32_t)(kWave * N * 4);
    const uint32_t frow = (uint32_t)(kWave * (N + 1) * 4);   // float rows
    const uint32_t brow = (uint32_t)(kWave * Geo<N>::NB);    // int8 decision rows
    uint32_t off = 0;
    L.off_stage = 0;
    const bool full = (flags & (kLeaf | kGt | kUhat)) != 0;
    if (R == N && !full) {
        // the staged tile is fully read into registers before the first leaf: decision rows alias it
        L.off_leaf = 0;
        L.off_gt = 0;
        L.off_u = 0;
        off = align16(stage > brow ? stage : brow);
        L.off_v = pac ? off : 0;
        if (pac) off = align16(off + brow);
        L.off_lvl = off;
        L.off_info = off;  // (no info table: decisions are kept in slot order)
        L.total = off;
        return L;
    }
    if (R == N) {
        // leaf-LLR rows alias the staging buffer (read into registers before the first leaf)
        L.off_leaf = 0;
        off = align16((flags & kLeaf) && frow > stage ? frow : stage);
        L.off_gt = (flags & kGt) ? off : 0;
        if (flags & kGt) off = align16(off + frow);
    } else {
        // no y tile stage: the root level is read from HBM per lane, or (N = 128) through an 8 KB chunk stage
        off = RS::kBytes;
        L.off_leaf = 0;  // leaf LLRs and genie rows go straight to/from HBM
        L.off_gt = 0;
    }
    L.off_u = off;
    if (!pac || full) off = align16(off + brow);  // msg-only PAC keeps no u rows (its decisions are the v rows)
    L.off_v = pac ? off : 0;
    if (pac) off = align16(off + (RS::vbits ? (uint32_t)(kWave * 2 * 4 * ((N + 31) / 32)) : brow));
    L.off_lvl = off;
    for (int d = 0; d < 9; ++d)
        if ((1 << d) > R && (1 << d) < N) off += (uint32_t)(kWave * ((1 << d) + 1) * 4);
    off = align16(off);
    L.off_info = off;
    L.total = off;
    return L;
}

template <int N, int R, bool PAC, bool FULL, class SP, bool GEN>
static int launch_t(const CodeParams& p, Args a, hipStream_t stream) {
    const Layout L = make_layout<N, R, RootStage<N, R, PAC, FULL, SP, GEN>>(PAC, a.flags);
    a.off_stage = L.off_stage;
    a.off_u = L.off_u;
    a.off_v = L.off_v;
    a.off_leaf = L.off_leaf;
    a.off_gt = L.off_gt;
    a.off_info = L.off_info;
    a.off_lvl = L.off_lvl;
    a.ntiles = (a.B + kWave - 1) / kWave;
    if (!GEN || a.n_seg < 1) a.n_seg = 1;  // streaming launches decode one segment (y is one (B, N) block)
    auto kern = sc_decode_kernel<N, R, PAC, FULL, SP, GEN>;
    static bool attr_set[2] = {false, false};  // per instantiation; benign race (idempotent)
    if (!attr_set[0] && L.total > 65536) {
        NPD_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
        attr_set[0] = true;
    }
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, kWave, L.total) != hipSuccess || occ <= 0) {
        (void)hipGetLastError();
        occ = 1;
    }
    const int grid = grid_for(a.ntiles * a.n_seg, occ, device_cu_count());
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kWave), L.total, stream, p, a);
    return launch_check("sc_decode_kernel launch");
}

template <bool PAC, bool FULL, bool GEN = false>
static int dispatch(const CodeParams& p, const Args& a, hipStream_t s) {
    switch (p.N) {
        case 4: return launch_t<4, 4, PAC, FULL, NoSpec, GEN>(p, a, s);
        case 8: return launch_t<8, 8, PAC, FULL, NoSpec, GEN>(p, a, s);
        case 16: return launch_t<16, 16, PAC, FULL, NoSpec, GEN>(p, a, s);
        case 32: return launch_t<32, 32, PAC, FULL, NoSpec, GEN>(p, a, s);
        case 64: return launch_t<64, 64, PAC, FULL, NoSpec, GEN>(p, a, s);
        case 128: return launch_t<128, 64, PAC, FULL, NoSpec, GEN>(p, a, s);
        case 256: return launch_t<256, 64, PAC, FULL, NoSpec, GEN>(p, a, s);
        default: return fail(NPD_EINVAL, "sc_decode: unsupported N");
    }
}

static int root_mode() {  // NPD_SC_ROOT=0/1: root-level mode of the msg-only PAC(128,64) RM kernel (A/B); per call
    const char* e = getenv("NPD_SC_ROOT");
    return (e && (e[0] == '0' || e[0] == '1')) ? e[0] - '0' : kRootModeDefault;
}

static bool spec_off() {  // NPD_SC_NOSPEC=1: generic frozen set everywhere (testing / A-B); read per call
    const char* e = getenv("NPD_SC_NOSPEC");
    return e && e[0] == '1';
}

static bool is_frozen_set(const CodeParams& p, uint64_t m0, uint64_t m1) {
    for (int i = 0; i < p.N; ++i) {
        const bool f = ((p.frozen[i >> 5] >> (i & 31)) & 1u) != 0;
        const bool g = (((i < 64) ? (m0 >> i) : (m1 >> (i - 64))) & 1ull) != 0;
        if (f != g) return false;
    }
    return true;
}

static int run(const npd_code* code, Args a, hipStream_t s) {
    if (a.B == 0) return NPD_OK;
    const bool full = (a.flags & (kLeaf | kGt | kUhat)) != 0;
    if (code->p.pac && !full && code->p.N == 128 && !spec_off() && is_frozen_set(code->p, 0x117177f177f7fffull, 0x101170117177full))
        switch (root_mode()) {
            case 1: return launch_t<128, 64, true, false, SpecPacRm128R<1>, false>(code->p, a, s);
            default: return launch_t<128, 64, true, false, SpecPacRm128, false>(code->p, a, s);
        }
    if (code->p.pac) return full ? dispatch<true, true>(code->p, a, s) : dispatch<true, false>(code->p, a, s);
    return full ? dispatch<false, true>(code->p, a, s) : dispatch<false, false>(code->p, a, s);
}

// fused Monte-Carlo sweep for every code the fast kernel does not take (PAC, Polar N >= 128, N = 4):
// generation in registers, SC decode, counts (and msg_hat) per SNR segment, one launch
static int gen_run(const npd_code* code, const float* sigma, const float* llr_scale, int n_seg, uint32_t snr_index0,
                   float* msg, unsigned long long* counters, uint64_t seed, uint64_t cw_offset, int64_t B, hipStream_t s) {
    Args a{};
    a.msg = msg;
    a.counters = counters;
    a.seed = seed;
    a.cw_offset = cw_offset;
    a.B = B;
    a.n_seg = n_seg;
    a.snr_index0 = snr_index0;
    for (int i = 0; i < n_seg; ++i) {
        a.seg_scale[i] = llr_scale[i];
        a.seg_sigma[i] = sigma[i];
    }
    a.flags = (counters ? kCount : 0u) | (msg ? kMsg : 0u);
    if (code->p.pac && code->p.N == 128 && !spec_off() && is_frozen_set(code->p, 0x117177f177f7fffull, 0x101170117177full))
        return launch_t<128, 64, true, false, SpecPacRm128, true>(code->p, a, s);
    return code->p.pac ? dispatch<true, false, true>(code->p, a, s) : dispatch<false, false, true>(code->p, a, s);
}

}  // namespace sc
}  // namespace npd

using namespace npd;

namespace npd {
bool sc_fast_eligible(const CodeParams& p, const void* y);
int sc_fast_run(const CodeParams& p, const float* y, const float* llr_scale, int n_seg, float* msg,
                unsigned long long* counters, uint64_t seed, uint64_t cw_offset, int64_t B, hipStream_t s);
}  // namespace npd

static bool fast_disabled() {  // NPD_SC_GENERIC=1: force the generic kernel (testing / A-B); read per call
    const char* e = getenv("NPD_SC_GENERIC");
    return e && *e && *e != '0';
}

extern "C" int npd_sc_decode(const npd_code* code, const float* y, float llr_scale, float* leaf_llr, float* msg_hat,
                             float* u_hat, const float* gt, int64_t B, void* stream) {
    NPD_ARG(code != nullptr, "npd_sc_decode: code is NULL");
    NPD_ARG(B >= 0, "npd_sc_decode: B < 0");
    NPD_ARG(B == 0 || y != nullptr, "npd_sc_decode: y is NULL");
    NPD_ARG(code->p.pac || u_hat == nullptr, "npd_sc_decode: u_hat is only produced for PAC codes");
    NPD_ARG((((uintptr_t)y) & 15) == 0, "npd_sc_decode: y must be 16-byte aligned");
    sc::Args a{};
    a.y = y;
    a.leaf = leaf_llr;
    a.msg = msg_hat;
    a.uhat = u_hat;
    a.gt = gt;
    a.B = B;
    a.scale = llr_scale;
    a.flags = (leaf_llr ? sc::kLeaf : 0u) | (msg_hat ? sc::kMsg : 0u) | (u_hat ? sc::kUhat : 0u) | (gt ? sc::kGt : 0u);
    if (!leaf_llr && !u_hat && !gt && B > 0 && !fast_disabled() && sc_fast_eligible(code->p, y))
        return sc_fast_run(code->p, y, &llr_scale, 1, msg_hat, nullptr, 0, 0, B, (hipStream_t)stream);
    return sc::run(code, a, (hipStream_t)stream);
}

extern "C" int npd_sc_decode_mc(const npd_code* code, const float* y, float llr_scale, float* msg_hat, uint64_t seed,
                                uint64_t cw_offset, int64_t B, unsigned long long* counters, void* stream) {
    NPD_ARG(code != nullptr, "npd_sc_decode_mc: code is NULL");
    NPD_ARG(B >= 0, "npd_sc_decode_mc: B < 0");
    NPD_ARG(B == 0 || y != nullptr, "npd_sc_decode_mc: y is NULL");
    NPD_ARG(counters != nullptr, "npd_sc_decode_mc: counters is NULL");
    NPD_ARG((((uintptr_t)y) & 15) == 0, "npd_sc_decode_mc: y must be 16-byte aligned");
    sc::Args a{};
    a.y = y;
    a.msg = msg_hat;
    a.counters = counters;
    a.seed = seed;
    a.cw_offset = cw_offset;
    a.B = B;
    a.scale = llr_scale;
    a.flags = sc::kCount | (msg_hat ? sc::kMsg : 0u);
    if (B > 0 && !fast_disabled() && sc_fast_eligible(code->p, y))
        return sc_fast_run(code->p, y, &llr_scale, 1, msg_hat, counters, seed, cw_offset, B, (hipStream_t)stream);
    return sc::run(code, a, (hipStream_t)stream);
}

extern "C" int npd_sc_decode_mc_sweep(const npd_code* code, int n_snr, const float* y, const float* llr_scale,
                                      float* msg_hat, uint64_t seed, uint64_t cw_offset, int64_t B,
                                      unsigned long long* counters, void* stream) {
    NPD_ARG(code != nullptr, "npd_sc_decode_mc_sweep: code is NULL");
    NPD_ARG(n_snr >= 1 && n_snr <= 16, "npd_sc_decode_mc_sweep: 1 <= n_snr <= 16");
    NPD_ARG(llr_scale != nullptr, "npd_sc_decode_mc_sweep: llr_scale is NULL");
    NPD_ARG(B >= 0, "npd_sc_decode_mc_sweep: B < 0");
    NPD_ARG(B == 0 || y != nullptr, "npd_sc_decode_mc_sweep: y is NULL");
    NPD_ARG(counters != nullptr, "npd_sc_decode_mc_sweep: counters is NULL");
    if (B == 0) return NPD_OK;
    if (!fast_disabled() && sc_fast_eligible(code->p, y))
        return sc_fast_run(code->p, y, llr_scale, n_snr, msg_hat, counters, seed, cw_offset, B, (hipStream_t)stream);
    const int N = code->p.N, K = code->p.K;
    for (int i = 0; i < n_snr; ++i) {
        const int rc = npd_sc_decode_mc(code, y + (int64_t)i * B * N, llr_scale[i],
                                        msg_hat ? msg_hat + (int64_t)i * B * K : nullptr, seed, cw_offset, B,
                                        counters + 2 * i, stream);
        if (rc) return rc;
    }
    return NPD_OK;
}

namespace npd {
int sc_fast_run_gen(const CodeParams& p, const float* sigma, const float* llr_scale, int n_seg, uint32_t snr_index0,
                    float* msg, unsigned long long* counters, uint64_t seed, uint64_t cw_offset, int64_t B,
                    hipStream_t s);
}

extern "C" int npd_sc_mc_sweep_fused(const npd_code* code, int n_snr, const float* sigma, const float* llr_scale,
                                     uint32_t snr_index0, uint64_t seed, uint64_t cw_offset, int64_t B, float* msg_hat,
                                     unsigned long long* counters, void* stream) {
    NPD_ARG(code != nullptr, "npd_sc_mc_sweep_fused: code is NULL");
    NPD_ARG(n_snr >= 1 && n_snr <= 16, "npd_sc_mc_sweep_fused: 1 <= n_snr <= 16");
    NPD_ARG(sigma != nullptr && llr_scale != nullptr, "npd_sc_mc_sweep_fused: sigma / llr_scale is NULL");
    NPD_ARG(B >= 0, "npd_sc_mc_sweep_fused: B < 0");
    NPD_ARG(counters != nullptr || msg_hat != nullptr, "npd_sc_mc_sweep_fused: no output");
    if (B == 0) return NPD_OK;
    const CodeParams& p = code->p;
    if (!p.pac && p.N >= 8 && p.N <= 64 && p.K <= 128 && !fast_disabled())
        return npd::sc_fast_run_gen(p, sigma, llr_scale, n_snr, snr_index0, msg_hat, counters, seed, cw_offset, B,
                                    (hipStream_t)stream);
    return sc::gen_run(code, sigma, llr_scale, n_snr, snr_index0, msg_hat, counters, seed, cw_offset, B,
                       (hipStream_t)stream);
}
