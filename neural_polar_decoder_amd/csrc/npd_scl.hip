// npd_scl.hip -- Polar SC-List decoding (PolarCode.scl_decode, polar.py:793-876, use_CRC=False).
//
// Layout: a list of L paths per codeword lives in G = pow2ceil(L) adjacent lanes, one path per lane,
// so 64/G codewords share a wave.  Every lane runs the same compile-time-unrolled min-sum SC schedule
// as npd_sc_fast.hip on its own path state (LLRs of each level and partial sums in VGPRs); the
// channel LLRs are identical for the whole group and never move.
//
// At an information leaf the group's 2s candidates (s = current list size) are, in the reference's
// list order, [keep_0 .. keep_{s-1}, flip_0 .. flip_{s-1}] with metrics m_j and fl32(m_j + |l_j|)
// (polar.py:830-843).  When 2s > L the survivors are torch.topk's choice (polar.py:777-791): if no
// metric tie straddles the L-th place the survivor set is unique and is found by rank counting (two
// ballots); otherwise the group runs the exact std::nth_element statement of npd_nth.hpp.  Survivors
// keep list order.  Lane j then takes its candidate's parent state through ds_bpermute -- only the
// values that are still live after this leaf (known at compile time from the leaf index), never the
// channel level.
//
// The final choice is the reference's ML step (polar.py:868-874): each path's codeword
// (encode_plotkin of its decisions, computed on sign/zero bit masks) is compared with y in fp32 and the
// first minimum wins.  The leaf LLRs of the chosen path (scl_decode's first output) equal a genie SC
// pass with gt = the chosen u_hat; the host wrapper runs npd_sc_decode for that when asked.
#include "npd_common.hpp"
#include "npd_nth.hpp"

namespace npd {
namespace scl {

struct Args {
    const float* y;
    float* msg;                    // (B,K) or null
    float* uhat;                   // (B,N) or null
    unsigned long long* counters;  // {bit errors, block errors} or null
    uint64_t seed;
    uint64_t cw_offset;
    int64_t B;
    int64_t ntiles;
    float scale;
    int L;
    uint32_t count;
};

typedef float f4 __attribute__((ext_vector_type(4)));

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

__device__ __forceinline__ float rmul(float a, float b) {
    float r = a * b;
    asm("" : "+v"(r));  // keep the product rounded (no fma contraction into a following add)
    return r;
}

__device__ __forceinline__ float f_minsum(float a, float b) {
    const float m = __builtin_fminf(__builtin_fabsf(a), __builtin_fabsf(b));
    return bitsf(fbits(m) | ((fbits(a) ^ fbits(b)) & 0x80000000u));
}

__device__ __forceinline__ float sgn_bits(float x) {
    const float s = bitsf((fbits(x) & 0x80000000u) | 0x3f800000u);
    return (x == 0.0f) ? 0.0f : s;
}

// value of lane (group base + T) for every lane of a G-lane group
template <int G, int T>
__device__ __forceinline__ float gb(float x, int src_lane) {
    if constexpr (G == 1) {
        return x;
    } else if constexpr (G == 2) {
        constexpr int ctl = T | (T << 2) | ((2 + T) << 4) | ((2 + T) << 6);
        return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), ctl, 0xF, 0xF, false));
    } else if constexpr (G == 4) {
        constexpr int ctl = T * 0x55;
        return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), ctl, 0xF, 0xF, false));
    } else {
        return __shfl(x, src_lane, 64);
    }
}

template <int N, int G>
struct Lane {
    static constexpr int W = (N + 31) / 32;
    float lv[2 * N];   // level d at lv[2^d .. 2^(d+1)); channel level at lv[N .. 2N)
    float beta[N];     // partial sums
    float m;           // path metric (polar.py:803)
    uint32_t sm[W];    // decision sign bits by position (u = -1)
    uint32_t zm[W];    // decision zero bits by position (u = 0, from sign(0))
    uint32_t fz[W];    // frozen bits (re-materialised per tile)
    int base;          // lane id of the group's first lane
    int j;             // index within the group (= list slot)
    uint32_t slot;     // wave-uniform: information bits decided so far
    int L;
};

// first position whose partial sum is still read after leaf I: the start of the highest ancestor that
// still needs its left block for a g-update, or that will combine partial sums (spine nodes skip it)
template <int N, int I>
constexpr int beta_live_start() {
    constexpr int n = log2c<N>();
    for (int D = n; D >= 1; --D) {
        const int S0 = (I >> D) << D;
        const int h = 1 << (D - 1);
        const bool inleft = (I - S0) < h;
        const bool spine = S0 + (1 << D) == N;
        if (inleft || !spine) return S0;
    }
    return I;
}

template <int N, int G, int I, int D>
__device__ __forceinline__ void copy_levels(Lane<N, G>& c, int src) {
    if constexpr (D >= 1) {
        if constexpr (((I >> (D - 1)) & 1) == 0) {  // I in the left child of its level-D ancestor: input live
#pragma unroll
            for (int k = (1 << D); k < (2 << D); ++k) c.lv[k] = __shfl(c.lv[k], src, 64);
        }
        copy_levels<N, G, I, D - 1>(c, src);
    }
}

template <int N, int G, int I>
__device__ __forceinline__ void copy_live(Lane<N, G>& c, int src) {
    constexpr int n = log2c<N>();
    copy_levels<N, G, I, n - 1>(c, src);
    constexpr int b0 = beta_live_start<N, I>();
#pragma unroll
    for (int k = b0; k < I; ++k) c.beta[k] = __shfl(c.beta[k], src, 64);
#pragma unroll
    for (int w = 0; w <= (I >> 5); ++w) {
        c.sm[w] = (uint32_t)__shfl((int)c.sm[w], src, 64);
        c.zm[w] = (uint32_t)__shfl((int)c.zm[w], src, 64);
    }
}

// survivors of pruneLists for one group when a metric tie straddles the L-th place (rare): exact rule
// km / fm arrive as 8-wide vectors (VGPRs): arrays passed by reference would live in scratch, stored at
// every information leaf whether or not the tie path is taken
typedef float f8v __attribute__((ext_vector_type(8)));
template <int G>
__device__ __noinline__ uint32_t exact_mask(f8v km, f8v fm, int s, int L) {
    float negm[16];
#pragma unroll
    for (int t = 0; t < G; ++t) {
        negm[t] = -1.0f * km[t];
        negm[G + t] = -1.0f * fm[t];
    }
    // list order is [keep_0..keep_{s-1}, flip_0..flip_{s-1}]: compact when s < G
    float v[16];
    for (int c2 = 0; c2 < s; ++c2) {
        v[c2] = negm[c2];
        v[s + c2] = negm[G + c2];
    }
    return nth::prune_mask(v, 2 * s, L);
}

// Surviving candidates of one group at an information leaf (pruneLists, polar.py:777-791), as a mask over
// the list order [keep_0 .. keep_{s-1}, flip_0 .. flip_{s-1}]; m = this lane's path metric, a = |LLR|.
template <int G>
__device__ __forceinline__ uint32_t list_select(float m, float a, int j, int bl, int s, int L) {
    if (2 * s <= L) return (1u << (2 * s)) - 1u;
    float km[G], fm[G];
    km[0] = gb<G, 0>(m, bl + 0);
    fm[0] = km[0] + gb<G, 0>(a, bl + 0);
    if constexpr (G > 1) {
        km[1] = gb<G, 1>(m, bl + 1);
        fm[1] = km[1] + gb<G, 1>(a, bl + 1);
    }
    if constexpr (G > 2) {
        km[2] = gb<G, 2>(m, bl + 2);
        fm[2] = km[2] + gb<G, 2>(a, bl + 2);
        km[3] = gb<G, 3>(m, bl + 3);
        fm[3] = km[3] + gb<G, 3>(a, bl + 3);
    }
    if constexpr (G > 4) {
#pragma unroll
        for (int t = 4; t < G; ++t) {
            km[t] = __shfl(m, bl + t, 64);
            fm[t] = km[t] + __shfl(a, bl + t, 64);
        }
    }
    const float vk = m, vf = m + a;
    int ltk = 0, lek = 0, ltf = 0, lef = 0;
#pragma unroll
    for (int t = 0; t < G; ++t) {
        if (t < s) {
            ltk += (km[t] < vk) + (fm[t] < vk);
            lek += (km[t] <= vk) + (fm[t] <= vk);
            ltf += (km[t] < vf) + (fm[t] < vf);
            lef += (km[t] <= vf) + (fm[t] <= vf);
        }
    }
    const bool act = j < s;
    const bool sk = act && ltk < L;
    const bool sf = act && ltf < L;
    const bool st = act && ((ltk < L && lek > L) || (ltf < L && lef > L));
    const unsigned long long bk = __ballot(sk), bf = __ballot(sf), bs = __ballot(st);
    const uint32_t lowm = (1u << s) - 1u;
    uint32_t msel = ((uint32_t)(bk >> bl) & lowm) | (((uint32_t)(bf >> bl) & lowm) << s);
    if (bs) {
        const bool mine = ((uint32_t)(bs >> bl) & ((G >= 32) ? 0xFFFFFFFFu : ((1u << G) - 1u))) != 0u;
        if (mine) {
            f8v kv = {}, fv = {};
#pragma unroll
            for (int t = 0; t < G; ++t) {
                kv[t] = km[t];
                fv[t] = fm[t];
            }
            msel = exact_mask<G>(kv, fv, s, L);
        }
    }
    return msel;
}

template <int N, int G, int I>
__device__ __forceinline__ void info_leaf(Lane<N, G>& c, float l, int lane) {
    const float a = __builtin_fabsf(l);
    const int L = c.L;
    const uint32_t slot = c.slot;
    const int s = slot >= 3u ? L : ((1 << slot) < L ? (1 << slot) : L);
    const uint32_t msel = list_select<G>(c.m, a, c.j, c.base, s, L);
    // list slot j takes the j-th surviving candidate (list order)
    uint32_t mm = msel;
#pragma unroll
    for (int t = 0; t < G - 1; ++t)
        if (t < c.j) mm &= mm - 1u;
    const int cidx = mm ? __builtin_ctz(mm) : c.j;
    const bool flip = mm ? (cidx >= s) : false;
    const int srcj = flip ? cidx - s : (mm ? cidx : c.j);
    float u;
    if constexpr (G == 1) {
        u = sgn_bits(l);
        if (flip) {
            u = -u;
            c.m = c.m + a;
        }
    } else {
        const int src = c.base + srcj;
        const float ls = __shfl(l, src, 64);
        const float ms = __shfl(c.m, src, 64);
        copy_live<N, G, I>(c, src);
        u = sgn_bits(ls);
        if (flip) u = -u;
        c.m = flip ? ms + __builtin_fabsf(ls) : ms;
    }
    c.beta[I] = u;
    c.sm[I >> 5] |= (u < 0.0f ? 1u : 0u) << (I & 31);
    c.zm[I >> 5] |= (u == 0.0f ? 1u : 0u) << (I & 31);
    c.slot = slot + 1u;
    (void)lane;
}

template <int N, int G, int I>
__device__ __forceinline__ void leaf(Lane<N, G>& c, float l, int lane) {
    const bool frozen = (c.fz[I >> 5] >> (I & 31)) & 1u;
    if (frozen) {
        const float pen = (l > 0.0f) ? 0.0f : __builtin_fabsf(l);  // |l| * (sign(l) != 1), polar.py:814
        c.m = c.m + pen;
        c.beta[I] = 1.0f;
    } else {
        info_leaf<N, G, I>(c, l, lane);
    }
}

template <int N, int G, int D, int S0>
__device__ __forceinline__ void node(Lane<N, G>& c, int lane) {
    if constexpr (D == 0) {
        leaf<N, G, S0>(c, c.lv[1], lane);
    } else {
        constexpr int h = 1 << (D - 1);
#pragma unroll
        for (int j = 0; j < h; ++j) c.lv[h + j] = f_minsum(c.lv[2 * h + j], c.lv[3 * h + j]);
        node<N, G, D - 1, S0>(c, lane);
#pragma unroll
        for (int j = 0; j < h; ++j) c.lv[h + j] = c.beta[S0 + j] * c.lv[2 * h + j] + c.lv[3 * h + j];
        node<N, G, D - 1, S0 + h>(c, lane);
        if constexpr (S0 + (1 << D) < N) {  // nodes on the right spine never feed a g-update
#pragma unroll
            for (int j = 0; j < h; ++j) c.beta[S0 + j] = c.beta[S0 + j] * c.beta[S0 + h + j];
        }
    }
}

template <int N, int G>
__global__ __launch_bounds__(64) void scl_kernel(const CodeParams p, const Args a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    constexpr int n = log2c<N>();
    constexpr int C = N / 4;      // 16-B chunks per row
    constexpr int T = 64 / G;     // codewords per wave tile
    constexpr int W = (N + 31) / 32;
    const int lane = threadIdx.x;
    const f4* y4 = reinterpret_cast<const f4*>(a.y);
    const int64_t last4 = a.B * C - 1;
    const int K = p.K;

    Lane<N, G> c;
    c.j = lane & (G - 1);
    c.base = lane - c.j;
    c.L = a.L;
    const int r = lane / G;       // row of this lane's codeword in the tile
    const int sw = swz<C>(r);
    const int s_final = K >= 3 ? a.L : ((1 << K) < a.L ? (1 << K) : a.L);

    uint32_t err_bits = 0, err_blocks = 0;
    for (int64_t t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
        const int64_t row0 = t * T;
        // ---- stage the tile's received words in LDS (coalesced), swizzled rows
        __syncthreads();
        for (int i = lane; i < T * C; i += 64) {
            const int rr = i / C, cc = i % C;
            int64_t gi = row0 * C + i;
            gi = gi < last4 ? gi : last4;
            *reinterpret_cast<f4*>(lds + 16 * (rr * C + (cc ^ swz<C>(rr)))) = y4[gi];
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < C; ++q) {
            const f4 v = *reinterpret_cast<const f4*>(lds + 16 * (r * C + (q ^ sw)));
            c.lv[N + 4 * q + 0] = rmul(a.scale, v.x);
            c.lv[N + 4 * q + 1] = rmul(a.scale, v.y);
            c.lv[N + 4 * q + 2] = rmul(a.scale, v.z);
            c.lv[N + 4 * q + 3] = rmul(a.scale, v.w);
        }
#pragma unroll
        for (int w = 0; w < W; ++w) {
            uint32_t fw = p.frozen[w];
            asm volatile("" : "+s"(fw));
            c.fz[w] = fw;
            c.sm[w] = 0u;
            c.zm[w] = 0u;
        }
        c.m = 0.0f;
        c.slot = 0u;
        node<N, G, n, 0>(c, lane);

        // ---- ML choice (polar.py:868-874): codeword of each path from its decision bits
        uint32_t S[W], Z[W];
#pragma unroll
        for (int w = 0; w < W; ++w) {
            S[w] = c.sm[w];
            Z[w] = c.zm[w];
        }
        constexpr uint32_t kLow[5] = {0x55555555u, 0x33333333u, 0x0F0F0F0Fu, 0x00FF00FFu, 0x0000FFFFu};
#pragma unroll
        for (int d = 0; d < (n < 5 ? n : 5); ++d) {
#pragma unroll
            for (int w = 0; w < W; ++w) {
                S[w] ^= (S[w] >> (1 << d)) & kLow[d];
                Z[w] |= (Z[w] >> (1 << d)) & kLow[d];
            }
        }
        if constexpr (n == 6) {
            S[0] ^= S[1];
            Z[0] |= Z[1];
        }
        float dist = 0.0f;
#pragma unroll
        for (int q = 0; q < C; ++q) {
            const f4 v = *reinterpret_cast<const f4*>(lds + 16 * (r * C + (q ^ sw)));
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int k = 4 * q + e;
                const uint32_t sb = (S[k >> 5] >> (k & 31)) & 1u, zb = (Z[k >> 5] >> (k & 31)) & 1u;
                const float cv = zb ? 0.0f : (sb ? -1.0f : 1.0f);
                const float dd = cv - v[e];
                dist = dist + rmul(dd, dd);
            }
        }
        float bd = c.j < s_final ? dist : __builtin_inff();
        int bi = c.j;
#pragma unroll
        for (int off = 1; off < G; off <<= 1) {
            const float od = __shfl_xor(bd, off, 64);
            const int oi = __shfl_xor(bi, off, 64);
            if (od < bd || (od == bd && oi < bi)) {
                bd = od;
                bi = oi;
            }
        }
        const int64_t cw = row0 + r;
        if (c.j == bi && cw < a.B) {
            uint32_t e = 0;
            uint32_t mw[4] = {0u, 0u, 0u, 0u};
            if (a.count) {
                const u32x4 o = philox_block(a.seed, kStreamMsg, a.cw_offset + (uint64_t)cw, 0u);
                mw[0] = o.x;
                mw[1] = o.y;
                mw[2] = o.z;
                mw[3] = o.w;
            }
            float* mrow = a.msg ? a.msg + cw * K : nullptr;
            for (int k = 0; k < K; ++k) {
                const int pos = p.info[k];
                const uint32_t sw0 = W > 1 && pos >= 32 ? c.sm[W - 1] : c.sm[0];
                const uint32_t zw0 = W > 1 && pos >= 32 ? c.zm[W - 1] : c.zm[0];
                const uint32_t sb = (sw0 >> (pos & 31)) & 1u, zb = (zw0 >> (pos & 31)) & 1u;
                if (mrow) mrow[k] = zb ? 0.0f : (sb ? -1.0f : 1.0f);
                e += ((sb ^ ((mw[k >> 5] >> (k & 31)) & 1u)) | zb);
            }
            if (a.uhat) {
                float* urow = a.uhat + cw * N;
#pragma unroll
                for (int k = 0; k < N; ++k) {
                    const uint32_t sb = (c.sm[k >> 5] >> (k & 31)) & 1u, zb = (c.zm[k >> 5] >> (k & 31)) & 1u;
                    urow[k] = zb ? 0.0f : (sb ? -1.0f : 1.0f);
                }
            }
            err_bits += e;
            err_blocks += e ? 1u : 0u;
        }
    }
    if (a.count) {
        const uint32_t eb = wave_sum_u32(err_bits);
        const uint32_t bl = wave_sum_u32(err_blocks);
        if (lane == 0) {
            atomicAdd(a.counters + 0, (unsigned long long)eb);
            atomicAdd(a.counters + 1, (unsigned long long)bl);
        }
    }
}

template <int N, int G>
static int launch(const CodeParams& p, Args a, hipStream_t s) {
    constexpr int T = 64 / G;
    const size_t lds = (size_t)T * N * 4;
    a.ntiles = (a.B + T - 1) / T;
    auto kern = scl_kernel<N, G>;
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, 64, lds) != hipSuccess || occ <= 0) {
        (void)hipGetLastError();
        occ = 1;
    }
    const int grid = grid_for(a.ntiles, occ, device_cu_count());
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64), lds, s, p, a);
    return launch_check("scl_kernel launch");
}

template <int N>
static int launch_n(const CodeParams& p, const Args& a, hipStream_t s) {
    if (a.L == 1) return launch<N, 1>(p, a, s);
    if (a.L == 2) return launch<N, 2>(p, a, s);
    if (a.L <= 4) return launch<N, 4>(p, a, s);
    return launch<N, 8>(p, a, s);
}

// ---------------------------------------------------------------------------------- N >= 128
// The register file cannot hold a path's N-1 internal LLRs at N >= 128 (and a compile-time-unrolled tree
// that large would not fit the instruction cache), so each lane's path state lives in LDS,
// lane-interleaved (element e of lane q at dword e*64 + q: every wave access is bank-conflict free) and
// the SC schedule is walked iteratively (leaf i: one g step at level ctz(i), f steps down to the leaf,
// partial-sum combines for the nodes finished at i).  Per lane:
//   LLR level d = 1..n-1 (2^d values) at rows [2^d - 2, 2^(d+1) - 2); level 0 is a register;
//   bit rows: beta sign | beta zero | decision (u < 0) | decision (u == 0), W = N/32 words each.
// Partial sums are values in {+-1, +-0}: the float sign bit and a zero flag reproduce the reference's
// fp32 products exactly (sign bits XOR, zero flags OR).  The channel level is never stored: the two
// root steps read y through L1/L2 (the G lanes of a codeword read the same row).
// At an information leaf a lane whose slot takes another path's state copies only the LLR levels still
// read later (level D iff leaf i is in the left child of its level-D node) and the bit rows; all lanes
// of the wave read element e before any lane writes it (one instruction stream), so copies between
// lanes of a group need no double buffer.
// N = 256: the top internal level (n-1, the root's two children, 128 values) is not stored but recomputed from y
// (L1/L2) and the path's own partial-sum bits at the four steps that read it (leaves 0, N/4, N/2, 3N/4): 158
// rows = 40 KB of LDS per wave instead of 73 KB, so four waves (one per SIMD) fit a CU instead of two; a path
// switch then never copies that level either.
template <int N>
struct LdsRows {
    static constexpr int n = log2c<N>();
    static constexpr int W = N / 32;
    static constexpr bool kTopRec = N >= 256;
    static constexpr int kLv = kTopRec ? N / 2 - 2 : N - 2;  // LLR rows (levels 1 .. n-1, or 1 .. n-2)
    static constexpr int kBS = kLv;          // beta sign words
    static constexpr int kBZ = kLv + W;      // beta zero words
    static constexpr int kDS = kLv + 2 * W;  // decision sign words
    static constexpr int kDZ = kLv + 3 * W;  // decision zero words
    static constexpr int kRows = kLv + 4 * W;
};

__device__ __forceinline__ float beta_val(uint32_t sw, uint32_t zw, int b) {
    return bitsf((((sw >> b) & 1u) << 31) | (((zw >> b) & 1u) ? 0u : 0x3f800000u));
}

// level n-1 of the tree (the root's left child if !right, else its right child), elements x .. x+3 of one
// lane's path: f / g on the channel LLRs (polar.py:805-866 via updateLLR), g with the path's partial sums of
// the root's left half (sign / zero bit words BS / BZ, positions 0 .. N/2-1)
template <int N>
__device__ __forceinline__ f4 top4(const f4* y4, float scale, int x, bool right, const uint32_t* BW, int rowBS,
                                   int rowBZ, int lane) {
    const f4 u = y4[x >> 2], v = y4[(x + N / 2) >> 2];
    f4 o;
    if (!right) {
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = f_minsum(rmul(scale, u[e]), rmul(scale, v[e]));
    } else {
        const uint32_t sw = BW[(rowBS + (x >> 5)) * kWave + lane], zw = BW[(rowBZ + (x >> 5)) * kWave + lane];
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = beta_val(sw, zw, (x + e) & 31) * rmul(scale, u[e]) + rmul(scale, v[e]);
    }
    return o;
}

template <int N, int G>
__global__ __launch_bounds__(64) void scl_lds_kernel(const CodeParams p, const Args a) {
    extern __shared__ __attribute__((aligned(16))) char lds_raw[];
    using R = LdsRows<N>;
    constexpr int n = R::n;
    constexpr int W = R::W;
    constexpr int T = 64 / G;
    const int lane = threadIdx.x;
    float* const LV = reinterpret_cast<float*>(lds_raw);
    uint32_t* const BW = reinterpret_cast<uint32_t*>(lds_raw);
#define LVL(row) LV[(row) * kWave + lane]
#define BWL(row) BW[(row) * kWave + lane]
    const int K = p.K;
    const int L = a.L;
    const int j = lane & (G - 1);
    const int base = lane - j;
    const int r = lane / G;
    const int s_final = K >= 3 ? L : ((1 << K) < L ? (1 << K) : L);

    uint32_t err_bits = 0, err_blocks = 0;
    for (int64_t t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
        const int64_t cw = t * T + r;
        const int64_t cwc = cw < a.B ? cw : a.B - 1;
        const float* yr = a.y + cwc * N;
        const f4* y4 = reinterpret_cast<const f4*>(yr);
#pragma unroll
        for (int w = 0; w < 4 * W; ++w) BWL(R::kBS + w) = 0u;
        float m = 0.0f;
        uint32_t slot = 0;

        for (int i = 0; i < N; ++i) {
            int d;  // level the f chain starts from
            if (R::kTopRec && (i & (N / 4 - 1)) == 0) {
                // level n-2 from the recomputed level n-1: f at leaves 0 and N/2 (left children), g at N/4 and 3N/4
                constexpr int h2 = N / 4;
                const bool right = i >= N / 2;
                const bool gstep = (i & (N / 2 - 1)) != 0;
                const int s0 = i - h2;  // g: the left sibling's partial sums are bits s0 .. s0 + h2 - 1
                for (int q = 0; q < h2 / 4; ++q) {
                    const f4 A = top4<N>(y4, a.scale, 4 * q, right, BW, R::kBS, R::kBZ, lane);
                    const f4 Bv = top4<N>(y4, a.scale, 4 * q + h2, right, BW, R::kBS, R::kBZ, lane);
                    if (!gstep) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) LVL(h2 - 2 + 4 * q + e) = f_minsum(A[e], Bv[e]);
                    } else {
                        const int q0 = s0 + 4 * q;
                        const uint32_t sw = BWL(R::kBS + (q0 >> 5)), zw = BWL(R::kBZ + (q0 >> 5));
#pragma unroll
                        for (int e = 0; e < 4; ++e) LVL(h2 - 2 + 4 * q + e) = beta_val(sw, zw, (q0 + e) & 31) * A[e] + Bv[e];
                    }
                }
                d = n - 2;
            } else if (i == 0) {  // left child of the root: f on the channel LLRs
                constexpr int h = N / 2;
                for (int q = 0; q < h / 4; ++q) {
                    const f4 u = y4[q], v = y4[q + h / 4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) LVL(h - 2 + 4 * q + e) = f_minsum(rmul(a.scale, u[e]), rmul(a.scale, v[e]));
                }
                d = n - 1;
            } else {  // right child of the node of 2^(k+1) leaves starting at i - 2^k
                const int k = __builtin_ctz((unsigned)i);
                const int h = 1 << k;
                const int s0 = i - h;
                if (k == 0) {
                    d = 0;
                } else if (k + 1 == n) {  // right child of the root: g on the channel LLRs
                    for (int q = 0; q < h / 4; ++q) {
                        const uint32_t sw = BWL(R::kBS + (q >> 3)), zw = BWL(R::kBZ + (q >> 3));
                        const f4 u = y4[q], v = y4[q + h / 4];
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const float b = beta_val(sw, zw, (4 * q + e) & 31);
                            LVL(h - 2 + 4 * q + e) = b * rmul(a.scale, u[e]) + rmul(a.scale, v[e]);
                        }
                    }
                    d = k;
                } else {
                    for (int j0 = 0; j0 < h; j0 += 32) {
                        const int q0 = s0 + j0;
                        const uint32_t sw = BWL(R::kBS + (q0 >> 5)) >> (q0 & 31);
                        const uint32_t zw = BWL(R::kBZ + (q0 >> 5)) >> (q0 & 31);
                        const int hw = h < 32 ? h : 32;
                        for (int jj = 0; jj < hw; ++jj) {
                            const float b = beta_val(sw, zw, jj);
                            LVL(h - 2 + j0 + jj) = b * LVL(2 * h - 2 + j0 + jj) + LVL(2 * h - 2 + h + j0 + jj);
                        }
                    }
                    d = k;
                }
            }
            for (int dd = d - 1; dd >= 1; --dd) {  // left children down to level 1
                const int h = 1 << dd;
                for (int jj = 0; jj < h; ++jj) LVL(h - 2 + jj) = f_minsum(LVL(2 * h - 2 + jj), LVL(2 * h - 2 + h + jj));
            }
            float l;
            if (d == 0) {  // leaf i is a right child: g from level 1 with the left sibling's decision
                const uint32_t sw = BWL(R::kBS + ((i - 1) >> 5)), zw = BWL(R::kBZ + ((i - 1) >> 5));
                l = beta_val(sw, zw, (i - 1) & 31) * LVL(0) + LVL(1);
            } else {
                l = f_minsum(LVL(0), LVL(1));
            }

            // ---- leaf (polar.py:805-866)
            const bool frozen = (p.frozen[i >> 5] >> (i & 31)) & 1u;
            const int wi = i >> 5;
            const uint32_t bi = 1u << (i & 31);
            if (frozen) {
                m = m + ((l > 0.0f) ? 0.0f : __builtin_fabsf(l));  // |l| * (sign(l) != 1), polar.py:814
                // u = +1: beta sign/zero bits stay clear
            } else {
                const float av = __builtin_fabsf(l);
                const int s = slot >= 3u ? L : ((1 << slot) < L ? (1 << slot) : L);
                float u;
                if constexpr (G == 1) {
                    u = sgn_bits(l);  // L = 1: plain SC with the metric tracked (pruning keeps the smaller one)
                    const uint32_t msel = list_select<G>(m, av, j, base, s, L);
                    if (!(msel & 1u)) {
                        u = -u;
                        m = m + av;
                    }
                } else {
                    const uint32_t msel = list_select<G>(m, av, j, base, s, L);
                    uint32_t mm = msel;
#pragma unroll
                    for (int q = 0; q < G - 1; ++q)
                        if (q < j) mm &= mm - 1u;
                    const int cidx = mm ? __builtin_ctz(mm) : j;
                    const bool flip = mm ? (cidx >= s) : false;
                    const int srcj = flip ? cidx - s : (mm ? cidx : j);
                    const int src = base + srcj;
                    const float ls = __shfl(l, src, 64);
                    const float ms = __shfl(m, src, 64);
                    if (src != lane) {
                        // live LLR levels: D in 1..n-1 with leaf i in the left child of its level-D node
                        for (int D = 1; D < (R::kTopRec ? n - 1 : n); ++D) {
                            if ((i >> (D - 1)) & 1) continue;
                            const int b0 = (1 << D) - 2;
                            for (int e = 0; e < (1 << D); ++e) LV[(b0 + e) * kWave + lane] = LV[(b0 + e) * kWave + src];
                        }
#pragma unroll
                        for (int w = 0; w < 4 * W; ++w) BW[(R::kBS + w) * kWave + lane] = BW[(R::kBS + w) * kWave + src];
                    }
                    u = sgn_bits(ls);
                    if (flip) u = -u;
                    m = flip ? ms + __builtin_fabsf(ls) : ms;
                }
                if (fbits(u) >> 31) BWL(R::kBS + wi) |= bi;
                if (u == 0.0f) BWL(R::kBZ + wi) |= bi;
                if (u < 0.0f) BWL(R::kDS + wi) |= bi;
                if (u == 0.0f) BWL(R::kDZ + wi) |= bi;
                slot = slot + 1u;
            }
            // ---- partial sums of the nodes whose right child ends at leaf i (the right spine is never read)
            if (i != N - 1) {
                for (int l2 = 0; (i >> l2) & 1; ++l2) {
                    const int h = 1 << l2;
                    const int s0 = i + 1 - 2 * h;
                    if (h < 32) {
                        const int w = s0 >> 5, o = s0 & 31;
                        const uint32_t lowm = (1u << h) - 1u;
                        uint32_t sw = BWL(R::kBS + w), zw = BWL(R::kBZ + w);
                        sw ^= ((sw >> (o + h)) & lowm) << o;
                        zw |= ((zw >> (o + h)) & lowm) << o;
                        BWL(R::kBS + w) = sw;
                        BWL(R::kBZ + w) = zw;
                    } else {
                        const int w0 = s0 >> 5, hw = h >> 5;
                        for (int q = 0; q < hw; ++q) {
                            BWL(R::kBS + w0 + q) ^= BWL(R::kBS + w0 + hw + q);
                            BWL(R::kBZ + w0 + q) |= BWL(R::kBZ + w0 + hw + q);
                        }
                    }
                }
            }
        }

        // ---- ML choice (polar.py:868-874): codeword of each path from its decision bits
        uint32_t S[W], Z[W];
#pragma unroll
        for (int w = 0; w < W; ++w) {
            S[w] = BWL(R::kDS + w);
            Z[w] = BWL(R::kDZ + w);
        }
        constexpr uint32_t kLow[5] = {0x55555555u, 0x33333333u, 0x0F0F0F0Fu, 0x00FF00FFu, 0x0000FFFFu};
#pragma unroll
        for (int dd = 0; dd < 5; ++dd) {
#pragma unroll
            for (int w = 0; w < W; ++w) {
                S[w] ^= (S[w] >> (1 << dd)) & kLow[dd];
                Z[w] |= (Z[w] >> (1 << dd)) & kLow[dd];
            }
        }
#pragma unroll
        for (int dd = 5; dd < n; ++dd) {
            const int st = 1 << (dd - 5);
#pragma unroll
            for (int w = 0; w < W; ++w) {
                if ((w & st) == 0) {
                    S[w] ^= S[w + st];
                    Z[w] |= Z[w + st];
                }
            }
        }
        float dist = 0.0f;
#pragma unroll
        for (int q = 0; q < N / 4; ++q) {
            const f4 v = y4[q];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int k = 4 * q + e;
                const uint32_t sb = (S[k >> 5] >> (k & 31)) & 1u, zb = (Z[k >> 5] >> (k & 31)) & 1u;
                const float cv = zb ? 0.0f : (sb ? -1.0f : 1.0f);
                const float dd = cv - v[e];
                dist = dist + rmul(dd, dd);
            }
        }
        float bd = j < s_final ? dist : __builtin_inff();
        int bj = j;
#pragma unroll
        for (int off = 1; off < G; off <<= 1) {
            const float od = __shfl_xor(bd, off, 64);
            const int oj = __shfl_xor(bj, off, 64);
            if (od < bd || (od == bd && oj < bj)) {
                bd = od;
                bj = oj;
            }
        }
        if (j == bj && cw < a.B) {
            uint32_t e = 0;
            uint32_t mw[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
            if (a.count) {
#pragma unroll
                for (int blk = 0; blk < 2; ++blk) {
                    if (blk * 128 < K) {
                        const u32x4 o = philox_block(a.seed, kStreamMsg, a.cw_offset + (uint64_t)cw, (uint32_t)blk);
                        mw[4 * blk + 0] = o.x;
                        mw[4 * blk + 1] = o.y;
                        mw[4 * blk + 2] = o.z;
                        mw[4 * blk + 3] = o.w;
                    }
                }
            }
            float* mrow = a.msg ? a.msg + cw * K : nullptr;
            for (int k = 0; k < K; ++k) {
                const int pos = p.info[k];
                const uint32_t sb = (BWL(R::kDS + (pos >> 5)) >> (pos & 31)) & 1u;
                const uint32_t zb = (BWL(R::kDZ + (pos >> 5)) >> (pos & 31)) & 1u;
                if (mrow) mrow[k] = zb ? 0.0f : (sb ? -1.0f : 1.0f);
                e += ((sb ^ ((mw[k >> 5] >> (k & 31)) & 1u)) | zb);
            }
            if (a.uhat) {
                float* urow = a.uhat + cw * N;
#pragma unroll
                for (int k = 0; k < N; ++k) {
                    const uint32_t sb = (BWL(R::kDS + (k >> 5)) >> (k & 31)) & 1u;
                    const uint32_t zb = (BWL(R::kDZ + (k >> 5)) >> (k & 31)) & 1u;
                    urow[k] = zb ? 0.0f : (sb ? -1.0f : 1.0f);
                }
            }
            err_bits += e;
            err_blocks += e ? 1u : 0u;
        }
    }
#undef LVL
#undef BWL
    if (a.count) {
        const uint32_t eb = wave_sum_u32(err_bits);
        const uint32_t bl = wave_sum_u32(err_blocks);
        if (lane == 0) {
            atomicAdd(a.counters + 0, (unsigned long long)eb);
            atomicAdd(a.counters + 1, (unsigned long long)bl);
        }
    }
}

template <int N, int G>
static int launch_lds(const CodeParams& p, Args a, hipStream_t s) {
    constexpr int T = 64 / G;
    const size_t lds = (size_t)LdsRows<N>::kRows * kWave * sizeof(float);
    a.ntiles = (a.B + T - 1) / T;
    auto kern = scl_lds_kernel<N, G>;
    static bool attr_set = false;  // benign race (idempotent)
    if (!attr_set && lds > 65536) {
        NPD_HIP(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
        attr_set = true;
    }
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, 64, lds) != hipSuccess || occ <= 0) {
        (void)hipGetLastError();
        occ = 1;
    }
    const int grid = grid_for(a.ntiles, occ, device_cu_count());
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64), lds, s, p, a);
    return launch_check("scl_lds_kernel launch");
}

template <int N>
static int launch_lds_n(const CodeParams& p, const Args& a, hipStream_t s) {
    if (a.L == 1) return launch_lds<N, 1>(p, a, s);
    if (a.L == 2) return launch_lds<N, 2>(p, a, s);
    if (a.L <= 4) return launch_lds<N, 4>(p, a, s);
    return launch_lds<N, 8>(p, a, s);
}

static int run(const npd_code* code, Args& a, hipStream_t s) {
    const CodeParams& p = code->p;
    if (p.pac) return fail(NPD_ENOTSUP, "scl_decode: the reference defines SC-List for Polar codes only");
    if (p.N < 8 || p.N > 256) return fail(NPD_ENOTSUP, "scl_decode: N must be 8..256");
    if (a.L < 1 || a.L > 8) return fail(NPD_EINVAL, "scl_decode: list size must be 1..8");
    if ((((uintptr_t)a.y) & 15) != 0) return fail(NPD_EINVAL, "scl_decode: y must be 16-byte aligned");
    if (a.B == 0) return NPD_OK;
    switch (p.N) {
        case 8: return launch_n<8>(p, a, s);
        case 16: return launch_n<16>(p, a, s);
        case 32: return launch_n<32>(p, a, s);
        case 64: return launch_n<64>(p, a, s);
        case 128: return launch_lds_n<128>(p, a, s);
        default: return launch_lds_n<256>(p, a, s);
    }
}

}  // namespace scl
}  // namespace npd

using namespace npd;

extern "C" int npd_scl_decode(const npd_code* code, const float* y, float llr_scale, int list_size, float* msg_hat,
                              float* u_hat, int64_t B, void* stream) {
    NPD_ARG(code != nullptr, "npd_scl_decode: code is NULL");
    NPD_ARG(B >= 0, "npd_scl_decode: B < 0");
    NPD_ARG(B == 0 || y != nullptr, "npd_scl_decode: y is NULL");
    scl::Args a{};
    a.y = y;
    a.msg = msg_hat;
    a.uhat = u_hat;
    a.B = B;
    a.scale = llr_scale;
    a.L = list_size;
    return scl::run(code, a, (hipStream_t)stream);
}

extern "C" int npd_scl_decode_mc(const npd_code* code, const float* y, float llr_scale, int list_size,
                                 float* msg_hat, uint64_t seed, uint64_t cw_offset, int64_t B,
                                 unsigned long long* counters, void* stream) {
    NPD_ARG(code != nullptr, "npd_scl_decode_mc: code is NULL");
    NPD_ARG(B >= 0, "npd_scl_decode_mc: B < 0");
    NPD_ARG(B == 0 || y != nullptr, "npd_scl_decode_mc: y is NULL");
    NPD_ARG(counters != nullptr, "npd_scl_decode_mc: counters is NULL");
    scl::Args a{};
    a.y = y;
    a.msg = msg_hat;
    a.counters = counters;
    a.seed = seed;
    a.cw_offset = cw_offset;
    a.B = B;
    a.scale = llr_scale;
    a.L = list_size;
    a.count = 1u;
    return scl::run(code, a, (hipStream_t)stream);
}

extern "C" int npd_list_prune_select(const float* neg_metrics, int n, int keep, uint32_t* mask_out) {
    NPD_ARG(neg_metrics != nullptr && mask_out != nullptr, "npd_list_prune_select: NULL pointer");
    NPD_ARG(n >= 1 && n <= 16 && keep >= 1 && keep <= n, "npd_list_prune_select: need 1 <= keep <= n <= 16");
    *mask_out = nth::prune_mask(neg_metrics, n, keep);
    return NPD_OK;
}
