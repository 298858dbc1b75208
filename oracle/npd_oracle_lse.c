/*
 * npd_oracle_lse.c -- CPU restatement of the reference's exact log-sum-exp SC decoder.
 *
 * TEST INFRASTRUCTURE ONLY (see npd_oracle.c): used by tests/ as the checker of npd_sc_decode_lse.
 *
 *   PolarCode.sc_decode / decode   polar.py:209-279  recursion decode(llrs, depth, bit_position): left
 *                                                    child on LSE(l[:h], l[h:]), right child on
 *                                                    u_hat*l[:h] + l[h:], two leaves per call at depth
 *                                                    n-1, frozen -> +1, info -> sign(L) (hard) or
 *                                                    tanh(L/2) (soft), returns cat(u*v, v)
 *   log_sum_avoid_NaN              utils.py:295-345  restated literally on each call's vector: the
 *                                                    patches run only when the vector holds a NaN/inf
 *                                                    (the GPU kernel patches per element; the tests
 *                                                    pin that the two agree)
 *   log_sum_avoid_zero_NaN         utils.py:348-397  (close_1/close_2 blend written as in the reference)
 *   PolarCode.sc_decode_soft       polar.py:281-358  decode_soft: nodes return LLRs, leaf clamp(L + prior,
 *                                                    +-1000) (Clamp, utils.py:259-263), no frozen rule
 *   PolarCode.sc_decode_soft_new   polar.py:485-607  the same recursion (see oracle_sc_decode_soft), leaf
 *                                                    clamp(L + prior) + prior, output sign(leaf)[:, info]
 *
 * Compiled with -ffp-contract=off.  exp/log/tanh are glibc's; torch's CPU path uses Sleef (<= 1 ulp), so
 * agreement with the reference is within a tolerance, pinned by tests/golden/lse_*.npz.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#define LSE_MAX_N 256

static inline float sgn(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); } /* torch.sign: NaN -> 0 */
static inline float tmax(float a, float b) { return (isnan(a) || isnan(b)) ? NAN : (a > b ? a : b); }
static inline float tmin(float a, float b) { return (isnan(a) || isnan(b)) ? NAN : (a < b ? a : b); }

/* utils.py:295-345 on a vector of n pairs */
static void log_sum_avoid_nan(const float* x, const float* y, float* out, int n) {
    int bad = 0;
    for (int i = 0; i < n; ++i) {
        float t1 = logf(1.0f + expf(x[i] + y[i]));
        float t3 = logf(1.0f + expf(y[i] - x[i]));
        out[i] = (t1 - x[i]) - t3;
        if (isnan(out[i]) || isinf(out[i])) bad = 1;
    }
    if (!bad) return;
    const float big = 200.0f;
    for (int i = 0; i < n; ++i) {
        float s = x[i] + y[i];
        float d = fabsf(x[i] - y[i]);
        float a = tmax(x[i], y[i]), b = tmin(x[i], y[i]);
        int idx1 = s > big, sub1 = idx1 && d < big;
        int idx2 = s < -big, sub2 = idx2 && d < big;
        int idx3 = (d > big) && (fabsf(s) < big);
        if (idx1) out[i] = sub1 ? y[i] - logf(1.0f + expf(y[i] - x[i])) : b;
        if (idx2) out[i] = sub2 ? -x[i] - logf(1.0f + expf(y[i] - x[i])) : -a;
        if (idx3) out[i] = logf(1.0f + expf(x[i] + y[i])) - a;
    }
}

/* utils.py:348-397 */
static void log_sum_avoid_zero_nan(const float* x, const float* y, float* out, int n) {
    log_sum_avoid_nan(x, y, out, n);
    for (int i = 0; i < n; ++i) {
        if (out[i] != 0.0f) continue;
        float s = x[i] + y[i];
        float nume = (s < 0.0f) ? 0.0f : s; /* torch.relu */
        float denom = tmax(x[i], y[i]);
        float term1 = 0.5f * (expf(-nume) + expf(s - nume));
        float term2 = 0.5f * (expf(x[i] - denom) + expf(y[i] - denom));
        float c1 = (fabsf(term1 - 1.0f) < 1e-7f) ? 1.0f : 0.0f;
        float T1 = (term1 - 1.0f) * c1 + logf(term1) * (1.0f - c1);
        float c2 = (fabsf(term2 - 1.0f) < 1e-7f) ? 1.0f : 0.0f;
        float T2 = (term2 - 1.0f) * c2 + logf(term2) * (1.0f - c2);
        float ans = ((nume - denom) + T1) - T2;
        if (ans == 0.0f) ans = (s > 0.0f) ? tmin(x[i], y[i]) : tmin(-x[i], -y[i]);
        out[i] = ans;
    }
}

typedef struct {
    int n;
    const uint8_t* frozen;
    int hard;
    float* bits; /* decoded_bits row */
} lse_ctx;

static inline float decide_c(int hard, float L) { return hard ? sgn(L) : tanhf(L / 2.0f); }
static inline float decide(const lse_ctx* c, float L) { return decide_c(c->hard, L); }

/* decode(llrs, depth, bit_position) (polar.py:226-279); ret = returned partial-sum vector (2*half) */
static void lse_decode(lse_ctx* c, const float* llrs, int depth, int bitpos, float* ret) {
    const int half = 1 << (c->n - depth - 1);
    if (depth == c->n - 1) {
        const int lp = 2 * bitpos, rp = 2 * bitpos + 1;
        float u = 1.0f, v = 1.0f;
        if (!c->frozen[lp]) {
            float Lu;
            log_sum_avoid_zero_nan(&llrs[0], &llrs[1], &Lu, 1);
            u = decide(c, Lu);
        }
        if (!c->frozen[rp]) {
            float Lv = u * llrs[0] + llrs[1];
            v = decide(c, Lv);
        }
        c->bits[lp] = u;
        c->bits[rp] = v;
        ret[0] = u * v;
        ret[1] = v;
        return;
    }
    float Lu[LSE_MAX_N / 2], uh[LSE_MAX_N / 2], Lv[LSE_MAX_N / 2], vh[LSE_MAX_N / 2];
    log_sum_avoid_zero_nan(llrs, llrs + half, Lu, half);
    lse_decode(c, Lu, depth + 1, 2 * bitpos, uh);
    for (int j = 0; j < half; ++j) Lv[j] = uh[j] * llrs[j] + llrs[half + j];
    lse_decode(c, Lv, depth + 1, 2 * bitpos + 1, vh);
    for (int j = 0; j < half; ++j) {
        ret[j] = uh[j] * vh[j];
        ret[half + j] = vh[j];
    }
}

/*
 * PolarCode.sc_decode(y, snr): llrs = llr_scale * y (llr_scale = fl32(2/sigma^2)); msg_hat (B,K) =
 * sign(decoded_bits)[:, info]; bits_out (B,N) = decoded_bits.  Either output may be NULL.
 */
void oracle_sc_decode_lse(const float* y, int64_t B, int N, int K, const int32_t* info, const uint8_t* frozen,
                          float llr_scale, int hard, float* msg_hat, float* bits_out) {
    int n = 0;
    while ((1 << n) < N) ++n;
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < B; ++b) {
        float llr[LSE_MAX_N], bits[LSE_MAX_N], ret[LSE_MAX_N];
        for (int i = 0; i < N; ++i) llr[i] = llr_scale * y[b * N + i];
        lse_ctx c = {n, frozen, hard, bits};
        lse_decode(&c, llr, 0, 0, ret);
        if (bits_out) memcpy(bits_out + b * N, bits, sizeof(float) * (size_t)N);
        if (msg_hat)
            for (int k = 0; k < K; ++k) msg_hat[b * K + k] = sgn(bits[info[k]]);
    }
}

/* ------------------------------------------------------------------ forward error bound of sc_decode */
/*
 * Running first-order error analysis of the same recursion (soft or hard decisions): alongside every
 * fp32 value v the double E(v) bounds |v - v_exact| when every operation is evaluated with relative error
 * at most eps_op: + - * and the LLR scaling are correctly rounded (1 unit of u = 2^-24); exp, log and
 * tanh are allowed 4 units (2 ulp: glibc, Sleef -- torch's CPU path -- and the device OCML are all within
 * that).  Propagation uses the exact sensitivities of each operation:
 *   boxplus f(x,y) = log((1+e^(x+y))/(e^x+e^y)):  df/dx = s(x+y) - s(x-y), df/dy = s(x+y) - s(y-x)
 *     (s = logistic), plus the rounding of its evaluated form log(1+e^(x+y)) - x - log(1+e^(y-x)),
 *     whose terms have magnitude ~|x| + |y| (the cancellation that makes a leaf's LLR conditioning-bound);
 *   g = u a + b;  tanh(L/2): 0.5 (1 - u^2);  partial-sum products u v.
 * Two implementations that both satisfy the model differ by at most 2 E per value; tests use that as a
 * per-entry bound on decoded_bits instead of a fixed tolerance.  Non-finite values (88 < x+y < 200: exp
 * overflows and no patch applies) get an infinite bound (the tests compare those by NaN position).
 */
#define U32 5.9604644775390625e-08 /* 2^-24 */
#define UT (4.0 * U32)             /* transcendental allowance */

static inline double logistic(double t) { return 1.0 / (1.0 + exp(-t)); }
/* m * e with 0 * inf = 0: an exactly known factor (error 0, or value 0) contributes nothing */
static inline double sm(double m, double e) { return (m == 0.0 || e == 0.0) ? 0.0 : fabs(m) * e; }

/* bound of u = tanh(L/2) given E(L): the tanh rounding plus the worst slope over [|L| - E, |L| + E];
   L = +-inf (same patch branch on both sides) gives u = +-1 exactly */
static inline double tanh_bound(float L, float u, double eL) {
    if (!isfinite(L)) return 0.0;
    if (!isfinite(eL)) return 1.0;
    const double lo = fabs((double)L) - eL;
    const double t = tanh((lo > 0.0 ? lo : 0.0) / 2.0);
    return UT * fabs((double)u) + 0.5 * (1.0 - t * t) * eL;
}

static double lse_bound(float x, float y, float out, double ex, double ey) {
    if (!isfinite(out)) return INFINITY;
    const double xd = x, yd = y, s = xd + yd, d = yd - xd;
    const double dfx = fabs(logistic(s) - logistic(xd - yd)), dfy = fabs(logistic(s) - logistic(d));
    /* every branch (the plain formula, the |x+y| > 200 / |x-y| > 200 patches, the zero re-evaluation)
       evaluates at most two log(1+e^t) terms and three subtractions on values of magnitude <= |x| + |y| */
    const double t1 = s < 88.0 ? log1p(exp(s)) : s, t3 = d < 88.0 ? log1p(exp(d)) : d;
    const double loc = U32 * (fabs(s) + fabs(d) + fabs(xd) + fabs(yd) + fabs((double)out)) + UT * (2.0 + t1 + t3);
    return sm(dfx, ex) + sm(dfy, ey) + loc;
}

typedef struct {
    int n;
    const uint8_t* frozen;
    int hard;
    float* bits;
    double* ebits;
    float* leaf;    /* decision LLR of every leaf (frozen leaves: NaN), or NULL */
    double* eleaf;  /* its bound */
} lseb_ctx;

static inline void put_leaf(float* leaf, double* eleaf, int pos, float L, double e) {
    if (leaf) {
        leaf[pos] = L;
        eleaf[pos] = e;
    }
}

static void lseb_decode(lseb_ctx* c, const float* llrs, const double* el, int depth, int bitpos, float* ret,
                        double* eret) {
    const int half = 1 << (c->n - depth - 1);
    if (depth == c->n - 1) {
        const int lp = 2 * bitpos, rp = 2 * bitpos + 1;
        float u = 1.0f, v = 1.0f;
        double eu = 0.0, ev = 0.0;
        if (!c->frozen[lp]) {
            float Lu;
            log_sum_avoid_zero_nan(&llrs[0], &llrs[1], &Lu, 1);
            const double eL = lse_bound(llrs[0], llrs[1], Lu, el[0], el[1]);
            u = decide_c(c->hard, Lu);
            eu = c->hard ? 0.0 : tanh_bound(Lu, u, eL);
            put_leaf(c->leaf, c->eleaf, lp, Lu, eL);
        } else {
            put_leaf(c->leaf, c->eleaf, lp, NAN, 0.0);
        }
        if (!c->frozen[rp]) {
            float Lv = u * llrs[0] + llrs[1];
            const double eL = sm(llrs[0], eu) + sm(u, el[0]) + el[1] + U32 * (fabs((double)u * llrs[0]) + fabs((double)Lv));
            v = decide_c(c->hard, Lv);
            ev = c->hard ? 0.0 : tanh_bound(Lv, v, eL);
            put_leaf(c->leaf, c->eleaf, rp, Lv, eL);
        } else {
            put_leaf(c->leaf, c->eleaf, rp, NAN, 0.0);
        }
        c->bits[lp] = u;
        c->bits[rp] = v;
        c->ebits[lp] = eu;
        c->ebits[rp] = ev;
        ret[0] = u * v;
        eret[0] = sm(u, ev) + sm(v, eu) + U32 * fabs((double)ret[0]);
        ret[1] = v;
        eret[1] = ev;
        return;
    }
    float Lu[LSE_MAX_N / 2], uh[LSE_MAX_N / 2], Lv[LSE_MAX_N / 2], vh[LSE_MAX_N / 2];
    double eLu[LSE_MAX_N / 2], euh[LSE_MAX_N / 2], eLv[LSE_MAX_N / 2], evh[LSE_MAX_N / 2];
    log_sum_avoid_zero_nan(llrs, llrs + half, Lu, half);
    for (int j = 0; j < half; ++j) eLu[j] = lse_bound(llrs[j], llrs[half + j], Lu[j], el[j], el[half + j]);
    lseb_decode(c, Lu, eLu, depth + 1, 2 * bitpos, uh, euh);
    for (int j = 0; j < half; ++j) {
        Lv[j] = uh[j] * llrs[j] + llrs[half + j];
        eLv[j] = sm(llrs[j], euh[j]) + sm(uh[j], el[j]) + el[half + j] +
                 U32 * (fabs((double)uh[j] * llrs[j]) + fabs((double)Lv[j]));
    }
    lseb_decode(c, Lv, eLv, depth + 1, 2 * bitpos + 1, vh, evh);
    for (int j = 0; j < half; ++j) {
        ret[j] = uh[j] * vh[j];
        eret[j] = sm(uh[j], evh[j]) + sm(vh[j], euh[j]) + U32 * fabs((double)ret[j]);
        ret[half + j] = vh[j];
        eret[half + j] = evh[j];
    }
}

/* decoded_bits (B,N) and their bounds ebits (B,N, double); optionally each leaf's decision LLR and its
   bound (B,N; frozen leaves NaN / 0) */
void oracle_sc_decode_lse_bound(const float* y, int64_t B, int N, const uint8_t* frozen, float llr_scale, int hard,
                                float* bits_out, double* ebits_out, float* leaf_out, double* eleaf_out) {
    int n = 0;
    while ((1 << n) < N) ++n;
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < B; ++b) {
        float llr[LSE_MAX_N], ret[LSE_MAX_N];
        double el[LSE_MAX_N], eret[LSE_MAX_N];
        for (int i = 0; i < N; ++i) {
            llr[i] = llr_scale * y[b * N + i];
            el[i] = 0.0; /* one correctly rounded product, identical everywhere */
        }
        lseb_ctx c = {n, frozen, hard, bits_out + b * N, ebits_out + b * N, leaf_out ? leaf_out + b * N : NULL,
                      eleaf_out ? eleaf_out + b * N : NULL};
        lseb_decode(&c, llr, el, 0, 0, ret, eret);
    }
}

/* ------------------------------------------------------------------ soft SC (polar.py:281-358) */
static inline float clamp1000(float x) { return x < -1000.0f ? -1000.0f : (x > 1000.0f ? 1000.0f : x); }

typedef struct {
    int n;
    const float* prior;
    int hard;
    float* bits;
    int twice; /* sc_decode_soft_new: stored leaf = clamp(L + prior) + prior (polar.py:518-546) */
    float* leaf;
} soft_ctx;

/* decode_soft(llrs, depth, bit_position, prior) (polar.py:305-358); ret = returned LLR vector (2*half) */
static void soft_decode(soft_ctx* c, const float* llrs, int depth, int bitpos, float* ret) {
    const int half = 1 << (c->n - depth - 1);
    if (depth == c->n - 1) {
        const int lp = 2 * bitpos, rp = 2 * bitpos + 1;
        float Lu, Luv, Lv, top;
        log_sum_avoid_zero_nan(&llrs[0], &llrs[1], &Lu, 1);
        Lu = clamp1000(Lu + c->prior[lp] * 1.0f);
        if (c->twice) Lu = Lu + c->prior[lp] * 1.0f;
        float u = c->hard ? sgn(Lu) : tanhf(Lu / 2.0f);
        log_sum_avoid_zero_nan(&Lu, &llrs[0], &Luv, 1);
        Lv = Luv + llrs[1];
        Lv = clamp1000(Lv + c->prior[rp] * 1.0f);
        if (c->twice) Lv = Lv + c->prior[rp] * 1.0f;
        float v = c->hard ? sgn(Lv) : tanhf(Lv / 2.0f);
        c->bits[lp] = u;
        c->bits[rp] = v;
        if (c->leaf) {
            c->leaf[lp] = Lu;
            c->leaf[rp] = Lv;
        }
        log_sum_avoid_zero_nan(&Lu, &Lv, &top, 1);
        ret[0] = top;
        ret[1] = Lv;
        return;
    }
    float Lu[LSE_MAX_N / 2], Lhu[LSE_MAX_N / 2], Luv[LSE_MAX_N / 2], Lv[LSE_MAX_N / 2], Lhv[LSE_MAX_N / 2];
    log_sum_avoid_zero_nan(llrs, llrs + half, Lu, half);
    soft_decode(c, Lu, depth + 1, 2 * bitpos, Lhu);
    log_sum_avoid_zero_nan(Lhu, llrs, Luv, half);
    for (int j = 0; j < half; ++j) Lv[j] = Luv[j] + llrs[half + j];
    soft_decode(c, Lv, depth + 1, 2 * bitpos + 1, Lhv);
    log_sum_avoid_zero_nan(Lhu, Lhv, ret, half);
    for (int j = 0; j < half; ++j) ret[half + j] = Lhv[j];
}

/* PolarCode.sc_decode_soft(y, snr, priors): msg_hat = sign(decoded_bits)[:, info]; priors (N) or NULL.
   twice = 1: PolarCode.sc_decode_soft_new (polar.py:485-607), whose per-leaf re-walk of the root-to-leaf
   path (partial_decode_soft) and rebuilt soft partial sums (updatePartialSums_soft: [a, b] -> [LSE(a, b), b]
   at stride 2^s over the leaves decided so far, zeros beyond) give, for every completed block, exactly
   the returned-LLR vectors of this recursion; its leaf stores clamp(L + prior) + prior and its output is
   sign(stored leaf)[:, info] (call with hard = 1).  leaf_out (B,N): every stored leaf LLR, or NULL. */
void oracle_sc_decode_soft(const float* y, int64_t B, int N, int K, const int32_t* info, const float* priors,
                           float llr_scale, int hard, int twice, float* msg_hat, float* bits_out, float* leaf_out) {
    int n = 0;
    while ((1 << n) < N) ++n;
    float zeros[LSE_MAX_N] = {0};
    const float* pr = priors ? priors : zeros;
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < B; ++b) {
        float llr[LSE_MAX_N], bits[LSE_MAX_N], ret[LSE_MAX_N];
        for (int i = 0; i < N; ++i) llr[i] = llr_scale * y[b * N + i];
        soft_ctx c = {n, pr, hard, bits, twice, leaf_out ? leaf_out + b * N : NULL};
        soft_decode(&c, llr, 0, 0, ret);
        if (bits_out) memcpy(bits_out + b * N, bits, sizeof(float) * (size_t)N);
        if (msg_hat)
            for (int k = 0; k < K; ++k) msg_hat[b * K + k] = sgn(bits[info[k]]);
    }
}

/* ------------------------------------------------------------------ forward error bound of sc_decode_soft */
/* Same error model as oracle_sc_decode_lse_bound, on decode_soft's recursion (nodes return LLRs; leaves
   clamp(L + prior, +-1000), which is 1-Lipschitz; bits = tanh(L/2) or sign(L)). */
typedef struct {
    int n;
    const float* prior;
    int hard;
    float* bits;
    double* ebits;
    float* leaf;
    double* eleaf;
    int twice;
} softb_ctx;

static inline double add_bound(float a, float b, float r, double ea, double eb) {
    (void)a; (void)b;
    return ea + eb + U32 * fabs((double)r);
}

static void softb_decode(softb_ctx* c, const float* llrs, const double* el, int depth, int bitpos, float* ret,
                         double* eret) {
    const int half = 1 << (c->n - depth - 1);
    if (depth == c->n - 1) {
        const int lp = 2 * bitpos, rp = 2 * bitpos + 1;
        float Lu0, Lu, Luv, Lv0, Lv, top;
        log_sum_avoid_zero_nan(&llrs[0], &llrs[1], &Lu0, 1);
        double eLu = lse_bound(llrs[0], llrs[1], Lu0, el[0], el[1]);
        Lu = clamp1000(Lu0 + c->prior[lp] * 1.0f);
        eLu = eLu + U32 * fabs((double)Lu0 + c->prior[lp]);
        if (c->twice) {
            Lu = Lu + c->prior[lp] * 1.0f;
            eLu = eLu + U32 * fabs((double)Lu);
        }
        float u = c->hard ? sgn(Lu) : tanhf(Lu / 2.0f);
        log_sum_avoid_zero_nan(&Lu, &llrs[0], &Luv, 1);
        const double eLuv = lse_bound(Lu, llrs[0], Luv, eLu, el[0]);
        Lv0 = Luv + llrs[1];
        double eLv = add_bound(Luv, llrs[1], Lv0, eLuv, el[1]);
        Lv = clamp1000(Lv0 + c->prior[rp] * 1.0f);
        eLv = eLv + U32 * fabs((double)Lv0 + c->prior[rp]);
        if (c->twice) {
            Lv = Lv + c->prior[rp] * 1.0f;
            eLv = eLv + U32 * fabs((double)Lv);
        }
        float v = c->hard ? sgn(Lv) : tanhf(Lv / 2.0f);
        c->bits[lp] = u;
        c->bits[rp] = v;
        c->ebits[lp] = c->hard ? 0.0 : tanh_bound(Lu, u, eLu);
        c->ebits[rp] = c->hard ? 0.0 : tanh_bound(Lv, v, eLv);
        put_leaf(c->leaf, c->eleaf, lp, Lu, eLu);
        put_leaf(c->leaf, c->eleaf, rp, Lv, eLv);
        log_sum_avoid_zero_nan(&Lu, &Lv, &top, 1);
        ret[0] = top;
        eret[0] = lse_bound(Lu, Lv, top, eLu, eLv);
        ret[1] = Lv;
        eret[1] = eLv;
        return;
    }
    float Lu[LSE_MAX_N / 2], Lhu[LSE_MAX_N / 2], Luv[LSE_MAX_N / 2], Lv[LSE_MAX_N / 2], Lhv[LSE_MAX_N / 2];
    double eLu[LSE_MAX_N / 2], eLhu[LSE_MAX_N / 2], eLv[LSE_MAX_N / 2], eLhv[LSE_MAX_N / 2];
    log_sum_avoid_zero_nan(llrs, llrs + half, Lu, half);
    for (int j = 0; j < half; ++j) eLu[j] = lse_bound(llrs[j], llrs[half + j], Lu[j], el[j], el[half + j]);
    softb_decode(c, Lu, eLu, depth + 1, 2 * bitpos, Lhu, eLhu);
    log_sum_avoid_zero_nan(Lhu, llrs, Luv, half);
    for (int j = 0; j < half; ++j) {
        const double e = lse_bound(Lhu[j], llrs[j], Luv[j], eLhu[j], el[j]);
        Lv[j] = Luv[j] + llrs[half + j];
        eLv[j] = add_bound(Luv[j], llrs[half + j], Lv[j], e, el[half + j]);
    }
    softb_decode(c, Lv, eLv, depth + 1, 2 * bitpos + 1, Lhv, eLhv);
    log_sum_avoid_zero_nan(Lhu, Lhv, ret, half);
    for (int j = 0; j < half; ++j) {
        eret[j] = lse_bound(Lhu[j], Lhv[j], ret[j], eLhu[j], eLhv[j]);
        ret[half + j] = Lhv[j];
        eret[half + j] = eLhv[j];
    }
}

void oracle_sc_decode_soft_bound(const float* y, int64_t B, int N, const float* priors, float llr_scale, int hard,
                                 int twice, float* bits_out, double* ebits_out, float* leaf_out, double* eleaf_out) {
    int n = 0;
    while ((1 << n) < N) ++n;
    float zeros[LSE_MAX_N] = {0};
    const float* pr = priors ? priors : zeros;
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < B; ++b) {
        float llr[LSE_MAX_N], ret[LSE_MAX_N];
        double el[LSE_MAX_N], eret[LSE_MAX_N];
        for (int i = 0; i < N; ++i) {
            llr[i] = llr_scale * y[b * N + i];
            el[i] = 0.0;
        }
        softb_ctx c = {n, pr, hard, bits_out + b * N, ebits_out + b * N, leaf_out ? leaf_out + b * N : NULL,
                       eleaf_out ? eleaf_out + b * N : NULL, twice};
        softb_decode(&c, llr, el, 0, 0, ret, eret);
    }
}
