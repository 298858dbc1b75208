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

static inline float decide(const lse_ctx* c, float L) { return c->hard ? sgn(L) : tanhf(L / 2.0f); }

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

/* ------------------------------------------------------------------ soft SC (polar.py:281-358) */
static inline float clamp1000(float x) { return x < -1000.0f ? -1000.0f : (x > 1000.0f ? 1000.0f : x); }

typedef struct {
    int n;
    const float* prior;
    int hard;
    float* bits;
} soft_ctx;

/* decode_soft(llrs, depth, bit_position, prior) (polar.py:305-358); ret = returned LLR vector (2*half) */
static void soft_decode(soft_ctx* c, const float* llrs, int depth, int bitpos, float* ret) {
    const int half = 1 << (c->n - depth - 1);
    if (depth == c->n - 1) {
        const int lp = 2 * bitpos, rp = 2 * bitpos + 1;
        float Lu, Luv, Lv, top;
        log_sum_avoid_zero_nan(&llrs[0], &llrs[1], &Lu, 1);
        Lu = clamp1000(Lu + c->prior[lp] * 1.0f);
        float u = c->hard ? sgn(Lu) : tanhf(Lu / 2.0f);
        log_sum_avoid_zero_nan(&Lu, &llrs[0], &Luv, 1);
        Lv = Luv + llrs[1];
        Lv = clamp1000(Lv + c->prior[rp] * 1.0f);
        float v = c->hard ? sgn(Lv) : tanhf(Lv / 2.0f);
        c->bits[lp] = u;
        c->bits[rp] = v;
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

/* PolarCode.sc_decode_soft(y, snr, priors): msg_hat = sign(decoded_bits)[:, info]; priors (N) or NULL */
void oracle_sc_decode_soft(const float* y, int64_t B, int N, int K, const int32_t* info, const float* priors,
                           float llr_scale, int hard, float* msg_hat, float* bits_out) {
    int n = 0;
    while ((1 << n) < N) ++n;
    float zeros[LSE_MAX_N] = {0};
    const float* pr = priors ? priors : zeros;
#pragma omp parallel for schedule(static)
    for (int64_t b = 0; b < B; ++b) {
        float llr[LSE_MAX_N], bits[LSE_MAX_N], ret[LSE_MAX_N];
        for (int i = 0; i < N; ++i) llr[i] = llr_scale * y[b * N + i];
        soft_ctx c = {n, pr, hard, bits};
        soft_decode(&c, llr, 0, 0, ret);
        if (bits_out) memcpy(bits_out + b * N, bits, sizeof(float) * (size_t)N);
        if (msg_hat)
            for (int k = 0; k < K; ++k) msg_hat[b * K + k] = sgn(bits[info[k]]);
    }
}
