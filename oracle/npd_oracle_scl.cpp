// npd_oracle_scl.cpp -- TEST INFRASTRUCTURE ONLY (imported by tests/, smoke(), bench cpu_baseline).
//
// CPU restatement of PolarCode.scl_decode (polar.py:793-876, use_CRC=False) with pruneLists
// (polar.py:777-791).  Written step by step like the reference: every leaf re-runs partial_decode
// (polar.py:380-456) from the root on each path's own (n+1) x N LLR / partial-sum arrays and
// updatePartialSums (polar.py:458-470) rebuilds the partial sums, so nothing here shares code or
// structure with the GPU kernel.
//
// Pruning: torch.topk(-metric, L, dim=0) on CPU (ATen TopKImpl.h, k*64 > n) is std::nth_element with
// the comparator `isnan(x) && !isnan(y) || x > y` over (value, index) pairs in list order, followed by a
// sort of the surviving indices (polar.py:779).  We call libstdc++'s std::nth_element itself, so ties
// resolve exactly as the reference's.  tests/test_oracle_golden.py checks this against torch.topk.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <utility>
#include <vector>

namespace {

inline float sgnf(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }

// utils.py:272-275 min_sum_log_sum_exp: sign(a) sign(b) min(|a|, |b|)
inline float f_minsum(float a, float b) { return sgnf(a) * sgnf(b) * std::fmin(std::fabs(a), std::fabs(b)); }

struct Path {
    std::vector<float> llr;  // (n+1) x N, level d at [d*N, (d+1)*N)
    std::vector<float> ps;   // partial sums, same shape
    std::vector<float> u;    // N decisions (u_hat_list row)
    float metric = 0.0f;
};

struct Ctx {
    int N, n;
};

// polar.py:380-456 (partial_decode), prior = zeros (scl_decode adds the frozen prior itself)
void partial_decode(const Ctx& c, Path& p, int depth, int bit_position, int leaf) {
    const int N = c.N;
    const int half = 1 << (depth - 1);
    const int at_depth = leaf >> (depth - 1);
    float* L = p.llr.data();
    const float* P = p.ps.data();
    const int left = 2 * bit_position, right = left + 1;
    if (depth == 1) {
        float u_hat = 0.0f;
        if (at_depth > left) {
            u_hat = P[0 * N + left];
        } else if (at_depth == left) {
            const float Lu = f_minsum(L[1 * N + left * half], L[1 * N + (left + 1) * half]);
            L[0 * N + left * half] = Lu + 0.0f;
            return;
        }
        if (at_depth == right) {
            const float Lv = u_hat * L[1 * N + left * half] + L[1 * N + (left + 1) * half];
            L[0 * N + right * half] = Lv + 0.0f;
        }
        return;
    }
    if (at_depth > left) {
        // Lu = stored level depth-1 values; u_hat = partial sums of the finished left block
        for (int j = 0; j < half; ++j) {
            const float u = P[(depth - 1) * N + left * half + j];
            const float Lv = u * L[depth * N + left * half + j] + L[depth * N + (left + 1) * half + j];
            L[(depth - 1) * N + right * half + j] = Lv;
        }
        partial_decode(c, p, depth - 1, right, leaf);
        return;
    }
    for (int j = 0; j < half; ++j)
        L[(depth - 1) * N + left * half + j] = f_minsum(L[depth * N + left * half + j], L[depth * N + (left + 1) * half + j]);
    partial_decode(c, p, depth - 1, left, leaf);
}

// polar.py:458-470 (updatePartialSums)
void update_partial_sums(const Ctx& c, Path& p, int leaf) {
    const int N = c.N;
    std::vector<float> u(p.u);
    for (int i = leaf + 1; i < N; ++i) u[i] = 0.0f;
    for (int d = 0; d < c.n; ++d) {
        std::memcpy(&p.ps[d * N], u.data(), sizeof(float) * N);
        const int nb = 1 << d;
        for (int i = 0; i < N; i += 2 * nb)
            for (int j = 0; j < nb; ++j) u[i + j] = u[i + j] * u[i + nb + j];
    }
    std::memcpy(&p.ps[c.n * N], u.data(), sizeof(float) * N);
}

// polar.py:128-148 encode_plotkin of one row (frozen = +1)
void encode_row(const float* u_in, float* x, int N) {
    std::memcpy(x, u_in, sizeof(float) * N);
    for (int nb = 1; nb < N; nb *= 2)
        for (int i = 0; i < N; i += 2 * nb)
            for (int j = 0; j < nb; ++j) x[i + j] = x[i + j] * x[i + nb + j];
}

typedef std::pair<double, int64_t> elem_t;

}  // namespace

extern "C" {

// Exact ATen CPU topk selection (largest, k <= n, k*64 > n): the surviving indices after
// std::nth_element, in queue order.  Exposed so tests can pin it against torch.topk directly.
void oracle_topk_nth(const float* vals, int n, int k, int64_t* out_idx) {
    std::vector<elem_t> q(n);
    for (int j = 0; j < n; ++j) q[j] = elem_t((double)vals[j], j);
    std::nth_element(q.begin(), q.begin() + k - 1, q.end(), [](const elem_t& x, const elem_t& y) {
        return (std::isnan(x.first) && !std::isnan(y.first)) || (x.first > y.first);
    });
    for (int j = 0; j < k; ++j) out_idx[j] = q[j].second;
}

// y (B,N) channel output; info sorted ascending; frozen[N] flags; llr_scale = fl32(2/sigma^2).
// Outputs: leaf_llr (B,N) or null, msg_hat (B,K), u_hat (B,N) or null.
void oracle_scl_decode(const float* y, int64_t B, int N, int K, const int32_t* info, const uint8_t* frozen,
                       float llr_scale, int L, float infty, float* leaf_llr, float* msg_hat, float* u_hat) {
    Ctx c;
    c.N = N;
    c.n = 0;
    while ((1 << c.n) < N) ++c.n;
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t b = 0; b < B; ++b) {
        const float* yr = y + b * N;
        std::vector<Path> list(1);
        list[0].llr.assign((size_t)(c.n + 1) * N, 0.0f);
        list[0].ps.assign((size_t)(c.n + 1) * N, 0.0f);
        list[0].u.assign(N, 0.0f);
        for (int i = 0; i < N; ++i) list[0].llr[(size_t)c.n * N + i] = llr_scale * yr[i];  // polar.py:796
        for (int ii = 0; ii < N; ++ii) {
            const size_t s = list.size();
            for (auto& p : list) partial_decode(c, p, c.n, 0, ii);
            if (frozen[ii]) {
                for (auto& p : list) {
                    const float l = p.llr[ii];
                    const float pen = std::fabs(l) * (sgnf(l) != 1.0f ? 1.0f : 0.0f);  // polar.py:814
                    p.llr[ii] = l + infty * 1.0f;                                       // polar.py:816
                    p.u[ii] = 1.0f;
                    update_partial_sums(c, p, ii);
                    p.metric = p.metric + pen;
                }
            } else {
                std::vector<Path> grown(2 * s);
                for (size_t j = 0; j < s; ++j) {
                    const float l = list[j].llr[ii];
                    grown[j] = list[j];
                    grown[s + j] = list[j];
                    grown[j].u[ii] = sgnf(l);
                    grown[s + j].u[ii] = -1.0f * sgnf(l);
                    grown[s + j].metric = list[j].metric + std::fabs(l);  // polar.py:843
                    update_partial_sums(c, grown[j], ii);
                    update_partial_sums(c, grown[s + j], ii);
                }
                if ((int)grown.size() > L) {  // pruneLists, polar.py:777-791
                    std::vector<float> negm(grown.size());
                    for (size_t j = 0; j < grown.size(); ++j) negm[j] = -1.0f * grown[j].metric;
                    std::vector<int64_t> keep(L);
                    oracle_topk_nth(negm.data(), (int)grown.size(), L, keep.data());
                    std::sort(keep.begin(), keep.end());
                    std::vector<Path> pruned(L);
                    for (int j = 0; j < L; ++j) pruned[j] = grown[keep[j]];
                    list.swap(pruned);
                } else {
                    list.swap(grown);
                }
            }
        }
        // ML choice among the list (polar.py:868-874): argmin of squared distance to y, first index on ties
        std::vector<float> x(N), uu(N);
        int best = 0;
        float bestd = 0.0f;
        for (size_t j = 0; j < list.size(); ++j) {
            for (int i = 0; i < N; ++i) uu[i] = 1.0f;
            for (int k = 0; k < K; ++k) uu[info[k]] = list[j].u[info[k]];
            encode_row(uu.data(), x.data(), N);
            float d = 0.0f;
            for (int i = 0; i < N; ++i) {
                const float t = x[i] - yr[i];
                const float t2 = t * t;
                d = d + t2;
            }
            if (j == 0 || d < bestd) {
                best = (int)j;
                bestd = d;
            }
        }
        const Path& w = list[best];
        for (int k = 0; k < K; ++k) msg_hat[b * K + k] = w.u[info[k]];
        if (u_hat)
            for (int i = 0; i < N; ++i) u_hat[b * N + i] = w.u[i];
        if (leaf_llr)
            for (int i = 0; i < N; ++i) leaf_llr[b * N + i] = w.llr[i];
    }
}

}  // extern "C"
