// npd_api.hip -- error plumbing, device queries and code handles (host side of the C ABI).
#include <string.h>

#include <mutex>
#include <new>
#include <string>

#include "npd_common.hpp"

namespace npd {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
    set_error(msg);
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return (int)e;
}

int device_cu_count() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    static int cached[64] = {0};
    if (dev >= 0 && dev < 64 && cached[dev]) return cached[dev];
    int cu = 256;
    if (hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cu <= 0) cu = 256;
    if (dev >= 0 && dev < 64) cached[dev] = cu;
    return cu;
}

}  // namespace npd

extern "C" {

int npd_abi_version(void) { return NPD_ABI_VERSION; }

const char* npd_last_error(void) { return npd::g_last_error.c_str(); }

int npd_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

int npd_code_create(int N, int K, const int32_t* info_sorted, int pac_g, float infty, npd_code** out) {
    NPD_ARG(out != nullptr, "npd_code_create: out is NULL");
    *out = nullptr;
    NPD_ARG(N >= 4 && N <= npd::kMaxN && (N & (N - 1)) == 0, "npd_code_create: N must be a power of two in [4, 256]");
    NPD_ARG(K >= 0 && K <= N, "npd_code_create: K must be in [0, N]");
    NPD_ARG(K == 0 || info_sorted != nullptr, "npd_code_create: info_sorted is NULL");
    npd_code* c = new (std::nothrow) npd_code;
    if (!c) return npd::fail(NPD_ENOMEM, "npd_code_create: out of memory");
    memset(c, 0, sizeof(*c));
    npd::CodeParams& p = c->p;
    p.N = N;
    p.K = K;
    p.n = 0;
    while ((1 << p.n) < N) ++p.n;
    p.infty = infty;
    for (int w = 0; w < npd::kMaxWords; ++w) p.frozen[w] = 0;
    for (int i = 0; i < N; ++i) p.frozen[i >> 5] |= 1u << (i & 31);
    int prev = -1;
    for (int k = 0; k < K; ++k) {
        const int i = info_sorted[k];
        if (i <= prev || i >= N) {
            delete c;
            return npd::fail(NPD_EINVAL, "npd_code_create: info positions must be strictly increasing in [0, N)");
        }
        prev = i;
        p.info[k] = i;
        p.rank[i] = (uint32_t)k;
        p.frozen[i >> 5] &= ~(1u << (i & 31));
    }
    for (int D = 1; D <= p.n; ++D)
        for (int s0 = 0; s0 < N; s0 += 1 << D) {
            int k = 0;
            for (int i = s0; i < s0 + (1 << D); ++i) k += ((p.frozen[i >> 5] >> (i & 31)) & 1u) ? 0 : 1;
            const bool last_info = !((p.frozen[(s0 + (1 << D) - 1) >> 5] >> ((s0 + (1 << D) - 1) & 31)) & 1u);
            uint32_t t = npd::kNodeMixed;
            if (k == 0) t = npd::kNodeRate0;
            else if (k == (1 << D)) t = npd::kNodeRate1;
            else if (k == 1 && last_info) t = npd::kNodeRep;
            const int id = (N >> D) + (s0 >> D);
            p.ntype[id >> 4] |= t << (2 * (id & 15));
        }
    if (pac_g != 0) {
        NPD_ARG(pac_g > 1, "npd_code_create: invalid PAC polynomial");
        int M = 0;
        while ((pac_g >> M) != 0) ++M;  // bit count; top bit (g_array[0] = -1) always set
        const int state_len = M - 1;
        if (state_len > 30) {
            delete c;
            return npd::fail(NPD_EINVAL, "npd_code_create: PAC polynomial too long");
        }
        uint32_t tap = 0;
        for (int j = 1; j < M; ++j)  // g_array[j] = 1 - 2*bit_j (MSB first), tap iff g_array[j] == -1
            if ((pac_g >> (M - 1 - j)) & 1) tap |= 1u << (j - 1);
        p.pac = 1;
        p.tapmask = tap;
        p.smask = (1u << state_len) - 1u;
    }
    if (hipGetDevice(&c->device) != hipSuccess) {
        (void)hipGetLastError();
        c->device = -1;
    }
    *out = c;
    return NPD_OK;
}

int npd_code_destroy(npd_code* code) {
    delete code;
    return NPD_OK;
}

}  // extern "C"
