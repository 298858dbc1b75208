// npd_stub.hip -- temporary: GRU / conv entry points before their kernels land.
#include "npd_common.hpp"

extern "C" {
int npd_conv_create(int, int, const float*, int64_t, int, npd_conv** out) {
    if (out) *out = nullptr;
    return npd::fail(NPD_ENOTSUP, "npd_conv_create: not built yet");
}
int npd_conv_destroy(npd_conv*) { return NPD_OK; }
int64_t npd_conv_workspace_bytes(const npd_conv*, int64_t) { return 0; }
int npd_conv_forward(const npd_conv*, const float*, float*, float*, void*, int64_t, void*) {
    return npd::fail(NPD_ENOTSUP, "npd_conv_forward: not built yet");
}
}
