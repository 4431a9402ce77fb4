// capi.cpp -- error reporting and version of the C ABI (include/dmdqn.h).
#include <stdarg.h>
#include <stdio.h>

#include "common.hpp"

namespace dmdqn {
static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}
}  // namespace dmdqn

extern "C" const char *dmdqn_last_error(void) { return dmdqn::g_err; }
extern "C" int dmdqn_version(void) { return 1; }

// A HIP stream whose kernels run only on the CUs set in `mask` (n_words
// 32-bit words, CU i = bit i % 32 of word i / 32): the trainer's side stream
// (act / sim / observe / sample of the next step) and the learn stream then
// split the chip instead of competing for the same CU slots.
extern "C" int dmdqn_stream_create_cumask(uint32_t n_words, const uint32_t *mask, void **out) {
    DMDQN_REQUIRE(n_words > 0 && mask && out, "dmdqn_stream_create_cumask: bad args");
    hipStream_t s = nullptr;
    const hipError_t e = hipExtStreamCreateWithCUMask(&s, n_words, mask);
    DMDQN_REQUIRE(e == hipSuccess, "hipExtStreamCreateWithCUMask: %s", hipGetErrorString(e));
    *out = s;
    return DMDQN_OK;
}

extern "C" int dmdqn_stream_destroy(void *stream) {
    DMDQN_REQUIRE(stream, "dmdqn_stream_destroy: null stream");
    const hipError_t e = hipStreamDestroy(reinterpret_cast<hipStream_t>(stream));
    DMDQN_REQUIRE(e == hipSuccess, "hipStreamDestroy: %s", hipGetErrorString(e));
    return DMDQN_OK;
}
