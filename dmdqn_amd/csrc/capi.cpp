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

// per-source-file debug flags (common.hpp DMDQN_DBG_READER)
int dbg_flags_sim();
int dbg_flags_rng();
int dbg_flags_learn();
namespace f16k { int dbg_flags(); }
namespace bf16k { int dbg_flags(); }
}  // namespace dmdqn

extern "C" int dmdqn_debug_status(void) {
    using namespace dmdqn;
    const int f[5] = {dbg_flags_sim(), dbg_flags_rng(), dbg_flags_learn(), f16k::dbg_flags(),
                      bf16k::dbg_flags()};
    int v = 0;
    for (int x : f) {
        if (x < 0) return -1;
        v |= x;
    }
    return v;
}

extern "C" int dmdqn_debug_build(void) {
#ifdef DMDQN_DEBUG_BOUNDS
    return 1;
#else
    return 0;
#endif
}

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
