// capi.cpp -- error reporting and version of the C ABI (include/dmdqn.h).
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "common.hpp"

namespace dmdqn {
static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

// Run-time options (dmdqn.h DMDQN_OPT_*), from the environment at load time.
static int g_opt[2] = {0, 32};

__attribute__((constructor)) static void read_options() {
    const char *p = getenv("DMDQN_SIM_PATH");
    if (p) g_opt[DMDQN_OPT_SIM_PATH] = !strcmp(p, "reg") ? 1 : !strcmp(p, "lds") ? 2
                                       : !strcmp(p, "global") ? 3 : 0;
    const char *t = getenv("DMDQN_SAMPLE_TLOG");
    if (t && atoi(t) >= 0 && atoi(t) <= 20) g_opt[DMDQN_OPT_SAMPLE_TLOG] = atoi(t);
}

int option(int which) { return g_opt[which]; }

// per-source-file debug flags (common.hpp DMDQN_DBG_READER)
int dbg_flags_sim();
int dbg_flags_rng();
int dbg_flags_learn();
int dbg_flags_replay();
namespace f16k { int dbg_flags(); }
namespace bf16k { int dbg_flags(); }
}  // namespace dmdqn

extern "C" int dmdqn_debug_status(void) {
    using namespace dmdqn;
    const int f[6] = {dbg_flags_sim(), dbg_flags_rng(), dbg_flags_learn(), f16k::dbg_flags(),
                      bf16k::dbg_flags(), dbg_flags_replay()};
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

extern "C" int dmdqn_set_option(int opt, int value) {
    DMDQN_REQUIRE(opt == DMDQN_OPT_SIM_PATH || opt == DMDQN_OPT_SAMPLE_TLOG,
                  "dmdqn_set_option: unknown option %d", opt);
    DMDQN_REQUIRE(opt != DMDQN_OPT_SIM_PATH || (value >= 0 && value <= 3),
                  "dmdqn_set_option: sim path %d (0 auto, 1 reg, 2 lds, 3 global)", value);
    DMDQN_REQUIRE(opt != DMDQN_OPT_SAMPLE_TLOG || (value >= 0 && value <= 20) || value == 32,
                  "dmdqn_set_option: sample tlog %d (0 .. 20, or 32 = no cap)", value);
    dmdqn::g_opt[opt] = value;
    return DMDQN_OK;
}

extern "C" int dmdqn_get_option(int opt) {
    DMDQN_REQUIRE(opt == DMDQN_OPT_SIM_PATH || opt == DMDQN_OPT_SAMPLE_TLOG,
                  "dmdqn_get_option: unknown option %d", opt);
    return dmdqn::g_opt[opt];
}

extern "C" const char *dmdqn_last_error(void) { return dmdqn::g_err; }
extern "C" int dmdqn_version(void) { return 4; }  // include/dmdqn.h

extern "C" int dmdqn_device_lds_per_cu(int device, size_t *out) {
    DMDQN_REQUIRE(out && device >= 0, "dmdqn_device_lds_per_cu: bad args");
    int v = 0;
    const hipError_t e =
        hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, device);
    if (e != hipSuccess) {
        dmdqn::set_error("hipDeviceGetAttribute(MaxSharedMemoryPerMultiprocessor): %s",
                         hipGetErrorString(e));
        return DMDQN_EHIP;
    }
    *out = (size_t)v;
    return DMDQN_OK;
}

namespace dmdqn {
// The current device's per-workgroup LDS limit, cached per device (the
// sampler's budget is clamped to it); 160 KB if the query fails.
size_t device_lds_per_block() {
    static size_t cache[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 160 * 1024;
    if (!cache[dev]) {
        int v = 0;
        cache[dev] = hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) ==
                                 hipSuccess && v > 0
                         ? (size_t)v
                         : 160 * 1024;
    }
    return cache[dev];
}
}  // namespace dmdqn

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

// Timing events without the system-scope fence (include/dmdqn.h): bench.py
// brackets every learn launch with two of them.
extern "C" int dmdqn_timing_event_create(void **out) {
    DMDQN_REQUIRE(out, "dmdqn_timing_event_create: null out");
    hipEvent_t ev = nullptr;
    const hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableSystemFence);
    DMDQN_REQUIRE(e == hipSuccess, "hipEventCreateWithFlags: %s", hipGetErrorString(e));
    *out = ev;
    return DMDQN_OK;
}

extern "C" int dmdqn_order_event_create(void **out) {
    DMDQN_REQUIRE(out, "dmdqn_order_event_create: null out");
    hipEvent_t ev = nullptr;
    const hipError_t e =
        hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventDisableSystemFence);
    DMDQN_REQUIRE(e == hipSuccess, "hipEventCreateWithFlags: %s", hipGetErrorString(e));
    *out = ev;
    return DMDQN_OK;
}

extern "C" int dmdqn_stream_wait_event(void *stream, void *event) {
    DMDQN_REQUIRE(event, "dmdqn_stream_wait_event: null event");
    const hipError_t e = hipStreamWaitEvent(reinterpret_cast<hipStream_t>(stream),
                                            reinterpret_cast<hipEvent_t>(event), 0);
    DMDQN_REQUIRE(e == hipSuccess, "hipStreamWaitEvent: %s", hipGetErrorString(e));
    return DMDQN_OK;
}

extern "C" int dmdqn_event_record(void *event, void *stream) {
    DMDQN_REQUIRE(event, "dmdqn_event_record: null event");
    const hipError_t e = hipEventRecord(reinterpret_cast<hipEvent_t>(event),
                                        reinterpret_cast<hipStream_t>(stream));
    DMDQN_REQUIRE(e == hipSuccess, "hipEventRecord: %s", hipGetErrorString(e));
    return DMDQN_OK;
}

extern "C" int dmdqn_event_synchronize(void *event) {
    DMDQN_REQUIRE(event, "dmdqn_event_synchronize: null event");
    const hipError_t e = hipEventSynchronize(reinterpret_cast<hipEvent_t>(event));
    DMDQN_REQUIRE(e == hipSuccess, "hipEventSynchronize: %s", hipGetErrorString(e));
    return DMDQN_OK;
}

extern "C" int dmdqn_event_elapsed_ms(void *start, void *end, float *ms) {
    DMDQN_REQUIRE(start && end && ms, "dmdqn_event_elapsed_ms: null argument");
    const hipError_t e = hipEventElapsedTime(ms, reinterpret_cast<hipEvent_t>(start),
                                             reinterpret_cast<hipEvent_t>(end));
    DMDQN_REQUIRE(e == hipSuccess, "hipEventElapsedTime: %s", hipGetErrorString(e));
    return DMDQN_OK;
}

extern "C" int dmdqn_event_destroy(void *event) {
    DMDQN_REQUIRE(event, "dmdqn_event_destroy: null event");
    const hipError_t e = hipEventDestroy(reinterpret_cast<hipEvent_t>(event));
    DMDQN_REQUIRE(e == hipSuccess, "hipEventDestroy: %s", hipGetErrorString(e));
    return DMDQN_OK;
}
