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
