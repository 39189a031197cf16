// Error reporting for the C ABI (ncn_last_error) and the library version.
#include <stdarg.h>
#include <stdio.h>
#include "common.h"

namespace ncn {
static thread_local char g_err[512] = "";
void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}
}  // namespace ncn

extern "C" const char* ncn_last_error(void) { return ncn::g_err; }
extern "C" int ncn_version(void) { return 1; }
