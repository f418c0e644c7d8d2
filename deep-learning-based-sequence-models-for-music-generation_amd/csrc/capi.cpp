// Error plumbing + version of the libmidiseq C ABI (include/midiseq.h).
#include <stdarg.h>
#include <stdio.h>

#include "../../include/midiseq.h"

static thread_local char g_err[512] = "";

int msq_set_error(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

extern "C" const char* msq_last_error(void) { return g_err; }

extern "C" int msq_version(void) { return 1; }
