#include "build_hash.h"
#include <stdarg.h>
#include <stdio.h>
static thread_local char g_err[1024] = "";
void srnn_set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}
extern "C" const char* srnn_last_error() { return g_err; }
extern "C" int srnn_abi_version() { return 1; }
// csrc/srchash.py's hash of the sources this library was compiled from (samplernn_hip.lib()
// compares it with the tree's)
extern "C" const char* srnn_build_hash() { return SRNN_BUILD_HASH; }
