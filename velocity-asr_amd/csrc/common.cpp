// Error state and version entry points of libvasr_hip.so.
#include <cstring>
#include <string>

#include "vasr_internal.h"

namespace vasr {

static thread_local char g_last_error[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
    va_end(ap);
}

void clear_error() { g_last_error[0] = '\0'; }

}  // namespace vasr

VASR_API int vasr_version(void) { return VASR_ABI_VERSION; }

VASR_API const char* vasr_last_error(void) { return vasr::g_last_error; }
