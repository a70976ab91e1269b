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

// A stream whose kernels run only on the CUs set in `mask` (bit i = logical CU i, `words`
// uint32 words), on the current device: lets two independent utterance groups each own part
// of the chip instead of competing for every CU.
VASR_API int vasr_stream_create_cu_mask(const uint32_t* mask, int words, void** stream_out) {
    VASR_CHECK_ARG(mask && words > 0 && stream_out, "vasr_stream_create_cu_mask: bad arguments");
    hipStream_t s = nullptr;
    const hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask);
    if (e != hipSuccess) {
        vasr::set_error("vasr_stream_create_cu_mask: %s", hipGetErrorString(e));
        return (int)e;
    }
    *stream_out = s;
    return VASR_OK;
}

VASR_API int vasr_stream_destroy(void* stream) {
    const hipError_t e = hipStreamDestroy(reinterpret_cast<hipStream_t>(stream));
    if (e != hipSuccess) {
        vasr::set_error("vasr_stream_destroy: %s", hipGetErrorString(e));
        return (int)e;
    }
    return VASR_OK;
}

VASR_API int vasr_device_cu_count(void) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -1;
    return n;
}
