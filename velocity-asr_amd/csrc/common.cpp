// Error state, version and tuning-option entry points of libvasr_hip.so.
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>
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

// Tuning options (vasr_set_option): process-wide, defaults from the environment read once.
namespace {
constexpr int kNumOptions = 7;
const char* const kOptionEnv[kNumOptions] = {"VASR_SCAN_NPL", "VASR_SCAN_T", "VASR_TAIL_ROWS", "VASR_GEMM_ENGINE",
                                               "VASR_TAIL_WAVES", "VASR_SCAN_SPLIT", "VASR_DW_ROWS"};
const int kOptionValues[kNumOptions][4] = {{0, 2, 4, -1}, {0, 16, 32, -1}, {0, 16, 32, -1},
                                           {0, 1, 2, -1}, {0, 4, 6, 12},   {0, 1, 2, -1}, {0, 4, 8, 16}};
std::atomic<int> g_options[kNumOptions];
std::once_flag g_options_once;

bool option_value_ok(int key, int v) {
    for (int a : kOptionValues[key])
        if (a >= 0 && v == a) return true;
    return false;
}

void options_init() {
    std::call_once(g_options_once, [] {
        for (int k = 0; k < kNumOptions; ++k) {
            const char* e = std::getenv(kOptionEnv[k]);
            const int v = e ? std::atoi(e) : 0;
            g_options[k].store(option_value_ok(k, v) ? v : 0, std::memory_order_relaxed);
        }
    });
}
}  // namespace

namespace vasr {
int option(int key) {
    options_init();
    return g_options[key].load(std::memory_order_relaxed);
}
}  // namespace vasr

VASR_API int vasr_set_option(int key, int value) {
    VASR_CHECK_ARG(key >= 0 && key < kNumOptions, "vasr_set_option: unknown option %d", key);
    options_init();
    if (value < 0) return g_options[key].load(std::memory_order_relaxed);
    VASR_CHECK_ARG(option_value_ok(key, value), "vasr_set_option: value %d not allowed for option %d", value, key);
    return g_options[key].exchange(value, std::memory_order_relaxed);
}
