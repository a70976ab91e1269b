// Internal helpers shared by the libvasr_hip.so translation units.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>

#include "../../include/vasr.h"

#define VASR_API extern "C" __attribute__((visibility("default")))

namespace vasr {

void set_error(const char* fmt, ...);
void clear_error();

// Record the launch status of the kernel just enqueued.
inline int launch_status(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: launch failed: %s", what, hipGetErrorString(e));
        return static_cast<int>(e);
    }
    return VASR_OK;
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

constexpr int kWave = 64;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}

// Exact (erf) GELU, nn.GELU() default.
__device__ __forceinline__ float gelu_erf(float x) {
    return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f));
}

// F.softplus(beta=1, threshold=20).
__device__ __forceinline__ float softplus20(float x) {
    return x > 20.0f ? x : log1pf(expf(x));
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

}  // namespace vasr

#define VASR_CHECK_ARG(cond, ...)            \
    do {                                     \
        if (!(cond)) {                       \
            ::vasr::set_error(__VA_ARGS__);  \
            return VASR_EINVAL;              \
        }                                    \
    } while (0)
