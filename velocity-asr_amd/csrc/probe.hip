// vasr_probe_clock (include/vasr.h): which XCD each workgroup of a launch runs on, and the shader
// clock over a fixed VALU chain.  Diagnostic only: bench.py records it beside the timings so a
// slow run can be told apart as a lower clock or a different workgroup placement (the scan's
// XCD-aware block map, scan_body.inc, assumes workgroup i runs on XCD i % 8).
#include "vasr_internal.h"

namespace {

__global__ __launch_bounds__(256) void probe_clock_kernel(int64_t* __restrict__ out, int iters) {
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    float v0 = threadIdx.x * 1e-3f;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; ++i) v0 = __builtin_fmaf(v0, 0.9999f, 1e-4f);  // one dependent chain
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        out[3 * blockIdx.x] = (int64_t)(xcc & 0xF) + (v0 == -1.f ? 1 : 0);  // keeps the chain live
        out[3 * blockIdx.x + 1] = (int64_t)(t1 - t0);
        out[3 * blockIdx.x + 2] = (int64_t)(r1 - r0);
    }
}

}  // namespace

VASR_API int vasr_probe_clock(int64_t* out, int blocks, int iters, void* stream) {
    VASR_CHECK_ARG(out, "vasr_probe_clock: null out");
    VASR_CHECK_ARG(blocks > 0 && blocks <= 65536 && iters >= 0 && iters <= (1 << 24), "vasr_probe_clock: bad size");
    hipLaunchKernelGGL(probe_clock_kernel, dim3(blocks), dim3(256), 0, vasr::as_stream(stream), out, iters);
    return vasr::launch_status("vasr_probe_clock");
}
