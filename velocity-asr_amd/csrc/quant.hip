// INT8 fake quantisation (BASELINE config C5, reference velocity_asr/quantize.py).
//
// At inference a calibrated FakeQuantize is a fixed elementwise map, so the model fuses the
// activation quantizers into the GEMM epilogues (gemm_common.h, qparams) and fake-quantizes
// each weight once per parameter version with fakequant_kernel.  minmax_kernel provides the
// range statistics calibration observes.  Both are HBM-bound streaming kernels: one wave per
// row, coalesced lanes along the row.
#include "vasr_internal.h"

namespace vasr {
namespace {

__global__ __launch_bounds__(256) void fakequant_kernel(const float* x, int64_t ldx, float* y, int64_t ldy,
                                                        int rows, int cols, const float* __restrict__ scale,
                                                        const float* __restrict__ zp, int per_row, float qmin,
                                                        float qmax) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const int lane = threadIdx.x & 63;
    const int qi = per_row ? row : 0;
    const float4 q = make_float4(scale[qi], zp[qi], qmin, qmax);
    const float* xr = x + (int64_t)row * ldx;
    float* yr = y + (int64_t)row * ldy;
    for (int c = lane; c < cols; c += 64) yr[c] = fake_quant(xr[c], q);
}

__device__ __forceinline__ float nan_min(float a, float b) { return (a != a || b != b) ? __builtin_nanf("") : fminf(a, b); }
__device__ __forceinline__ float nan_max(float a, float b) { return (a != a || b != b) ? __builtin_nanf("") : fmaxf(a, b); }

__global__ __launch_bounds__(256) void minmax_kernel(const float* __restrict__ x, int64_t ldx, int rows, int cols,
                                                     float* __restrict__ out_min, float* __restrict__ out_max) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const int lane = threadIdx.x & 63;
    const float* xr = x + (int64_t)row * ldx;
    float mn = __builtin_inff(), mx = -__builtin_inff();
    for (int c = lane; c < cols; c += 64) {
        const float v = xr[c];
        mn = nan_min(mn, v);
        mx = nan_max(mx, v);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mn = nan_min(mn, __shfl_xor(mn, o, kWave));
        mx = nan_max(mx, __shfl_xor(mx, o, kWave));
    }
    if (lane == 0) {
        out_min[row] = mn;
        out_max[row] = mx;
    }
}

}  // namespace
}  // namespace vasr

VASR_API int vasr_fakequant_f32(const float* x, int64_t ldx, float* y, int64_t ldy, int rows, int cols,
                                const float* scale, const float* zero_point, int per_row, float qmin, float qmax,
                                void* stream) {
    using namespace vasr;
    VASR_CHECK_ARG(x && y && scale && zero_point, "vasr_fakequant_f32: null pointer");
    VASR_CHECK_ARG(rows >= 0 && cols >= 0 && ldx >= cols && ldy >= cols, "vasr_fakequant_f32: bad shape");
    VASR_CHECK_ARG(qmin <= qmax, "vasr_fakequant_f32: qmin > qmax");
    if (rows == 0 || cols == 0) return VASR_OK;
    hipLaunchKernelGGL(fakequant_kernel, dim3((rows + 3) / 4), dim3(256), 0, as_stream(stream), x, ldx, y, ldy, rows,
                       cols, scale, zero_point, per_row, qmin, qmax);
    return launch_status("vasr_fakequant_f32");
}

VASR_API int vasr_minmax_f32(const float* x, int64_t ldx, int rows, int cols, float* out_min, float* out_max,
                             void* stream) {
    using namespace vasr;
    VASR_CHECK_ARG(x && out_min && out_max, "vasr_minmax_f32: null pointer");
    VASR_CHECK_ARG(rows >= 0 && cols > 0 && ldx >= cols, "vasr_minmax_f32: bad shape rows=%d cols=%d", rows, cols);
    if (rows == 0) return VASR_OK;
    hipLaunchKernelGGL(minmax_kernel, dim3((rows + 3) / 4), dim3(256), 0, as_stream(stream), x, ldx, rows, cols,
                       out_min, out_max);
    return launch_status("vasr_minmax_f32");
}
