// Microbenchmark: sustained bf16 MFMA rate and shader clock on gfx950 (diagnostic).
// Every wave issues back-to-back v_mfma_f32_32x32x16_bf16 on 4 independent accumulators;
// clock = d(s_memtime) / d(s_memrealtime) x 100 MHz, measured inside the kernel.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(256) void k(float* out, unsigned long long* clk, int iters) {
    bf16x8 a, b;
    for (int j = 0; j < 8; ++j) {
        a[j] = (__bf16)(threadIdx.x * 1e-3f + j);
        b[j] = (__bf16)(j * 0.5f);
    }
    floatx16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; ++i) {
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c3, 0, 0, 0);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.f;
    for (int j = 0; j < 16; ++j) s += c0[j] + c1[j] + c2[j] + c3[j];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

int main() {
    const int blocks = 256 * 2, iters = 20000;
    float* out;
    unsigned long long* clk;
    hipMalloc(&out, blocks * 256 * 4);
    hipMalloc(&clk, blocks * 16);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, clk, 100);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, clk, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        std::vector<unsigned long long> h(blocks * 2);
        hipMemcpy(h.data(), clk, blocks * 16, hipMemcpyDeviceToHost);
        std::vector<double> mhz;
        for (int b = 0; b < blocks; ++b) mhz.push_back(100.0 * h[2 * b] / std::max(1ull, h[2 * b + 1]));
        std::sort(mhz.begin(), mhz.end());
        const double flops = 2.0 * 32 * 32 * 16 * 4.0 * iters * 4 /*waves*/ * blocks;
        printf("rep %d: %.3f ms, %.0f TFLOP/s bf16, in-kernel clock median %.0f MHz (min %.0f, max %.0f)\n", rep, ms,
               flops / ms / 1e9, mhz[blocks / 2], mhz[0], mhz[blocks - 1]);
    }
    return 0;
}
