// Microbenchmark: VALU throughput of fp32 mul, packed mul, fma, exp on gfx950 (diagnostic).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));

template <int KIND>
__global__ __launch_bounds__(256) void k(float* out, float s, int iters) {
    float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7};
    const f2 ss = {s, s};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if constexpr (KIND == 0) {  // 8 independent v_mul_f32
                a0 *= s; a1 *= s; a2 *= s; a3 *= s; a4 *= s; a5 *= s; a6 *= s; a7 *= s;
            } else if constexpr (KIND == 1) {  // 4 independent v_pk_mul_f32 (8 flops-lanes)
                p0 *= ss; p1 *= ss; p2 *= ss; p3 *= ss;
            } else if constexpr (KIND == 2) {  // 8 independent v_fma_f32
                a0 = __builtin_fmaf(a0, s, s); a1 = __builtin_fmaf(a1, s, s); a2 = __builtin_fmaf(a2, s, s);
                a3 = __builtin_fmaf(a3, s, s); a4 = __builtin_fmaf(a4, s, s); a5 = __builtin_fmaf(a5, s, s);
                a6 = __builtin_fmaf(a6, s, s); a7 = __builtin_fmaf(a7, s, s);
            } else if constexpr (KIND == 3) {  // 8 independent v_exp_f32
                a0 = __builtin_amdgcn_exp2f(a0); a1 = __builtin_amdgcn_exp2f(a1); a2 = __builtin_amdgcn_exp2f(a2);
                a3 = __builtin_amdgcn_exp2f(a3); a4 = __builtin_amdgcn_exp2f(a4); a5 = __builtin_amdgcn_exp2f(a5);
                a6 = __builtin_amdgcn_exp2f(a6); a7 = __builtin_amdgcn_exp2f(a7);
            } else if constexpr (KIND == 4) {  // 4 v_pk_fma_f32
                p0 = p0 * ss + ss; p1 = p1 * ss + ss; p2 = p2 * ss + ss; p3 = p3 * ss + ss;
            } else {  // dependent chain of v_mul_f32 (latency)
                a0 *= s; a0 *= s; a0 *= s; a0 *= s; a0 *= s; a0 *= s; a0 *= s; a0 *= s;
            }
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + p0.x + p0.y + p1.x + p1.y + p2.x +
                                          p2.y + p3.x + p3.y;
}

template <int KIND>
double run(float* d, int blocks, int iters, int per_iter_instr, const char* name, double& ops_lane) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    k<KIND><<<blocks, 256>>>(d, 0.999f, iters);
    hipEventRecord(a);
    k<KIND><<<blocks, 256>>>(d, 0.999f, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    double instr = (double)blocks * 4 /*waves*/ * iters * 8 * per_iter_instr;
    double per_simd = instr / 1024.0;
    printf("%-28s blocks=%5d  %.3f ms  %.2f wave-instr/ns/chip  -> cycles per wave-instr per SIMD at 2.4GHz: %.2f\n",
           name, blocks, ms, instr / (ms * 1e6), (ms * 1e-3 * 2.4e9) / per_simd);
    return ms;
}

int main() {
    float* d;
    hipMalloc(&d, 1 << 24);
    double o;
    for (int blocks : {1024, 2048, 4096}) {
        run<0>(d, blocks, 2000, 8, "v_mul_f32 (indep x8)", o);
        run<1>(d, blocks, 2000, 4, "v_pk_mul_f32 (indep x4)", o);
        run<2>(d, blocks, 2000, 8, "v_fma_f32 (indep x8)", o);
        run<4>(d, blocks, 2000, 4, "v_pk_fma_f32 (indep x4)", o);
        run<3>(d, blocks, 2000, 8, "v_exp_f32 (indep x8)", o);
        run<5>(d, blocks, 2000, 8, "v_mul_f32 dependent chain", o);
    }
    return 0;
}
