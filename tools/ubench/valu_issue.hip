// Microbenchmark (diagnostic): VALU issue cost and dependent-issue latency on gfx950, with the
// instructions pinned by inline asm (the compiler cannot re-pack or fuse them), and whether
// v_exp_f32 overlaps independent packed VALU work of the same wave.
// Build: hipcc --offload-arch=gfx950 -O3 valu_issue.hip -o valu_issue
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));

#define MUL(x) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x) : "v"(s))
#define FMA(x) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"(s))
#define PKMUL(x) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(x) : "v"(ss))
#define PKFMA(x) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"(ss))
#define EXP(x) asm volatile("v_exp_f32 %0, %0" : "+v"(x))

template <int KIND>
__global__ __launch_bounds__(256) void k(float* out, float s, int iters) {
    float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
          a7 = a0 + 7;
    f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}, p4 = p0 + 1.f, p5 = p1 + 1.f, p6 = p2 + 1.f,
       p7 = p3 + 1.f;
    const f2 ss = {s, s};
    for (int i = 0; i < iters; ++i) {
        if constexpr (KIND == 0) {  // 8 independent v_mul_f32
            MUL(a0); MUL(a1); MUL(a2); MUL(a3); MUL(a4); MUL(a5); MUL(a6); MUL(a7);
        } else if constexpr (KIND == 1) {  // 8 independent v_fma_f32
            FMA(a0); FMA(a1); FMA(a2); FMA(a3); FMA(a4); FMA(a5); FMA(a6); FMA(a7);
        } else if constexpr (KIND == 2) {  // 8 independent v_pk_mul_f32
            PKMUL(p0); PKMUL(p1); PKMUL(p2); PKMUL(p3); PKMUL(p4); PKMUL(p5); PKMUL(p6); PKMUL(p7);
        } else if constexpr (KIND == 3) {  // 8 independent v_pk_fma_f32
            PKFMA(p0); PKFMA(p1); PKFMA(p2); PKFMA(p3); PKFMA(p4); PKFMA(p5); PKFMA(p6); PKFMA(p7);
        } else if constexpr (KIND == 4) {  // 8 independent v_exp_f32
            EXP(a0); EXP(a1); EXP(a2); EXP(a3); EXP(a4); EXP(a5); EXP(a6); EXP(a7);
        } else if constexpr (KIND == 5) {  // 4 exp + 4 pk_fma interleaved, independent
            EXP(a0); PKFMA(p0); EXP(a1); PKFMA(p1); EXP(a2); PKFMA(p2); EXP(a3); PKFMA(p3);
        } else if constexpr (KIND == 6) {  // 2 exp + 6 pk_fma
            EXP(a0); PKFMA(p0); PKFMA(p1); PKFMA(p2); EXP(a1); PKFMA(p3); PKFMA(p4); PKFMA(p5);
        } else if constexpr (KIND == 7) {  // 4 exp + 4 v_fma interleaved
            EXP(a0); FMA(a4); EXP(a1); FMA(a5); EXP(a2); FMA(a6); EXP(a3); FMA(a7);
        } else if constexpr (KIND == 8) {  // dependent chain of v_mul_f32
            MUL(a0); MUL(a0); MUL(a0); MUL(a0); MUL(a0); MUL(a0); MUL(a0); MUL(a0);
        } else if constexpr (KIND == 9) {  // dependent chain of v_pk_fma_f32
            PKFMA(p0); PKFMA(p0); PKFMA(p0); PKFMA(p0); PKFMA(p0); PKFMA(p0); PKFMA(p0); PKFMA(p0);
        } else if constexpr (KIND == 10) {  // dependent chain of v_exp_f32
            EXP(a0); EXP(a0); EXP(a0); EXP(a0); EXP(a0); EXP(a0); EXP(a0); EXP(a0);
        } else if constexpr (KIND == 11) {  // two interleaved dependent pk_fma chains
            PKFMA(p0); PKFMA(p1); PKFMA(p0); PKFMA(p1); PKFMA(p0); PKFMA(p1); PKFMA(p0); PKFMA(p1);
        } else if constexpr (KIND == 12) {  // four interleaved dependent pk_fma chains
            PKFMA(p0); PKFMA(p1); PKFMA(p2); PKFMA(p3); PKFMA(p0); PKFMA(p1); PKFMA(p2); PKFMA(p3);
        } else if constexpr (KIND == 13) {  // exp feeding a pk_mul (the dA -> tree dependence), 2 chains
            EXP(a0); EXP(a1); p0.x = a0; p1.x = a1; PKMUL(p0); PKMUL(p1); a0 = p0.y; a1 = p1.y;
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + p0.x + p0.y + p1.x + p1.y + p2.x +
                                          p2.y + p3.x + p3.y + p4.x + p5.y + p6.x + p7.y;
}

template <int KIND>
void run(float* d, int blocks, int iters, const char* name) {
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
    const double waves_per_simd = blocks * 4.0 / 1024.0;
    const double instr_per_simd = waves_per_simd * iters * 8.0;
    printf("%-34s waves/SIMD %4.1f  %.3f ms  cycles per wave-instr per SIMD (2.4 GHz): %.2f\n", name, waves_per_simd,
           ms, (ms * 1e-3 * 2.4e9) / instr_per_simd);
}

int main() {
    float* d;
    hipMalloc(&d, 1 << 24);
    for (int blocks : {256, 512, 1024}) {
        run<0>(d, blocks, 20000, "v_mul_f32 indep");
        run<1>(d, blocks, 20000, "v_fma_f32 indep");
        run<2>(d, blocks, 20000, "v_pk_mul_f32 indep");
        run<3>(d, blocks, 20000, "v_pk_fma_f32 indep");
        run<4>(d, blocks, 20000, "v_exp_f32 indep");
        run<5>(d, blocks, 20000, "4 exp + 4 pk_fma");
        run<6>(d, blocks, 20000, "2 exp + 6 pk_fma");
        run<7>(d, blocks, 20000, "4 exp + 4 fma");
        run<8>(d, blocks, 20000, "v_mul_f32 dep chain");
        run<9>(d, blocks, 20000, "v_pk_fma_f32 dep chain");
        run<10>(d, blocks, 20000, "v_exp_f32 dep chain");
        run<11>(d, blocks, 20000, "pk_fma 2 chains");
        run<12>(d, blocks, 20000, "pk_fma 4 chains");
        run<13>(d, blocks, 20000, "exp->pk_mul 2 chains (8 instr)");
    }
    return 0;
}
