// REFUTED HYPOTHESIS, kept as the record (profiles/r05b/, r05c/): does a packed-fp32 VALU op (VOP3P,
// 64-bit operands) that reads an SGPR pair see a LATER SALU write of that pair when another wave's
// MFMAs share the SIMD?  stft.hip's SLP build reads its DFT constants as SGPR pairs in v_pk_fma_f32
// and re-assigns them with s_mov_b32 2-23 instructions later.  Result: 0 bad lanes in every variant
// below, alone / beside MFMA / beside VALU chains; and the SLP stft with the constants in VGPRs
// still failed 19/400 (r05c).  The cause is the swapped-source packed form (tools/isa/isa_scan.py).
//
// Victim: every iteration sets s[20:21] = (a, b), runs one packed op reading s[20:21], then
// overwrites s20 and s21 with c.  With x = (1, 1), r.x counts a and r.y counts b; a lane whose pack
// read the overwritten value shows c in its sum.  Bad lanes are split by half-wave.
// Aggressors on a second stream: MFMA chains (v_mfma_f32_32x32x16_bf16), or VALU-only chains.
// Variants: 0 pk_fma s-pair, WAR distance 1; 1 distance 3 (two VALU between); 2 op_sel_hi:[1,0,1]
// (hi lanes read s20) then s20 overwritten; 3 control: two scalar v_fma_f32 (s20, s21) then the
// overwrite; 4 pk_fma s-pair, s_nop 4 before the overwrite; 5 pk_fma with a VGPR-pair source;
// 6 the pair written right before the packed read and overwritten right after (no wait states);
// 7 written right before, overwritten only after s_nop 4.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

template <int V>
__global__ __launch_bounds__(256) void victim(float* out, int iters, float a, float b, float c) {
    f2 r = {0.f, 0.f};
    const f2 x = {1.f, 1.f};
    float d0 = 0.f, d1 = 0.f;
    for (int i = 0; i < iters; ++i) {
        if constexpr (V == 0) {
            asm volatile("s_mov_b32 s20, %2\n\ts_mov_b32 s21, %3\n\ts_nop 4\n\t"
                         "v_pk_fma_f32 %0, %1, s[20:21], %0\n\t"
                         "s_mov_b32 s20, %4\n\ts_mov_b32 s21, %4"
                         : "+v"(r) : "v"(x), "s"(a), "s"(b), "s"(c) : "s20", "s21");
        } else if constexpr (V == 1) {
            asm volatile("s_mov_b32 s20, %4\n\ts_mov_b32 s21, %5\n\ts_nop 4\n\t"
                         "v_pk_fma_f32 %0, %3, s[20:21], %0\n\t"
                         "v_add_f32 %1, 1.0, %1\n\tv_add_f32 %2, 1.0, %2\n\t"
                         "s_mov_b32 s20, %6\n\ts_mov_b32 s21, %6"
                         : "+v"(r), "+v"(d0), "+v"(d1) : "v"(x), "s"(a), "s"(b), "s"(c) : "s20", "s21");
        } else if constexpr (V == 2) {
            // lo lanes: x.lo * s20, hi lanes: x.hi * s20 (op_sel_hi of src1 = 0): both halves read s20
            asm volatile("s_mov_b32 s20, %2\n\ts_mov_b32 s21, %3\n\ts_nop 4\n\t"
                         "v_pk_fma_f32 %0, %1, s[20:21], %0 op_sel_hi:[1,0,1]\n\t"
                         "s_mov_b32 s20, %4\n\ts_mov_b32 s21, %4"
                         : "+v"(r) : "v"(x), "s"(a), "s"(b), "s"(c) : "s20", "s21");
        } else if constexpr (V == 3) {
            asm volatile("s_mov_b32 s20, %4\n\ts_mov_b32 s21, %5\n\ts_nop 4\n\t"
                         "v_fma_f32 %0, %2, s20, %0\n\tv_fma_f32 %1, %3, s21, %1\n\t"
                         "s_mov_b32 s20, %6\n\ts_mov_b32 s21, %6"
                         : "+v"(r.x), "+v"(r.y) : "v"(x.x), "v"(x.y), "s"(a), "s"(b), "s"(c) : "s20", "s21");
        } else if constexpr (V == 4) {
            asm volatile("s_mov_b32 s20, %2\n\ts_mov_b32 s21, %3\n\ts_nop 4\n\t"
                         "v_pk_fma_f32 %0, %1, s[20:21], %0\n\ts_nop 4\n\t"
                         "s_mov_b32 s20, %4\n\ts_mov_b32 s21, %4"
                         : "+v"(r) : "v"(x), "s"(a), "s"(b), "s"(c) : "s20", "s21");
        } else if constexpr (V == 6) {
            // the compiler's form: SGPR pair written right before the packed read (RAW distance 1)
            // and overwritten right after it (WAR distance 1), no wait states anywhere
            asm volatile("s_mov_b32 s20, %2\n\ts_mov_b32 s21, %3\n\t"
                         "v_pk_fma_f32 %0, %1, s[20:21], %0\n\t"
                         "s_mov_b32 s20, %4\n\ts_mov_b32 s21, %4"
                         : "+v"(r) : "v"(x), "s"(a), "s"(b), "s"(c) : "s20", "s21");
        } else if constexpr (V == 7) {
            // RAW distance 1 only: the pair written right before the packed read, no overwrite soon after
            asm volatile("s_mov_b32 s20, %2\n\ts_mov_b32 s21, %3\n\t"
                         "v_pk_fma_f32 %0, %1, s[20:21], %0\n\ts_nop 4\n\t"
                         "s_mov_b32 s20, %4\n\ts_mov_b32 s21, %4"
                         : "+v"(r) : "v"(x), "s"(a), "s"(b), "s"(c) : "s20", "s21");
        } else {
            f2 s = {a, b};
            const f2 cc = {c, c};
            asm volatile("s_nop 4\n\tv_pk_fma_f32 %0, %2, %1, %0\n\t"
                         "v_pk_mov_b32 %1, %3, %3"
                         : "+v"(r), "+v"(s) : "v"(x), "v"(cc));
        }
    }
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    out[2 * t] = r.x + 0.f * d0;
    out[2 * t + 1] = r.y + 0.f * d1;
}

__global__ __launch_bounds__(256) void mfma_aggressor(float* out, int iters, float seed) {
    bf16x8 fa, fb;
    for (int j = 0; j < 8; ++j) {
        fa[j] = (__bf16)(seed * (threadIdx.x + j));
        fb[j] = (__bf16)(seed * (j - (int)threadIdx.x));
    }
    floatx16 acc = {};
    for (int i = 0; i < iters; ++i) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb, acc, 0, 0, 0);
    float s = 0.f;
    for (int i = 0; i < 16; ++i) s += acc[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void valu_aggressor(float* out, int iters, float seed) {
    float v0 = seed * threadIdx.x, v1 = v0 + 1.f, v2 = v0 + 2.f, v3 = v0 + 3.f;
    for (int i = 0; i < iters * 8; ++i) {
        v0 = __builtin_fmaf(v0, 0.999f, 0.5f);
        v1 = __builtin_fmaf(v1, 0.999f, 0.5f);
        v2 = __builtin_fmaf(v2, 0.999f, 0.5f);
        v3 = __builtin_fmaf(v3, 0.999f, 0.5f);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = v0 + v1 + v2 + v3;
}

template <int V>
static void launch_victim(dim3 g, hipStream_t s, float* out, int iters) {
    hipLaunchKernelGGL(victim<V>, g, dim3(256), 0, s, out, iters, 1.0f, 2.0f, 4096.0f);
}

int main(int argc, char** argv) {
    const int trials = argc > 1 ? atoi(argv[1]) : 20;
    const int iters = argc > 2 ? atoi(argv[2]) : 4000;
    const int agg_iters = argc > 3 ? atoi(argv[3]) : 6000;
    const int nblk = 1024, nthr = nblk * 256;
    float *out, *aout;
    (void)hipMalloc(&out, (size_t)nthr * 2 * sizeof(float));
    (void)hipMalloc(&aout, (size_t)nthr * sizeof(float));
    hipStream_t s0, s1;
    (void)hipStreamCreateWithFlags(&s0, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
    std::vector<float> h((size_t)nthr * 2);
    void (*launch[8])(dim3, hipStream_t, float*, int) = {launch_victim<0>, launch_victim<1>, launch_victim<2>,
                                                        launch_victim<3>, launch_victim<4>, launch_victim<5>,
                                                        launch_victim<6>, launch_victim<7>};
    const char* names[8] = {"pk_fma s-pair, WAR dist 1", "pk_fma s-pair, WAR dist 3", "pk_fma op_sel_hi:[1,0,1]",
                            "scalar v_fma x2 (control)", "pk_fma s-pair, s_nop 4", "pk_fma v-pair (control)",
                            "pk_fma s-pair, RAW 1 + WAR 1", "pk_fma s-pair, RAW 1 only"};
    const char* aggn[3] = {"alone", "beside MFMA", "beside VALU"};
    for (int v = 0; v < 8; ++v) {
        for (int ag = 0; ag < 3; ++ag) {
            long bad_lo = 0, bad_hi = 0, bad_launch = 0;
            for (int t = 0; t < trials; ++t) {
                if (ag == 1) hipLaunchKernelGGL(mfma_aggressor, dim3(nblk), dim3(256), 0, s1, aout, agg_iters, 0.01f);
                if (ag == 2) hipLaunchKernelGGL(valu_aggressor, dim3(nblk), dim3(256), 0, s1, aout, agg_iters, 0.01f);
                launch[v](dim3(nblk), s0, out, iters);
                (void)hipDeviceSynchronize();
                (void)hipMemcpy(h.data(), out, h.size() * sizeof(float), hipMemcpyDeviceToHost);
                long bl = 0;
                const float ex = (v == 2) ? (float)iters * 1.0f : (float)iters * 1.0f;  // r.x
                const float ey = (v == 2) ? (float)iters * 1.0f : (float)iters * 2.0f;  // r.y
                for (int i = 0; i < nthr; ++i) {
                    const bool bad = h[2 * i] != ex || h[2 * i + 1] != ey;
                    if (bad) {
                        ++bl;
                        if ((i & 63) < 32) ++bad_lo; else ++bad_hi;
                    }
                }
                if (bl) ++bad_launch;
            }
            printf("%-28s %-12s launches with a bad lane %3ld / %d   bad lanes: lanes 0-31 %8ld  lanes 32-63 %8ld\n",
                   names[v], aggn[ag], bad_launch, trials, bad_lo, bad_hi);
            fflush(stdout);
        }
    }
    (void)hipFree(out);
    (void)hipFree(aout);
    return 0;
}
