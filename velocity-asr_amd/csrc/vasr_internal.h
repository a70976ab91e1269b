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

// Current value of a vasr_set_option key (enum vasr_option); 0 = automatic.
int option(int key);

// mel.hip: the stats + normalisation passes of the chunked log-mel front end (kFC = 16 frames
// per chunk) over a workspace laid out as vasr_mel_workspace_floats describes.
constexpr int kMelChunk = 16;
// frames (optional, device): per-utterance frame counts <= F (vasr_mel_log_norm_var_f32)
int mel_chunk_finish(float* workspace, float* out, int64_t out_stride, int frame_off, int B, int F, int n_mels,
                     int normalize, hipStream_t s, const int32_t* frames = nullptr);

constexpr int kWave = 64;

#ifndef VASR_FE_XCD
#define VASR_FE_XCD 0  // front end XCD-run block order, bit mask: 1 STFT, 2 log-mel, 4 norm (r06ay: off)
#endif
// Workgroups id, id + 8, id + 16, ... are dealt to the same XCD (round-robin dispatch); the
// returned work index gives each XCD a contiguous run of the n work items, so neighbouring
// items (and a consumer kernel mapped the same way) share that XCD's L2.
__device__ __forceinline__ int xcd_run(int id, int n) {
    const int q8 = n / 8, r8 = n % 8, xg = id % 8;
    return (xg < r8 ? xg * (q8 + 1) : r8 * (q8 + 1) + (xg - r8) * q8) + id / 8;
}

// Sum over the 64 lanes, broadcast to all: DPP within and across 16-lane rows (no LDS
// round trips, unlike a ds_bpermute butterfly): row sums by quad_perm / half-mirror / mirror,
// then row_bcast15 / row_bcast31 chain the rows into lane 63, read back as a scalar.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROWMASK, 0xF, false));
}
__device__ __forceinline__ float wave_sum(float v) {
    v += dpp_f<0xB1, 0xF>(v);   // quad_perm [1,0,3,2]
    v += dpp_f<0x4E, 0xF>(v);   // quad_perm [2,3,0,1]
    v += dpp_f<0x141, 0xF>(v);  // row_half_mirror
    v += dpp_f<0x140, 0xF>(v);  // row_mirror: every lane holds its row's sum
    v += dpp_f<0x142, 0xA>(v);  // row_bcast15 -> rows 1, 3: r0+r1, r2+r3
    v += dpp_f<0x143, 0xC>(v);  // row_bcast31 -> rows 2, 3: row 3 = r0+r1+r2+r3
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
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

// Epilogue forms on the hardware transcendentals (v_exp_f32 / v_log_f32 / v_rcp_f32, ~1 ulp
// each): 12-20 instructions instead of the 55-130 of the libm forms above, which dominated
// the GEMM epilogues.  Accuracy is stated per function; the parity tests bound the effect.
__device__ __forceinline__ float fast_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.44269504088896341f); }

// erfc(a) for a >= 0 as q(t) exp(-a^2), t = 1 / (1 + p a) (Abramowitz & Stegun 7.1.26,
// |error of erf| <= 1.5e-7); GELU(x) = x (1 - q/2) for x >= 0 and x q/2 below, which keeps
// the small negative tail relatively accurate.
__device__ __forceinline__ float gelu_fast(float x) {
    const float a = fabsf(x) * 0.70710678118654752440f;
    const float t = __builtin_amdgcn_rcpf(__builtin_fmaf(0.3275911f, a, 1.0f));
    float q = __builtin_fmaf(1.061405429f, t, -1.453152027f);
    q = __builtin_fmaf(q, t, 1.421413741f);
    q = __builtin_fmaf(q, t, -0.284496736f);
    q = __builtin_fmaf(q, t, 0.254829592f);
    q = q * t * fast_exp(-a * a);
    return x >= 0.0f ? x * __builtin_fmaf(-0.5f, q, 1.0f) : 0.5f * x * q;
}

// softplus(x) = max(x, 0) + log1p(exp(-|x|)); log1p(e) = log(u) * e / (u - 1) with u = 1 + e
// (compensates the rounding of u), e itself when u rounds to 1.  Threshold 20 as torch.
__device__ __forceinline__ float softplus20_fast(float x) {
    const float e = fast_exp(-fabsf(x));
    const float u = 1.0f + e;
    const float d = u - 1.0f;
    const float l = d == 0.0f ? e : __builtin_amdgcn_logf(u) * 0.69314718055994531f * (e * __builtin_amdgcn_rcpf(d));
    return x > 20.0f ? x : fmaxf(x, 0.0f) + l;
}

__device__ __forceinline__ float sigmoid_fast(float x) { return __builtin_amdgcn_rcpf(1.0f + fast_exp(-x)); }

// FakeQuantize._quantize/_dequantize + straight-through form (quantize.py:97, :118-133) with
// every operation IEEE-rounded in torch's order: contraction is switched off for this block
// (HIP compiles with -ffp-contract=fast, which would fuse (q - zp) * s into the following
// subtraction and move results by an ulp); the division is the correctly rounded one.
// q = {scale, zp, qmin, qmax}.  scale == 0 (never produced by calibration, which clamps it to
// >= 1e-10) marks a column that is not quantized, so one parameter array can cover fused
// quantized / plain outputs.
__device__ __forceinline__ float fake_quant(float x, float4 q) {
#pragma clang fp contract(off)
    if (q.x == 0.0f) return x;
    const float t = x / q.x + q.y;
    const float r = fminf(fmaxf(__builtin_rintf(t), q.z), q.w);
    const float xdq = (r - q.y) * q.x;
    return x + (xdq - x);
}

}  // namespace vasr

#define VASR_CHECK_ARG(cond, ...)            \
    do {                                     \
        if (!(cond)) {                       \
            ::vasr::set_error(__VA_ARGS__);  \
            return VASR_EINVAL;              \
        }                                    \
    } while (0)
