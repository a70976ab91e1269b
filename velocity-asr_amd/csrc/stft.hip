// Power spectrogram of the reference front end (audio.py:97-115: periodic Hann(400), reflect
// pad 200, torch.stft n_fft 400 hop 160 center=False, |X|^2) as a real FFT, for n_fft = 400.
//
// Each workgroup takes 6 consecutive frames of one utterance, read straight from the unpadded
// audio (reflect padding resolved per sample, no padded copy; overlapping frames hit in L2),
// windowed and packed as z[n] = x[2n] + i x[2n+1] (a 200-point complex FFT of the even / odd samples),
// transformed in LDS as 200 = 8 x (5 x 5) (Cooley-Tukey: 25 radix-8 DFTs with twiddles, then
// two rounds of 40 radix-5 DFTs), and unpacked to the 201 bins of the real 400-point DFT:
//   X[k] = (Z[k] + conj Z[200-k]) / 2 + W400^k (Z[k] - conj Z[200-k]) / (2i),  P[k] = |X[k]|^2.
// ~1 % of the flops of the windowed-DFT GEMM it replaces, and no MFMA (the north star keeps the
// matrix cores for the projection GEMMs); the work is HBM / LDS-bound.
#include <cmath>

#include "vasr_internal.h"

namespace vasr {
namespace {

struct cf {
    float x, y;
};
__device__ __forceinline__ cf operator+(cf a, cf b) { return {a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ cf operator-(cf a, cf b) { return {a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ cf cmul(cf a, cf b) { return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }
__device__ __forceinline__ cf mul_mi(cf a) { return {a.y, -a.x}; }  // -i a
__device__ __forceinline__ cf mul_pi(cf a) { return {-a.y, a.x}; }  // +i a
__device__ __forceinline__ cf scale(cf a, float s) { return {a.x * s, a.y * s}; }

constexpr int kNfft = 400, kHop = 160, kHalf = 200, kBins = 201;
constexpr int kFPB = 6;                                // frames per workgroup (power rows out)

// Twiddle tables, evaluated at compile time in double (Taylor series about pi) and rounded once:
// tw200[j] = W200^j = e^{-2 pi i j / 200}, tw400[k] = W400^k, k = 0..200.
constexpr double kPi = 3.14159265358979323846;
constexpr double taylor_sin(double y) {  // |y| <= pi
    double term = y, sum = y;
    for (int n = 1; n < 30; ++n) {
        term *= -y * y / ((2.0 * n) * (2.0 * n + 1.0));
        sum += term;
    }
    return sum;
}
constexpr double taylor_cos(double y) {
    double term = 1.0, sum = 1.0;
    for (int n = 1; n < 30; ++n) {
        term *= -y * y / ((2.0 * n - 1.0) * (2.0 * n));
        sum += term;
    }
    return sum;
}
struct TwTable {
    cf w200[kHalf];
    cf w400[kBins];
};
constexpr TwTable make_twiddles() {
    TwTable t{};
    for (int j = 0; j < kHalf; ++j) {
        const double y = 2.0 * kPi * j / kHalf - kPi;  // e^{-i x} = (cos x, -sin x), x = y + pi
        t.w200[j] = cf{(float)(-taylor_cos(y)), (float)(taylor_sin(y))};
    }
    for (int k = 0; k < kBins; ++k) {
        const double y = 2.0 * kPi * k / kNfft - kPi;
        t.w400[k] = cf{(float)(-taylor_cos(y)), (float)(taylor_sin(y))};
    }
    return t;
}
__constant__ constexpr TwTable kTw = make_twiddles();

// Diagnostic builds only (tools/runs/r05c.sh): VASR_STFT_VGPR_CONSTS=1 holds the
// DFT constants in VGPRs (opaque to the compiler), so an SLP-vectorised build has packed-fp32 ops
// with VGPR operands only, instead of SGPR-pair operands.
#ifndef VASR_STFT_VGPR_CONSTS
#define VASR_STFT_VGPR_CONSTS 0
#endif
__device__ __forceinline__ float kconst(float c) {
    if constexpr (VASR_STFT_VGPR_CONSTS) asm volatile("" : "+v"(c));
    return c;
}
// VASR_STFT_OPAQUE_INDEX=1 hides the thread index's range from the compiler, so the stages' index
// arithmetic (t / 25, t / 40, r / 5) is 32-bit, not the 16-bit SDWA / packed-u16 forms it
// otherwise narrows to.
#ifndef VASR_STFT_OPAQUE_INDEX
#define VASR_STFT_OPAQUE_INDEX 0
#endif
__device__ __forceinline__ int kindex(int t) {
    if constexpr (VASR_STFT_OPAQUE_INDEX) asm volatile("" : "+v"(t));
    return t;
}

// Forward DFT-8 (radix-2, decimation in time), in place.
__device__ __forceinline__ void dft8(cf (&v)[8]) {
    const float r = kconst(0.70710678118654752440f);
    const cf a0 = v[0] + v[4], a1 = v[0] - v[4], a2 = v[2] + v[6], a3 = v[2] - v[6];
    const cf a4 = v[1] + v[5], a5 = v[1] - v[5], a6 = v[3] + v[7], a7 = v[3] - v[7];
    const cf b0 = a0 + a2, b2 = a0 - a2, b1 = a1 + mul_mi(a3), b3 = a1 + mul_pi(a3);
    const cf c0 = a4 + a6, c2 = a4 - a6, c1 = a5 + mul_mi(a7), c3 = a5 + mul_pi(a7);
    const cf w1c1 = cmul(c1, cf{r, -r});   // W8^1 = (1 - i) / sqrt 2
    const cf w3c3 = cmul(c3, cf{-r, -r});  // W8^3 = (-1 - i) / sqrt 2
    v[0] = b0 + c0;
    v[4] = b0 - c0;
    v[2] = b2 + mul_mi(c2);
    v[6] = b2 + mul_pi(c2);
    v[1] = b1 + w1c1;
    v[5] = b1 - w1c1;
    v[3] = b3 + w3c3;
    v[7] = b3 - w3c3;
}

// Forward DFT-5, in place.
__device__ __forceinline__ void dft5(cf (&v)[5]) {
    const float c1 = kconst(0.30901699437494742410f), c2 = kconst(-0.80901699437494742410f);
    const float s1 = kconst(0.95105651629515357212f), s2 = kconst(0.58778525229247312917f);
    const cf t1 = v[1] + v[4], t2 = v[2] + v[3], t3 = v[1] - v[4], t4 = v[2] - v[3];
    const cf x0 = v[0];
    const cf p1 = x0 + scale(t1, c1) + scale(t2, c2);
    const cf p2 = x0 + scale(t1, c2) + scale(t2, c1);
    const cf q1 = scale(t3, s1) + scale(t4, s2);   // y1 = p1 - i q1, y4 = p1 + i q1
    const cf q2 = scale(t3, s2) - scale(t4, s1);   // y2 = p2 - i q2, y3 = p2 + i q2
    v[0] = x0 + t1 + t2;
    v[1] = p1 + mul_mi(q1);
    v[4] = p1 + mul_pi(q1);
    v[2] = p2 + mul_mi(q2);
    v[3] = p2 + mul_pi(q2);
}

// FPB frames per workgroup, |X|^2 rows to `power`.
template <int FPB>
__global__ __launch_bounds__(256) void stft_power_400_kernel(const float* __restrict__ audio, int64_t ld_audio,
                                                             int S, const int32_t* __restrict__ samples, int F,
                                                             const float* __restrict__ window,
                                                             float* __restrict__ power, int64_t ldp,
                                                             int64_t stridep) {
    __shared__ cf tw[kHalf + kBins];  // W200^j, then W400^k
    __shared__ cf za[FPB][kHalf];
    __shared__ cf zb[FPB][kHalf];
    int b = blockIdx.y, fb = blockIdx.x;
    if (VASR_FE_XCD & 1) {  // (b, frame-block) runs per XCD, as the mel pass reads them
        const int w = xcd_run(fb + b * (int)gridDim.x, (int)(gridDim.x * gridDim.y));
        b = w / (int)gridDim.x;
        fb = w - b * (int)gridDim.x;
    }
    const int f0 = fb * FPB;
    const int tid = threadIdx.x;
    const float* ab = audio + (int64_t)b * ld_audio;
    // 1. windowed even / odd sample pairs packed as complex, straight from the unpadded audio
    //    (reflect padding of n_fft / 2 resolved per sample; the overlapping frames hit in L2).
    //    Every global load of the block (twiddles, samples, window) is issued before the first
    //    use, so the block waits for one memory latency, not one per loop trip.
    constexpr int kTwIt = (kHalf + kBins + 255) / 256, kPackIt = (FPB * kHalf + 255) / 256;
    const float2* win2 = reinterpret_cast<const float2*>(window);
    const cf* twg = reinterpret_cast<const cf*>(&kTw);  // w200 then w400, contiguous
    cf twv[kTwIt];
#pragma unroll
    for (int it = 0; it < kTwIt; ++it) twv[it] = twg[min(tid + it * 256, kHalf + kBins - 1)];
    // samples (optional): this utterance's own length; its reflect padding is taken at its own
    // end (frames past its last one read clamped data and are ignored downstream)
    const int Sb = samples ? samples[b] : S;
    auto reflect = [Sb](int j) {
        j = j < 0 ? -j : j;
        j = j >= Sb ? 2 * (Sb - 1) - j : j;
        return min(max(j, 0), Sb - 1);  // frames past F read clamped data, never stored
    };
    float x0[kPackIt], x1[kPackIt];
    float2 w[kPackIt];
#pragma unroll
    for (int it = 0; it < kPackIt; ++it) {
        const int i = min(tid + it * 256, FPB * kHalf - 1);
        const int q = i / kHalf, n = i - q * kHalf;
        const int j0 = (f0 + q) * kHop + 2 * n - kNfft / 2;  // unpadded index of sample 2n
        x0[it] = ab[reflect(j0)];
        x1[it] = ab[reflect(j0 + 1)];
        w[it] = win2[n];
    }
#pragma unroll
    for (int it = 0; it < kTwIt; ++it)
        if (tid + it * 256 < kHalf + kBins) tw[tid + it * 256] = twv[it];
#pragma unroll
    for (int it = 0; it < kPackIt; ++it) {
        const int i = tid + it * 256;
        if (i < FPB * kHalf) (&za[0][0])[i] = cf{x0[it] * w[it].x, x1[it] * w[it].y};
    }
    __syncthreads();
    // 3. radix-8 over n1 (n = 25 n1 + n2), twiddle W200^(n2 k1); out [q][k1 * 25 + n2]
    for (int t = kindex(tid); t < FPB * 25; t += 256) {
        const int q = t / 25, n2 = t - q * 25;
        cf v[8];
#pragma unroll
        for (int n1 = 0; n1 < 8; ++n1) v[n1] = za[q][25 * n1 + n2];
        dft8(v);
#pragma unroll
        for (int k1 = 0; k1 < 8; ++k1) zb[q][k1 * 25 + n2] = k1 == 0 ? v[0] : cmul(v[k1], tw[(n2 * k1) % kHalf]);
    }
    __syncthreads();
    // 4. radix-5 over m1 (n2 = 5 m1 + m2), twiddle W25^(m2 j1) = W200^(8 m2 j1); out [q][k1*25 + m2*5 + j1]
    for (int t = kindex(tid); t < FPB * 40; t += 256) {
        const int q = t / 40, r = t - q * 40, k1 = r / 5, m2 = r - k1 * 5;
        cf v[5];
#pragma unroll
        for (int m1 = 0; m1 < 5; ++m1) v[m1] = zb[q][k1 * 25 + 5 * m1 + m2];
        dft5(v);
#pragma unroll
        for (int j1 = 0; j1 < 5; ++j1)
            za[q][k1 * 25 + m2 * 5 + j1] = j1 == 0 ? v[0] : cmul(v[j1], tw[(8 * m2 * j1) % kHalf]);
    }
    __syncthreads();
    // 5. radix-5 over m2 -> Z[k1 + 8 (j1 + 5 j2)] in natural order
    for (int t = kindex(tid); t < FPB * 40; t += 256) {
        const int q = t / 40, r = t - q * 40, k1 = r / 5, j1 = r - k1 * 5;
        cf v[5];
#pragma unroll
        for (int m2 = 0; m2 < 5; ++m2) v[m2] = za[q][k1 * 25 + m2 * 5 + j1];
        dft5(v);
#pragma unroll
        for (int j2 = 0; j2 < 5; ++j2) zb[q][k1 + 8 * (j1 + 5 * j2)] = v[j2];
    }
    __syncthreads();
    // 6. real-FFT unpack by bin pairs (k, 200 - k), k = 0..100: with A, B the even / odd spectra
    //    at k, X[k] = A + W400^k B and X[200 - k] = conj(A - W400^k B).  |X|^2 is formed as
    //    re^2 + im^2 (the reference rounds through abs(): at most 1 ulp apart).
    float* pb = power + (int64_t)b * stridep + (int64_t)f0 * ldp;  // uniform base
    const int ldp32 = (int)ldp;
    for (int i = kindex(tid); i < FPB * 101; i += 256) {
        const int q = i / 101, k = i - q * 101;
        if (f0 + q >= F) continue;
        const cf zk = zb[q][k];
        const cf zm = zb[q][k == 0 ? 0 : kHalf - k];
        const cf zc = cf{zm.x, -zm.y};
        const cf A = scale(zk + zc, 0.5f);
        const cf WB = cmul(tw[kHalf + k], scale(mul_mi(zk - zc), 0.5f));
        const cf X1 = A + WB, X2 = A - WB;
        float* row = pb + q * ldp32;
        row[k] = X1.x * X1.x + X1.y * X1.y;
        row[kHalf - k] = X2.x * X2.x + X2.y * X2.y;
    }
}

}  // namespace
}  // namespace vasr

static int stft_power_400(const float* audio, int64_t ld_audio, int B, int S, const int32_t* samples,
                          const float* window, float* power, int64_t ldp, int64_t stride_power, void* stream,
                          const char* who) {
    using namespace vasr;
    VASR_CHECK_ARG(audio && window && power, "%s: null pointer", who);
    VASR_CHECK_ARG(((uintptr_t)window & 7) == 0, "%s: window must be 8-byte aligned", who);
    VASR_CHECK_ARG(B >= 0 && S > kNfft / 2 && ld_audio >= S && ldp >= kBins, "%s: bad shape", who);
    const int F = (S + 2 * (kNfft / 2) - kNfft) / kHop + 1;
    VASR_CHECK_ARG(stride_power >= (int64_t)F * ldp, "%s: stride_power too small", who);
    if (B == 0) return VASR_OK;
    hipLaunchKernelGGL((stft_power_400_kernel<kFPB>), dim3((F + kFPB - 1) / kFPB, B), dim3(256), 0,
                       as_stream(stream), audio, ld_audio, S, samples, F, window, power, ldp, stride_power);
    return launch_status(who);
}

VASR_API int vasr_stft_power_400_f32(const float* audio, int64_t ld_audio, int B, int S, const float* window,
                                     float* power, int64_t ldp, int64_t stride_power, void* stream) {
    return stft_power_400(audio, ld_audio, B, S, nullptr, window, power, ldp, stride_power, stream,
                          "vasr_stft_power_400_f32");
}

// Utterances of different lengths in one zero-padded (B, S) batch: samples[b] <= S is
// utterance b's own length (> 200), on the device.  Frames f < samples[b] / 160 + 1 are those
// of the utterance alone; later frames are ignored by the _var mel pass.
VASR_API int vasr_stft_power_400_var_f32(const float* audio, int64_t ld_audio, int B, int S, const int32_t* samples,
                                         const float* window, float* power, int64_t ldp, int64_t stride_power,
                                         void* stream) {
    VASR_CHECK_ARG(samples, "vasr_stft_power_400_var_f32: null samples");
    return stft_power_400(audio, ld_audio, B, S, samples, window, power, ldp, stride_power, stream,
                          "vasr_stft_power_400_var_f32");
}
