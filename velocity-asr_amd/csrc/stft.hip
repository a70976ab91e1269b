// Power spectrogram of the reference front end (audio.py:97-115: periodic Hann(400), reflect
// pad 200, torch.stft n_fft 400 hop 160 center=False, |X|^2) as a real FFT, for n_fft = 400.
//
// Each workgroup takes 6 consecutive frames of one utterance: their 1200-sample span is read
// once (reflect padding applied on the fly from the unpadded audio, no padded copy), windowed
// and packed as z[n] = x[2n] + i x[2n+1] (a 200-point complex FFT of the even / odd samples),
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
constexpr int kFPB = 6;                                // frames per workgroup
constexpr int kSpan = (kFPB - 1) * kHop + kNfft;       // 1200 samples

// Forward DFT-8 (radix-2, decimation in time), in place.
__device__ __forceinline__ void dft8(cf (&v)[8]) {
    const float r = 0.70710678118654752440f;
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
    const float c1 = 0.30901699437494742410f, c2 = -0.80901699437494742410f;
    const float s1 = 0.95105651629515357212f, s2 = 0.58778525229247312917f;
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

__global__ __launch_bounds__(256) void stft_power_400_kernel(const float* __restrict__ audio, int64_t ld_audio,
                                                             int S, int F, const float* __restrict__ window,
                                                             float* __restrict__ power, int64_t ldp,
                                                             int64_t stridep) {
    __shared__ float samp[kSpan];
    __shared__ float win[kNfft];
    __shared__ cf tw200[kHalf];   // W200^j
    __shared__ cf tw400[kBins];   // W400^k
    __shared__ cf za[kFPB][kHalf];
    __shared__ cf zb[kFPB][kHalf];
    const int b = blockIdx.y, f0 = blockIdx.x * kFPB;
    const int tid = threadIdx.x;
    const float* ab = audio + (int64_t)b * ld_audio;
    // 1. span (reflect padding of n_fft / 2 on the fly), window, twiddles
    const int pad = kNfft / 2;
    for (int i = tid; i < kSpan; i += 256) {
        int j = f0 * kHop + i - pad;
        j = j < 0 ? -j : j;
        j = j >= S ? 2 * (S - 1) - j : j;
        samp[i] = (j >= 0 && j < S) ? ab[j] : 0.f;  // frames past F read clamped data, never stored
    }
    for (int i = tid; i < kNfft; i += 256) win[i] = window[i];
    for (int i = tid; i < kHalf + kBins; i += 256) {
        float s, c;
        if (i < kHalf) {
            sincospif(2.0f * (float)i / (float)kHalf, &s, &c);
            tw200[i] = cf{c, -s};
        } else {
            const int k = i - kHalf;
            sincospif(2.0f * (float)k / (float)kNfft, &s, &c);
            tw400[k] = cf{c, -s};
        }
    }
    __syncthreads();
    // 2. windowed even / odd samples packed as complex
    for (int i = tid; i < kFPB * kHalf; i += 256) {
        const int q = i / kHalf, n = i - q * kHalf;
        const float* fr = samp + q * kHop;
        za[q][n] = cf{fr[2 * n] * win[2 * n], fr[2 * n + 1] * win[2 * n + 1]};
    }
    __syncthreads();
    // 3. radix-8 over n1 (n = 25 n1 + n2), twiddle W200^(n2 k1); out [q][k1 * 25 + n2]
    if (tid < kFPB * 25) {
        const int q = tid / 25, n2 = tid - q * 25;
        cf v[8];
#pragma unroll
        for (int n1 = 0; n1 < 8; ++n1) v[n1] = za[q][25 * n1 + n2];
        dft8(v);
#pragma unroll
        for (int k1 = 0; k1 < 8; ++k1) zb[q][k1 * 25 + n2] = k1 == 0 ? v[0] : cmul(v[k1], tw200[(n2 * k1) % kHalf]);
    }
    __syncthreads();
    // 4. radix-5 over m1 (n2 = 5 m1 + m2), twiddle W25^(m2 j1) = W200^(8 m2 j1); out [q][k1*25 + m2*5 + j1]
    if (tid < kFPB * 40) {
        const int q = tid / 40, r = tid - q * 40, k1 = r / 5, m2 = r - k1 * 5;
        cf v[5];
#pragma unroll
        for (int m1 = 0; m1 < 5; ++m1) v[m1] = zb[q][k1 * 25 + 5 * m1 + m2];
        dft5(v);
#pragma unroll
        for (int j1 = 0; j1 < 5; ++j1)
            za[q][k1 * 25 + m2 * 5 + j1] = j1 == 0 ? v[0] : cmul(v[j1], tw200[(8 * m2 * j1) % kHalf]);
    }
    __syncthreads();
    // 5. radix-5 over m2 -> Z[k1 + 8 (j1 + 5 j2)] in natural order
    if (tid < kFPB * 40) {
        const int q = tid / 40, r = tid - q * 40, k1 = r / 5, j1 = r - k1 * 5;
        cf v[5];
#pragma unroll
        for (int m2 = 0; m2 < 5; ++m2) v[m2] = za[q][k1 * 25 + m2 * 5 + j1];
        dft5(v);
#pragma unroll
        for (int j2 = 0; j2 < 5; ++j2) zb[q][k1 + 8 * (j1 + 5 * j2)] = v[j2];
    }
    __syncthreads();
    // 6. real-FFT unpack and power, coalesced rows
    for (int i = tid; i < kFPB * kBins; i += 256) {
        const int q = i / kBins, k = i - q * kBins;
        const int f = f0 + q;
        if (f >= F) continue;
        const cf zk = zb[q][k % kHalf];
        const cf zm = zb[q][(kHalf - k) % kHalf];
        const cf zc = cf{zm.x, -zm.y};
        const cf A = scale(zk + zc, 0.5f);
        const cf Bv = scale(mul_mi(zk - zc), 0.5f);
        const cf X = A + cmul(tw400[k], Bv);
        const float m = sqrtf(X.x * X.x + X.y * X.y);  // |X| squared, as abs()**2
        power[(int64_t)b * stridep + (int64_t)f * ldp + k] = m * m;
    }
}

}  // namespace
}  // namespace vasr

VASR_API int vasr_stft_power_400_f32(const float* audio, int64_t ld_audio, int B, int S, const float* window,
                                     float* power, int64_t ldp, int64_t stride_power, void* stream) {
    using namespace vasr;
    VASR_CHECK_ARG(audio && window && power, "vasr_stft_power_400_f32: null pointer");
    VASR_CHECK_ARG(B >= 0 && S > kNfft / 2 && ld_audio >= S && ldp >= kBins, "vasr_stft_power_400_f32: bad shape");
    const int F = (S + 2 * (kNfft / 2) - kNfft) / kHop + 1;
    VASR_CHECK_ARG(stride_power >= (int64_t)F * ldp, "vasr_stft_power_400_f32: stride_power too small");
    if (B == 0) return VASR_OK;
    hipLaunchKernelGGL(stft_power_400_kernel, dim3((F + kFPB - 1) / kFPB, B), dim3(256), 0, as_stream(stream), audio,
                       ld_audio, S, F, window, power, ldp, stride_power);
    return launch_status("vasr_stft_power_400_f32");
}
