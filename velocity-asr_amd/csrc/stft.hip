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

// FPB frames per workgroup.  MEL = false: |X|^2 rows to `power` (FPB = 6).  MEL = true (FPB =
// kFC = 16, one log-mel chunk): the power rows stay in LDS and the chunk's log-mel rows and
// fp64 (sum, sum of squares) partials are written exactly as mel_chunk_log_kernel writes them
// (mel.hip), so the two-kernel and the fused front end agree bit for bit.
struct MelArgs {
    const int32_t* rowptr;
    const int32_t* col;
    const float* val;
    float* tmp;     // (B, F, n_mels) log-mel rows
    double* part;   // (B, nch, n_mels, 2) fp64 partials
    int n_mels;
};
constexpr int kMelMaxNnz = 1024, kMelMaxBins = 85;

template <int FPB, bool MEL>
__global__ __launch_bounds__(256) void stft_power_400_kernel(const float* __restrict__ audio, int64_t ld_audio,
                                                             int S, const int32_t* __restrict__ samples, int F,
                                                             const float* __restrict__ window,
                                                             float* __restrict__ power, int64_t ldp,
                                                             int64_t stridep, MelArgs ma) {
    __shared__ cf tw[kHalf + kBins];  // W200^j, then W400^k
    __shared__ cf za[FPB][kHalf];
    __shared__ cf zb[FPB][kHalf];
    __shared__ int rp_s[MEL ? kMelMaxBins + 1 : 1];
    __shared__ int col_s[MEL ? kMelMaxNnz : 1];
    __shared__ float val_s[MEL ? kMelMaxNnz : 1];
    __shared__ float vals[MEL ? FPB * kMelMaxBins : 1];
    const int b = blockIdx.y, f0 = blockIdx.x * FPB;
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
    bool csr_lds = false;  // MEL: the CSR in LDS when it has <= kMelMaxNnz entries (393 for 80 x 201)
    if constexpr (MEL) {
        const int nnz = ma.rowptr[ma.n_mels];
        csr_lds = nnz <= kMelMaxNnz;
        for (int i = tid; i <= ma.n_mels; i += 256) rp_s[i] = ma.rowptr[i];
        if (csr_lds)
            for (int i = tid; i < nnz; i += 256) {
                col_s[i] = ma.col[i];
                val_s[i] = ma.val[i];
            }
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
    for (int t = tid; t < FPB * 25; t += 256) {
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
    for (int t = tid; t < FPB * 40; t += 256) {
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
    for (int t = tid; t < FPB * 40; t += 256) {
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
    float* pw = reinterpret_cast<float*>(&za[0][0]);  // MEL: power rows [FPB][kBins] (za is free)
    float* pb = MEL ? pw : power + (int64_t)b * stridep + (int64_t)f0 * ldp;  // uniform base
    const int ldp32 = MEL ? kBins : (int)ldp;
    for (int i = tid; i < FPB * 101; i += 256) {
        const int q = i / 101, k = i - q * 101;
        if (!MEL && f0 + q >= F) continue;
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
    if constexpr (MEL) {
        // 7. log-mel of the chunk and its fp64 partials (mel_chunk_log_kernel's arithmetic)
        __syncthreads();
        const int n_mels = ma.n_mels, nch = gridDim.x;
        const int nf = min(FPB, F - f0);
        float* tb = ma.tmp + ((int64_t)b * F + f0) * n_mels;
        for (int i = tid; i < nf * n_mels; i += 256) {
            const int fl = i / n_mels, m = i - fl * n_mels;
            const float* prow = pw + fl * kBins;
            float acc = 0.f;
            if (csr_lds)
                for (int e = rp_s[m]; e < rp_s[m + 1]; ++e) acc = __builtin_fmaf(val_s[e], prow[col_s[e]], acc);
            else
                for (int e = rp_s[m]; e < rp_s[m + 1]; ++e) acc = __builtin_fmaf(ma.val[e], prow[ma.col[e]], acc);
            const float v = logf(acc + 1e-10f);
            vals[i] = v;
            tb[i] = v;
        }
        __syncthreads();
        for (int m = tid; m < n_mels; m += 256) {
            double Ssum = 0.0, Q = 0.0;
            for (int fl = 0; fl < nf; ++fl) {
                const double v = (double)vals[fl * n_mels + m];
                Ssum += v;
                Q += v * v;
            }
            double* pp = ma.part + (((int64_t)b * nch + blockIdx.x) * n_mels + m) * 2;
            pp[0] = Ssum;
            pp[1] = Q;
        }
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
    hipLaunchKernelGGL((stft_power_400_kernel<kFPB, false>), dim3((F + kFPB - 1) / kFPB, B), dim3(256), 0,
                       as_stream(stream), audio, ld_audio, S, samples, F, window, power, ldp, stride_power, MelArgs{});
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

VASR_API int vasr_stft_logmel_400_f32(const float* audio, int64_t ld_audio, int B, int S, const float* window,
                                      const int32_t* fb_rowptr, const int32_t* fb_col, const float* fb_val,
                                      float* out, int64_t out_stride, int frame_off, int n_mels, int normalize,
                                      float* workspace, void* stream) {
    using namespace vasr;
    VASR_CHECK_ARG(audio && window && fb_rowptr && fb_col && fb_val && out && workspace,
                   "vasr_stft_logmel_400_f32: null pointer");
    VASR_CHECK_ARG(((uintptr_t)window & 7) == 0, "vasr_stft_logmel_400_f32: window must be 8-byte aligned");
    VASR_CHECK_ARG(B >= 0 && S > kNfft / 2 && ld_audio >= S && n_mels >= 1 && n_mels <= kMelMaxBins && frame_off >= 0,
                   "vasr_stft_logmel_400_f32: bad shape (S=%d n_mels=%d)", S, n_mels);
    const int F = (S + 2 * (kNfft / 2) - kNfft) / kHop + 1;
    VASR_CHECK_ARG(out_stride >= (int64_t)(F + frame_off) * n_mels, "vasr_stft_logmel_400_f32: out_stride too small");
    if (B == 0) return VASR_OK;
    static_assert(kMelChunk == 16, "one log-mel chunk per workgroup");
    hipStream_t s = as_stream(stream);
    const int nch = (F + kMelChunk - 1) / kMelChunk;
    MelArgs ma{fb_rowptr, fb_col, fb_val, workspace,
               reinterpret_cast<double*>(workspace + (((int64_t)B * F * n_mels + 1) & ~(int64_t)1)), n_mels};
    hipLaunchKernelGGL((stft_power_400_kernel<kMelChunk, true>), dim3(nch, B), dim3(256), 0, s, audio, ld_audio, S,
                       nullptr, F, window, nullptr, 0, 0, ma);
    const int rc = launch_status("vasr_stft_logmel_400_f32");
    if (rc) return rc;
    return mel_chunk_finish(workspace, out, out_stride, frame_off, B, F, n_mels, normalize, s);
}
