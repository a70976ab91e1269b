// Log-mel front end (reference velocity_asr/audio.py:65-143) minus the STFT itself,
// which runs as a windowed-DFT GEMM with the PAIR_POWER epilogue (gemm_f32.hip).
//
//  reflect_pad : audio (B, S) -> xp (B, ld_out): reflect pad n_fft/2 (audio.py:100-101);
//                frames are then rows of stride `hop` of xp (torch.stft center=False).
//  mel_log     : mel[b,f,m] = log(sum_k fb[m,k] P[b,f,k] + 1e-10)   (audio.py:126-129);
//                fb is the 80 x 201 HTK filterbank in CSR form (393 non-zeros).
//  mel_norm    : per (b, m): (x - mean_f) / (std_unbiased_f + 1e-10)   (audio.py:132-135),
//                statistics accumulated in fp64 (exact for constant rows: zero audio -> 0).
#include <algorithm>

#include "vasr_internal.h"

namespace vasr {
namespace {

__global__ void reflect_pad_kernel(const float* __restrict__ audio, int64_t ld_audio, float* __restrict__ xp,
                                   int64_t ld_out, int S, int pad) {
    const int b = blockIdx.y;
    const int64_t total = ld_out;
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < total; j += (int64_t)gridDim.x * blockDim.x) {
        float v = 0.f;
        if (j < (int64_t)S + 2 * pad) {
            int64_t i = j - pad;
            if (i < 0) i = -i;
            if (i >= S) i = 2 * (int64_t)(S - 1) - i;
            v = audio[(int64_t)b * ld_audio + i];
        }
        xp[(int64_t)b * ld_out + j] = v;
    }
}

__global__ void mel_log_kernel(const float* __restrict__ P, int64_t ldp, int64_t stridep,
                               const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                               const float* __restrict__ val, float* __restrict__ tmp, int B, int F, int n_mels) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)B * F * n_mels;
    if (idx >= total) return;
    const int m = idx % n_mels;
    const int64_t bf = idx / n_mels;
    const int b = bf / F, f = bf - (int64_t)b * F;
    const float* prow = P + (int64_t)b * stridep + (int64_t)f * ldp;
    float acc = 0.f;
    for (int e = rowptr[m]; e < rowptr[m + 1]; ++e) acc = __builtin_fmaf(val[e], prow[col[e]], acc);
    tmp[idx] = logf(acc + 1e-10f);
}

// grid (ceil(n_mels/16), B); block 256 = 16 mel bins x 16 frame phases.
__global__ __launch_bounds__(256) void mel_norm_kernel(const float* __restrict__ tmp, float* __restrict__ out,
                                                       int64_t out_stride, int frame_off, int F, int n_mels,
                                                       int normalize) {
    __shared__ double red[16][17];
    __shared__ float stat[2][16];
    const int b = blockIdx.y;
    const int mi = threadIdx.x & 15, ph = threadIdx.x >> 4;
    const int m = blockIdx.x * 16 + mi;
    const bool valid = m < n_mels;
    const float* src = tmp + (int64_t)b * F * n_mels;
    float mean = 0.f, denom = 1.f;
    if (normalize) {
        double s = 0.0;
        if (valid)
            for (int f = ph; f < F; f += 16) s += (double)src[(int64_t)f * n_mels + m];
        red[ph][mi] = s;
        __syncthreads();
        if (ph == 0) {
            double t = 0.0;
            for (int k = 0; k < 16; ++k) t += red[k][mi];
            stat[0][mi] = (float)(t / (double)F);
        }
        __syncthreads();
        mean = stat[0][mi];
        double q = 0.0;
        if (valid)
            for (int f = ph; f < F; f += 16) {
                const double d = (double)src[(int64_t)f * n_mels + m] - (double)mean;
                q += d * d;
            }
        __syncthreads();
        red[ph][mi] = q;
        __syncthreads();
        if (ph == 0) {
            double t = 0.0;
            for (int k = 0; k < 16; ++k) t += red[k][mi];
            // unbiased (torch.std default); F == 1 gives nan like the reference
            stat[1][mi] = (float)sqrt(t / (double)(F - 1));
        }
        __syncthreads();
        denom = stat[1][mi] + 1e-10f;
    }
    if (!valid) return;
    float* dst = out + (int64_t)b * out_stride + (int64_t)frame_off * n_mels;
    for (int f = ph; f < F; f += 16) {
        const float x = src[(int64_t)f * n_mels + m];
        dst[(int64_t)f * n_mels + m] = normalize ? (x - mean) / denom : x;
    }
}

__global__ void pad_frames_kernel(const float* __restrict__ x, float* __restrict__ out, int out_frames, int off,
                                  int F, int C) {
    const int b = blockIdx.y;
    const int64_t n_out = (int64_t)out_frames * C;
    const int64_t lo = (int64_t)off * C, hi = (int64_t)(off + F) * C;
    const float* xb = x + (int64_t)b * F * C;
    float* ob = out + (int64_t)b * n_out;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_out; i += (int64_t)gridDim.x * blockDim.x)
        ob[i] = (i >= lo && i < hi) ? xb[i - lo] : 0.0f;
}

}  // namespace
}  // namespace vasr

VASR_API int vasr_reflect_pad_f32(const float* audio, int64_t ld_audio, float* xp, int64_t ld_out, int B, int S,
                                  int pad, void* stream) {
    using namespace vasr;
    VASR_CHECK_ARG(audio && xp, "vasr_reflect_pad_f32: null pointer");
    VASR_CHECK_ARG(B >= 0 && pad >= 0 && S > pad, "vasr_reflect_pad_f32: reflect padding needs S > pad (S=%d pad=%d)",
                   S, pad);
    VASR_CHECK_ARG(ld_out >= (int64_t)S + 2 * pad, "vasr_reflect_pad_f32: ld_out too small");
    if (B == 0) return VASR_OK;
    const int blocks = (int)std::min<int64_t>((ld_out + 255) / 256, (int64_t)1024);
    hipLaunchKernelGGL(reflect_pad_kernel, dim3(blocks, B), dim3(256), 0, as_stream(stream), audio, ld_audio, xp,
                       ld_out, S, pad);
    return launch_status("vasr_reflect_pad_f32");
}

VASR_API int vasr_mel_log_norm_f32(const float* power, int64_t ld_power, int64_t stride_power,
                                   const int32_t* fb_rowptr, const int32_t* fb_col, const float* fb_val, float* out,
                                   int64_t out_stride, int frame_off, int B, int F, int n_mels, int normalize,
                                   float* workspace, void* stream) {
    using namespace vasr;
    VASR_CHECK_ARG(power && fb_rowptr && fb_col && fb_val && out && workspace, "vasr_mel_log_norm_f32: null pointer");
    VASR_CHECK_ARG(B >= 0 && F >= 1 && n_mels >= 1 && frame_off >= 0, "vasr_mel_log_norm_f32: bad shape");
    VASR_CHECK_ARG(out_stride >= (int64_t)(F + frame_off) * n_mels, "vasr_mel_log_norm_f32: out_stride too small");
    if (B == 0) return VASR_OK;
    hipStream_t s = as_stream(stream);
    const int64_t total = (int64_t)B * F * n_mels;
    hipLaunchKernelGGL(mel_log_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, power, ld_power,
                       stride_power, fb_rowptr, fb_col, fb_val, workspace, B, F, n_mels);
    int rc = launch_status("vasr_mel_log_norm_f32/log");
    if (rc) return rc;
    hipLaunchKernelGGL(mel_norm_kernel, dim3((n_mels + 15) / 16, B), dim3(256), 0, s, workspace, out, out_stride,
                       frame_off, F, n_mels, normalize);
    return launch_status("vasr_mel_log_norm_f32/norm");
}

VASR_API int64_t vasr_mel_workspace_floats(int B, int F, int n_mels) { return (int64_t)B * F * n_mels; }

VASR_API int vasr_pad_frames_f32(const float* x, float* out, int out_frames, int off, int B, int F, int C,
                                 void* stream) {
    using namespace vasr;
    VASR_CHECK_ARG(x && out, "vasr_pad_frames_f32: null pointer");
    VASR_CHECK_ARG(out_frames >= F + off && off >= 0 && F >= 0 && C >= 1, "vasr_pad_frames_f32: bad layout");
    if (B == 0) return VASR_OK;
    const int blocks = (int)std::min<int64_t>(((int64_t)out_frames * C + 255) / 256, (int64_t)1024);
    hipLaunchKernelGGL(pad_frames_kernel, dim3(blocks, B), dim3(256), 0, as_stream(stream), x, out, out_frames, off,
                       F, C);
    return launch_status("vasr_pad_frames_f32");
}
