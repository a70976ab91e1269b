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

// Chunked form of mel_log + mel_norm (used when the filterbank fits the LDS tables): blocks of
// kFC frames per utterance, so the grid is B * ceil(F / kFC) blocks (1008 at B = 16, F = 1001):
//  A (mel_chunk_log_kernel): stage the chunk's power rows (coalesced) and the CSR in LDS, write
//    the log-mel rows to the workspace and per-(chunk, bin) fp64 sums of x and x^2;
//  B (mel_chunk_norm_kernel): per bin, the chunk partials summed in chunk order (deterministic):
//    mean = S / F, unbiased var = (Q - S mean) / (F - 1) in fp64 (exact mean for constant rows,
//    so silent audio still gives 0), then the chunk's normalised rows.
constexpr int kFC = kMelChunk;  // frames per chunk (vasr_internal.h)
constexpr int kMaxLdp = 256;
constexpr int kMaxNnz = 1024;
constexpr int kMaxMels = 85;  // 3 bins-wide phases of a 256-thread block

__global__ __launch_bounds__(256) void mel_chunk_log_kernel(const float* __restrict__ P, int64_t ldp, int64_t stridep,
                                                            const int32_t* __restrict__ rowptr,
                                                            const int32_t* __restrict__ col,
                                                            const float* __restrict__ val, float* __restrict__ tmp,
                                                            double* __restrict__ part, int F, int n_mels,
                                                            const int32_t* __restrict__ frames) {
    __shared__ float rows[kFC * kMaxLdp];
    __shared__ float vals[kFC * kMaxMels];
    __shared__ int rp_s[kMaxMels + 1];
    __shared__ int col_s[kMaxNnz];
    __shared__ float val_s[kMaxNnz];
    const int nch = gridDim.x;
    int b = blockIdx.y, c = blockIdx.x;
    if (VASR_FE_XCD & 2) {  // the STFT's (b, frame) runs per XCD: its power rows are read from this L2
        const int w = xcd_run(c + b * nch, nch * (int)gridDim.y);
        b = w / nch;
        c = w - b * nch;
    }
    const int f0 = c * kFC;
    const int nf = min(kFC, F - f0);
    const int nnz = rowptr[n_mels];
    const bool csr_lds = nnz <= kMaxNnz;  // else read the CSR from global memory
    for (int i = threadIdx.x; i <= n_mels; i += blockDim.x) rp_s[i] = rowptr[i];
    if (csr_lds)
        for (int i = threadIdx.x; i < nnz; i += blockDim.x) {
            col_s[i] = col[i];
            val_s[i] = val[i];
        }
    const float* Pb = P + (int64_t)b * stridep + (int64_t)f0 * ldp;
    const int nrow = nf * (int)ldp;
    for (int i0 = threadIdx.x; i0 < nrow; i0 += 8 * 256) {  // 8 independent loads in flight per thread
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = (i0 + u * 256 < nrow) ? Pb[i0 + u * 256] : 0.f;
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (i0 + u * 256 < nrow) rows[i0 + u * 256] = v[u];
    }
    __syncthreads();
    float* tb = tmp + ((int64_t)b * F + f0) * n_mels;
    for (int i = threadIdx.x; i < nf * n_mels; i += blockDim.x) {
        const int fl = i / n_mels, m = i - fl * n_mels;
        const float* prow = rows + fl * ldp;
        float acc = 0.f;
        if (csr_lds) {
            // 8 entries' indices, weights and power values read before their fmas (independent
            // LDS reads in flight instead of two dependent round trips per entry), fmas in
            // entry order: the same sum
            const int e1 = rp_s[m + 1];
            for (int e0 = rp_s[m]; e0 < e1; e0 += 8) {
                int cj[8];
                float wj[8], pj[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    cj[j] = e0 + j < e1 ? col_s[e0 + j] : 0;
                    wj[j] = e0 + j < e1 ? val_s[e0 + j] : 0.f;
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) pj[j] = prow[cj[j]];
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (e0 + j < e1) acc = __builtin_fmaf(wj[j], pj[j], acc);
            }
        } else
            for (int e = rp_s[m]; e < rp_s[m + 1]; ++e) acc = __builtin_fmaf(val[e], prow[col[e]], acc);
        const float v = logf(acc + 1e-10f);
        vals[i] = v;
        tb[i] = v;
    }
    __syncthreads();
    // frames (optional): only this utterance's own frames enter its statistics
    const int nfs = frames ? max(min(nf, frames[b] - f0), 0) : nf;
    for (int m = threadIdx.x; m < n_mels; m += blockDim.x) {
        double S = 0.0, Q = 0.0;
        for (int fl = 0; fl < nfs; ++fl) {
            const double v = (double)vals[fl * n_mels + m];
            S += v;
            Q += v * v;
        }
        double* pp = part + (((int64_t)b * nch + c) * n_mels + m) * 2;
        pp[0] = S;
        pp[1] = Q;
    }
}

// Per (b, bin): the chunk partials summed in a fixed order (3 interleaved phases, then the
// phases in order) -> {mean, std + 1e-10} as floats.
// One workgroup per utterance; up to kStatPh phases of n_mels threads each sum a strided subset
// of the chunk partials (4 accumulator pairs, loads in flight together), then the phases are
// combined in a fixed order.  1024 threads: ~5 chunks per thread at F = 1001, so the kernel is
// two memory round trips long instead of six (10.4 -> see DESIGN).
constexpr int kStatPh = 12;
__global__ __launch_bounds__(1024) void mel_chunk_stats_kernel(const double* __restrict__ part, float* __restrict__ stats,
                                                               int nch, int F, int n_mels, int normalize,
                                                               const int32_t* __restrict__ frames) {
    __shared__ double red[2][kStatPh][kMaxMels];
    const int b = blockIdx.x;
    if (frames) F = frames[b];  // chunks past the utterance's end hold zero partials
    const int m = threadIdx.x % n_mels, ph = threadIdx.x / n_mels;  // phases of n_mels threads (n_mels <= 85)
    const int nph = min(kStatPh, (int)blockDim.x / n_mels);
    if (ph < nph) {
        // four independent accumulator pairs (loads in flight together), combined in a fixed order
        double S[4] = {0.0, 0.0, 0.0, 0.0}, Q[4] = {0.0, 0.0, 0.0, 0.0};
        for (int k0 = ph; k0 < nch; k0 += 4 * nph) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int k = k0 + u * nph;
                if (k < nch) {
                    const double* pp = part + (((int64_t)b * nch + k) * n_mels + m) * 2;
                    S[u] += pp[0];
                    Q[u] += pp[1];
                }
            }
        }
        red[0][ph][m] = (S[0] + S[1]) + (S[2] + S[3]);
        red[1][ph][m] = (Q[0] + Q[1]) + (Q[2] + Q[3]);
    }
    __syncthreads();
    if (threadIdx.x < n_mels) {
        double S = 0.0, Q = 0.0;
        for (int q = 0; q < nph; ++q) {
            S += red[0][q][m];
            Q += red[1][q][m];
        }
        float mean = 0.f, denom = 1.f;
        if (normalize) {
            const double mu = S / (double)F;
            // unbiased (torch.std default); F == 1 gives nan like the reference
            const double var = fmax(Q - S * mu, 0.0) / (double)(F - 1);
            mean = (float)mu;
            denom = (float)sqrt(var) + 1e-10f;
        }
        stats[((int64_t)b * n_mels + m) * 2] = mean;
        stats[((int64_t)b * n_mels + m) * 2 + 1] = denom;
    }
}

__global__ __launch_bounds__(256) void mel_chunk_norm_kernel(const float* __restrict__ tmp,
                                                             const float* __restrict__ stats, float* __restrict__ out,
                                                             int64_t out_stride, int frame_off, int F, int n_mels,
                                                             int normalize, const int32_t* __restrict__ frames) {
    __shared__ float st_s[2 * kMaxMels];
    int b = blockIdx.y, c = blockIdx.x;
    if (VASR_FE_XCD & 4) {  // the log pass's runs: its log-mel rows are read from this L2
        const int w = xcd_run(c + b * (int)gridDim.x, (int)(gridDim.x * gridDim.y));
        b = w / (int)gridDim.x;
        c = w - b * (int)gridDim.x;
    }
    const int f0 = c * kFC;
    const int nf = min(kFC, F - f0);
    const int nv = frames ? max(min(nf, frames[b] - f0), 0) : nf;  // frames past the utterance's end -> 0
    for (int i = threadIdx.x; i < 2 * n_mels; i += blockDim.x) st_s[i] = stats[(int64_t)b * n_mels * 2 + i];
    __syncthreads();
    const float* tb = tmp + ((int64_t)b * F + f0) * n_mels;
    float* dst = out + (int64_t)b * out_stride + (int64_t)(frame_off + f0) * n_mels;
    for (int i = threadIdx.x; i < nf * n_mels; i += blockDim.x) {
        const int m = i % n_mels;
        const float x = tb[i];
        dst[i] = i >= nv * n_mels ? 0.0f : normalize ? (x - st_s[2 * m]) / st_s[2 * m + 1] : x;
    }
    // the zero frames of a padded layout: [0, frame_off) by the first chunk, [frame_off + F,
    // out_stride / n_mels) by the last (the temporal conv's zero padding, no separate pass)
    float* ob = out + (int64_t)b * out_stride;
    if (c == 0)
        for (int i = threadIdx.x; i < frame_off * n_mels; i += blockDim.x) ob[i] = 0.0f;
    if (c == gridDim.x - 1) {
        const int64_t lo = (int64_t)(frame_off + F) * n_mels, hi = out_stride / n_mels * n_mels;
        for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) ob[i] = 0.0f;
    }
}

// The same zero frames for the unchunked path (n_mels > kMaxMels or wide power rows).
__global__ void zero_frames_kernel(float* __restrict__ out, int64_t out_stride, int frame_off, int F, int n_mels) {
    float* ob = out + (int64_t)blockIdx.x * out_stride;
    const int64_t lo = (int64_t)(frame_off + F) * n_mels, hi = out_stride / n_mels * n_mels;
    for (int64_t i = threadIdx.x; i < hi; i += blockDim.x)
        if (i < (int64_t)frame_off * n_mels || i >= lo) ob[i] = 0.0f;
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

// Stats + normalisation passes of the chunked front end over the workspace written by the
// chunk-log pass (mel_chunk_log_kernel).
int mel_chunk_finish(float* workspace, float* out, int64_t out_stride, int frame_off, int B, int F, int n_mels,
                     int normalize, hipStream_t s, const int32_t* frames) {
    const int nch = (F + kFC - 1) / kFC;
    double* part = reinterpret_cast<double*>(workspace + (((int64_t)B * F * n_mels + 1) & ~(int64_t)1));
    float* stats = reinterpret_cast<float*>(part + (int64_t)B * nch * n_mels * 2);
    hipLaunchKernelGGL(mel_chunk_stats_kernel, dim3(B), dim3(1024), 0, s, part, stats, nch, F, n_mels, normalize,
                       frames);
    int rc = launch_status("mel stats");
    if (rc) return rc;
    hipLaunchKernelGGL(mel_chunk_norm_kernel, dim3(nch, B), dim3(256), 0, s, workspace, stats, out, out_stride,
                       frame_off, F, n_mels, normalize, frames);
    return launch_status("mel norm");
}

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

static int mel_log_norm(const float* power, int64_t ld_power, int64_t stride_power, const int32_t* fb_rowptr,
                        const int32_t* fb_col, const float* fb_val, float* out, int64_t out_stride, int frame_off,
                        int B, int F, int n_mels, int normalize, float* workspace, const int32_t* frames,
                        void* stream, const char* who) {
    using namespace vasr;
    VASR_CHECK_ARG(power && fb_rowptr && fb_col && fb_val && out && workspace, "%s: null pointer", who);
    VASR_CHECK_ARG(B >= 0 && F >= 1 && n_mels >= 1 && frame_off >= 0, "%s: bad shape", who);
    VASR_CHECK_ARG(out_stride >= (int64_t)(F + frame_off) * n_mels, "%s: out_stride too small", who);
    if (B == 0) return VASR_OK;
    hipStream_t s = as_stream(stream);
    if (ld_power <= kMaxLdp && n_mels <= kMaxMels) {
        // the chunked pair (the CSR goes to LDS when it has <= kMaxNnz entries: the 80 x 201
        // HTK bank has 393)
        const int nch = (F + kFC - 1) / kFC;
        double* part = reinterpret_cast<double*>(workspace + (((int64_t)B * F * n_mels + 1) & ~(int64_t)1));
        hipLaunchKernelGGL(mel_chunk_log_kernel, dim3(nch, B), dim3(256), 0, s, power, ld_power, stride_power,
                           fb_rowptr, fb_col, fb_val, workspace, part, F, n_mels, frames);
        int rc = launch_status(who);
        if (rc) return rc;
        return mel_chunk_finish(workspace, out, out_stride, frame_off, B, F, n_mels, normalize, s, frames);
    }
    VASR_CHECK_ARG(!frames, "%s: per-utterance frame counts need ld_power <= %d and n_mels <= %d", who, kMaxLdp,
                   kMaxMels);
    const int64_t total = (int64_t)B * F * n_mels;
    hipLaunchKernelGGL(mel_log_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, power, ld_power,
                       stride_power, fb_rowptr, fb_col, fb_val, workspace, B, F, n_mels);
    int rc = launch_status(who);
    if (rc) return rc;
    hipLaunchKernelGGL(mel_norm_kernel, dim3((n_mels + 15) / 16, B), dim3(256), 0, s, workspace, out, out_stride,
                       frame_off, F, n_mels, normalize);
    rc = launch_status(who);
    if (rc || (frame_off == 0 && out_stride / n_mels == F)) return rc;
    hipLaunchKernelGGL(zero_frames_kernel, dim3(B), dim3(256), 0, s, out, out_stride, frame_off, F, n_mels);
    return launch_status(who);
}

VASR_API int vasr_mel_log_norm_f32(const float* power, int64_t ld_power, int64_t stride_power,
                                   const int32_t* fb_rowptr, const int32_t* fb_col, const float* fb_val, float* out,
                                   int64_t out_stride, int frame_off, int B, int F, int n_mels, int normalize,
                                   float* workspace, void* stream) {
    return mel_log_norm(power, ld_power, stride_power, fb_rowptr, fb_col, fb_val, out, out_stride, frame_off, B, F,
                        n_mels, normalize, workspace, nullptr, stream, "vasr_mel_log_norm_f32");
}

// frames[b] <= F (device): utterance b's own frame count.  Its statistics cover those frames
// only (the same sums, in the same order, as the utterance alone) and its frames past them are
// written as 0 (the zero padding the stride-2 temporal conv then sees).
VASR_API int vasr_mel_log_norm_var_f32(const float* power, int64_t ld_power, int64_t stride_power,
                                       const int32_t* fb_rowptr, const int32_t* fb_col, const float* fb_val,
                                       float* out, int64_t out_stride, int frame_off, int B, int F, int n_mels,
                                       int normalize, const int32_t* frames, float* workspace, void* stream) {
    VASR_CHECK_ARG(frames, "vasr_mel_log_norm_var_f32: null frames");
    return mel_log_norm(power, ld_power, stride_power, fb_rowptr, fb_col, fb_val, out, out_stride, frame_off, B, F,
                        n_mels, normalize, workspace, frames, stream, "vasr_mel_log_norm_var_f32");
}

VASR_API int64_t vasr_mel_workspace_floats(int B, int F, int n_mels) {
    const int64_t nch = (F + vasr::kFC - 1) / vasr::kFC;
    // log-mel rows + fp64 (S, Q) partials per (chunk, bin) + {mean, denom} per bin
    return (((int64_t)B * F * n_mels + 1) & ~(int64_t)1) + 4 * (int64_t)B * nch * n_mels + 2 * (int64_t)B * n_mels;
}

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
