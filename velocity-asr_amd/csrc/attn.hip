// Hierarchical global context pieces that are not GEMMs (reference velocity_asr/attention.py):
//  adaptive_pool     : F.adaptive_avg_pool1d over time (AdaptivePool.forward, :69-73).
//  pooled_attention  : softmax(q k^T / sqrt(hd)) v of MultiHeadAttention.forward (:143-160)
//                      where the keys/values are the <= 64 pooled global tokens.  With so few
//                      keys the whole K/V set of an utterance sits in LDS and every
//                      (token, head) is one thread: two passes over the keys (max, then
//                      exp-sum and weighted V), no score matrix in HBM.
#include "vasr_internal.h"

namespace vasr {
namespace {

__global__ void adaptive_pool_kernel(const float* __restrict__ x, float* __restrict__ out, int B, int L, int C, int K) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)B * K * C;
    if (idx >= total) return;
    const int c = idx % C;
    const int64_t bi = idx / C;
    const int i = bi % K;
    const int b = bi / K;
    const int s = (int)(((int64_t)i * L) / K);
    const int e = (int)(((int64_t)(i + 1) * L + K - 1) / K);
    const float* xb = x + ((int64_t)b * L) * C + c;
    float acc = 0.f;
    for (int t = s; t < e; ++t) acc += xb[(int64_t)t * C];
    out[idx] = acc / (float)(e - s);
}

constexpr int kMaxKeys = 64;
constexpr int kMaxHd = 32;
constexpr int kMaxA = 256;  // heads * head_dim (LDS: Kp * 2A floats <= 128 KiB)

// grid (ceil(L*heads/256), B); one thread per (token, head).  HD = head_dim as a compile-time
// constant (the model's 12, and 8 / 16), 0 = runtime head_dim <= kMaxHd with guarded loops.
template <int HD>
__global__ __launch_bounds__(256) void pooled_attention_kernel(const float* __restrict__ q, int64_t ld_q,
                                                               const float* __restrict__ kv, float* __restrict__ out,
                                                               int L, int Kp, int heads, int hd_rt) {
    constexpr int JM = HD ? HD : kMaxHd;
    const int hd = HD ? HD : hd_rt;
    extern __shared__ __attribute__((aligned(16))) float kvs[];  // Kp x 2A
    const int b = blockIdx.y;
    const int A = heads * hd;
    const float* kvb = kv + (int64_t)b * Kp * 2 * A;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = idx < L * heads;
    const int t = live ? idx / heads : 0, hh = live ? idx - t * heads : 0;
    // issue the query loads before the K/V staging so both latencies overlap
    const float* qr = q + ((int64_t)b * L + t) * ld_q + hh * hd;
    float qv[JM];
#pragma unroll
    for (int j = 0; j < JM; ++j) qv[j] = (live && j < hd) ? qr[j] : 0.f;
    const int n4 = (Kp * 2 * A) / 4;  // K/V set is whole float4s (A % 4 == 0 is checked)
    for (int i = threadIdx.x; i < n4; i += blockDim.x)
        reinterpret_cast<float4*>(kvs)[i] = reinterpret_cast<const float4*>(kvb)[i];
    __syncthreads();
    if (!live) return;
    const float scale = sqrtf((float)hd);
    float mx = -INFINITY;
    for (int k = 0; k < Kp; ++k) {
        const float* kr = kvs + k * 2 * A + hh * hd;
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < JM; ++j)
            if (j < hd) s = __builtin_fmaf(qv[j], kr[j], s);
        mx = fmaxf(mx, s / scale);
    }
    float acc[JM];
#pragma unroll
    for (int j = 0; j < JM; ++j) acc[j] = 0.f;
    float sum = 0.f;
    for (int k = 0; k < Kp; ++k) {
        const float* kr = kvs + k * 2 * A + hh * hd;
        const float* vr = kvs + k * 2 * A + A + hh * hd;
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < JM; ++j)
            if (j < hd) s = __builtin_fmaf(qv[j], kr[j], s);
        const float p = expf(s / scale - mx);
        sum += p;
#pragma unroll
        for (int j = 0; j < JM; ++j)
            if (j < hd) acc[j] = __builtin_fmaf(p, vr[j], acc[j]);
    }
    const float inv = 1.0f / sum;
    float* orow = out + ((int64_t)b * L + t) * A + hh * hd;
#pragma unroll
    for (int j = 0; j < JM; ++j)
        if (j < hd) orow[j] = acc[j] * inv;
}

}  // namespace
}  // namespace vasr

VASR_API int vasr_adaptive_pool_f32(const float* x, float* out, int B, int L, int C, int K, void* stream) {
    using namespace vasr;
    VASR_CHECK_ARG(x && out, "vasr_adaptive_pool_f32: null pointer");
    VASR_CHECK_ARG(B >= 0 && L >= 1 && C >= 1 && K >= 1 && K <= L, "vasr_adaptive_pool_f32: need 1 <= K <= L (K=%d L=%d)",
                   K, L);
    if (B == 0) return VASR_OK;
    const int64_t total = (int64_t)B * K * C;
    hipLaunchKernelGGL(adaptive_pool_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, as_stream(stream), x,
                       out, B, L, C, K);
    return launch_status("vasr_adaptive_pool_f32");
}

VASR_API int vasr_pooled_attention_f32(const float* q, int64_t ld_q, const float* kv, float* out, int B, int L, int Kp,
                                       int heads, int head_dim, void* stream) {
    using namespace vasr;
    VASR_CHECK_ARG(q && kv && out, "vasr_pooled_attention_f32: null pointer");
    VASR_CHECK_ARG(Kp >= 1 && Kp <= kMaxKeys && head_dim >= 1 && head_dim <= kMaxHd && heads >= 1 &&
                       heads * head_dim <= kMaxA && L >= 0 && B >= 0,
                   "vasr_pooled_attention_f32: unsupported shape Kp=%d heads=%d head_dim=%d", Kp, heads, head_dim);
    if (B == 0 || L == 0) return VASR_OK;
    const int work = L * heads;
    const size_t lds = (size_t)Kp * 2 * heads * head_dim * sizeof(float);
    VASR_CHECK_ARG(lds <= 65536, "vasr_pooled_attention_f32: K/V set exceeds 64 KiB of LDS");
    VASR_CHECK_ARG((heads * head_dim) % 4 == 0 && (reinterpret_cast<uintptr_t>(kv) & 15) == 0,
                   "vasr_pooled_attention_f32: heads*head_dim must be a multiple of 4 and kv 16-byte aligned");
    const dim3 grid((work + 255) / 256, B);
    hipStream_t s = as_stream(stream);
    switch (head_dim) {
        case 8: hipLaunchKernelGGL(pooled_attention_kernel<8>, grid, dim3(256), lds, s, q, ld_q, kv, out, L, Kp, heads, 8); break;
        case 12: hipLaunchKernelGGL(pooled_attention_kernel<12>, grid, dim3(256), lds, s, q, ld_q, kv, out, L, Kp, heads, 12); break;
        case 16: hipLaunchKernelGGL(pooled_attention_kernel<16>, grid, dim3(256), lds, s, q, ld_q, kv, out, L, Kp, heads, 16); break;
        default: hipLaunchKernelGGL(pooled_attention_kernel<0>, grid, dim3(256), lds, s, q, ld_q, kv, out, L, Kp, heads, head_dim);
    }
    return launch_status("vasr_pooled_attention_f32");
}
