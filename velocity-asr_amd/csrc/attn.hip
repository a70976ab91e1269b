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

// lens / ks (optional, device): utterance b pools its own first lens[b] rows into ks[b] bins
// (the sizes it has alone); its bins past ks[b] are written as 0.  x keeps the row stride L.
__global__ void adaptive_pool_kernel(const float* __restrict__ x, float* __restrict__ out, int B, int L, int C, int K,
                                     const int32_t* __restrict__ lens, const int32_t* __restrict__ ks) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t total = (int64_t)B * K * C;
    if (idx >= total) return;
    const int c = idx % C;
    const int64_t bi = idx / C;
    const int i = bi % K;
    const int b = bi / K;
    const int Lb = lens ? lens[b] : L, Kb = ks ? ks[b] : K;
    if (i >= Kb) {
        out[idx] = 0.f;
        return;
    }
    const int s = (int)(((int64_t)i * Lb) / Kb);
    const int e = (int)(((int64_t)(i + 1) * Lb + Kb - 1) / Kb);
    const float* xb = x + ((int64_t)b * L) * C + c;
    // the window's rows loaded 8 at a time before they are added (independent loads in flight
    // instead of one load latency per row), then added in row order: the same sum as a plain loop
    float acc = 0.f;
    for (int t0 = s; t0 < e; t0 += 8) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = t0 + j < e ? xb[(int64_t)(t0 + j) * C] : 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (t0 + j < e) acc += v[j];
    }
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
                                                               int L, int Kp, int heads, int hd_rt,
                                                               const int32_t* __restrict__ kps) {
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
    // kps (optional): utterance b attends over its own first kps[b] keys (batch stride stays Kp)
    const int Kb = kps ? kps[b] : Kp;
    for (int i = threadIdx.x; i < n4; i += blockDim.x)
        reinterpret_cast<float4*>(kvs)[i] = reinterpret_cast<const float4*>(kvb)[i];
    __syncthreads();
    if (!live) return;
    const float scale = sqrtf((float)hd);
    float mx = -INFINITY;
    for (int k = 0; k < Kb; ++k) {
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
    for (int k = 0; k < Kb; ++k) {
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

static int adaptive_pool(const float* x, float* out, int B, int L, int C, int K, const int32_t* lens,
                         const int32_t* ks, void* stream, const char* who) {
    using namespace vasr;
    VASR_CHECK_ARG(x && out, "%s: null pointer", who);
    VASR_CHECK_ARG(B >= 0 && L >= 1 && C >= 1 && K >= 1 && K <= L, "%s: need 1 <= K <= L (K=%d L=%d)", who, K, L);
    if (B == 0) return VASR_OK;
    const int64_t total = (int64_t)B * K * C;
    hipLaunchKernelGGL(adaptive_pool_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, as_stream(stream), x,
                       out, B, L, C, K, lens, ks);
    return launch_status(who);
}

VASR_API int vasr_adaptive_pool_f32(const float* x, float* out, int B, int L, int C, int K, void* stream) {
    return adaptive_pool(x, out, B, L, C, K, nullptr, nullptr, stream, "vasr_adaptive_pool_f32");
}

// Per-utterance sizes (device): 1 <= ks[b] <= lens[b] <= L, ks[b] <= K.
VASR_API int vasr_adaptive_pool_var_f32(const float* x, float* out, int B, int L, int C, int K, const int32_t* lens,
                                        const int32_t* ks, void* stream) {
    VASR_CHECK_ARG(lens && ks, "vasr_adaptive_pool_var_f32: null lens / ks");
    return adaptive_pool(x, out, B, L, C, K, lens, ks, stream, "vasr_adaptive_pool_var_f32");
}

static int pooled_attention(const float* q, int64_t ld_q, const float* kv, float* out, int B, int L, int Kp,
                            int heads, int head_dim, const int32_t* kps, void* stream, const char* who) {
    using namespace vasr;
    VASR_CHECK_ARG(q && kv && out, "%s: null pointer", who);
    VASR_CHECK_ARG(Kp >= 1 && Kp <= kMaxKeys && head_dim >= 1 && head_dim <= kMaxHd && heads >= 1 &&
                       heads * head_dim <= kMaxA && L >= 0 && B >= 0,
                   "%s: unsupported shape Kp=%d heads=%d head_dim=%d", who, Kp, heads, head_dim);
    if (B == 0 || L == 0) return VASR_OK;
    const int work = L * heads;
    const size_t lds = (size_t)Kp * 2 * heads * head_dim * sizeof(float);
    VASR_CHECK_ARG(lds <= 65536, "%s: K/V set exceeds 64 KiB of LDS", who);
    VASR_CHECK_ARG((heads * head_dim) % 4 == 0 && (reinterpret_cast<uintptr_t>(kv) & 15) == 0,
                   "%s: heads*head_dim must be a multiple of 4 and kv 16-byte aligned", who);
    const dim3 grid((work + 255) / 256, B);
    hipStream_t s = as_stream(stream);
    switch (head_dim) {
        case 8: hipLaunchKernelGGL(pooled_attention_kernel<8>, grid, dim3(256), lds, s, q, ld_q, kv, out, L, Kp, heads, 8, kps); break;
        case 12: hipLaunchKernelGGL(pooled_attention_kernel<12>, grid, dim3(256), lds, s, q, ld_q, kv, out, L, Kp, heads, 12, kps); break;
        case 16: hipLaunchKernelGGL(pooled_attention_kernel<16>, grid, dim3(256), lds, s, q, ld_q, kv, out, L, Kp, heads, 16, kps); break;
        default: hipLaunchKernelGGL(pooled_attention_kernel<0>, grid, dim3(256), lds, s, q, ld_q, kv, out, L, Kp, heads, head_dim, kps);
    }
    return launch_status(who);
}

VASR_API int vasr_pooled_attention_f32(const float* q, int64_t ld_q, const float* kv, float* out, int B, int L, int Kp,
                                       int heads, int head_dim, void* stream) {
    return pooled_attention(q, ld_q, kv, out, B, L, Kp, heads, head_dim, nullptr, stream,
                            "vasr_pooled_attention_f32");
}

// kps (device): 1 <= kps[b] <= Kp keys for utterance b (kv keeps the batch stride Kp * 2A).
VASR_API int vasr_pooled_attention_var_f32(const float* q, int64_t ld_q, const float* kv, float* out, int B, int L,
                                           int Kp, int heads, int head_dim, const int32_t* kps, void* stream) {
    VASR_CHECK_ARG(kps, "vasr_pooled_attention_var_f32: null kps");
    return pooled_attention(q, ld_q, kv, out, B, L, Kp, heads, head_dim, kps, stream,
                            "vasr_pooled_attention_var_f32");
}
