// LayerNorm and the SSMBlock pre-norm + causal depthwise conv.
//
// Both are HBM-bound row kernels: one wave per 192-float token row, three floats per
// lane, statistics by wave butterfly (no LDS round trip).  The fused LN+dwconv tile
// normalises TT + Kc - 1 rows (the Kc - 1 history rows of the causal window are
// recomputed, not re-read) into LDS and emits TT output rows.
#include "vasr_internal.h"

namespace vasr {
namespace {

constexpr int kMaxPerLane = 16;  // C <= 1024

// CPL: floats per lane as a compile-time constant when C = 64 * CPL (the model's C = 192 is
// CPL = 3), so every load and store is unguarded and all of a row's loads issue before the
// first reduction; CPL = 0 is the generic path (C <= 1024, per-element guards).  Both add the
// same values in the same order (the generic path's extra terms are exact zeros), so the
// result is bitwise the same.
template <int CPL>
constexpr int ln_per_lane() { return CPL > 0 ? CPL : kMaxPerLane; }

// v[i] = column i * 64 + lane of one row (0 past C) -> its LayerNorm, in place (0 past C).
template <int CPL>
__device__ __forceinline__ void ln_vals(float (&v)[ln_per_lane<CPL>()], const float* __restrict__ w,
                                        const float* __restrict__ b, int C, float eps, int lane) {
    constexpr int PL = ln_per_lane<CPL>();
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < PL; ++i) s += v[i];
    const float mean = wave_sum(s) / (float)C;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < PL; ++i) {
        const int c = i * 64 + lane;
        const float d = (CPL > 0 || c < C) ? v[i] - mean : 0.f;
        // explicit fma chain (q starts at 0: the first term is d * d rounded once): a bare
        // q += d * d may be contracted in one kernel and SLP-packed into separate multiplies and
        // adds in another, which moved some rows' variance by an ulp between the kernels that
        // share this function
        q = __builtin_fmaf(d, d, q);
    }
    const float var = wave_sum(q) / (float)C;
    const float rstd = 1.0f / sqrtf(var + eps);
#pragma unroll
    for (int i = 0; i < PL; ++i) {
        const int c = i * 64 + lane;
        v[i] = (CPL > 0 || c < C) ? __builtin_fmaf((v[i] - mean) * rstd, w[c], b[c]) : 0.f;  // as the GEMM LN prologue
    }
}

// CPL: floats per lane as a compile-time constant when C = 64 * CPL (the model's C = 192 is
// CPL = 3), so every load and store is unguarded and all of a row's loads issue before the
// first reduction; CPL = 0 is the generic path (C <= 1024, per-element guards).  Both add the
// same values in the same order (the generic path's extra terms are exact zeros), so the
// result is bitwise the same.
template <int CPL>
__device__ __forceinline__ void ln_load(float (&v)[ln_per_lane<CPL>()], const float* __restrict__ x, int C, int lane) {
#pragma unroll
    for (int i = 0; i < ln_per_lane<CPL>(); ++i) {
        const int c = i * 64 + lane;
        v[i] = (CPL > 0 || c < C) ? x[c] : 0.f;
    }
}

template <int CPL>
__device__ __forceinline__ void ln_store(const float (&v)[ln_per_lane<CPL>()], float* __restrict__ y, int C, int lane) {
#pragma unroll
    for (int i = 0; i < ln_per_lane<CPL>(); ++i) {
        const int c = i * 64 + lane;
        if (CPL > 0 || c < C) y[c] = v[i];
    }
}

template <int CPL>
__global__ __launch_bounds__(256) void layer_norm_kernel(const float* __restrict__ x, int64_t ldx,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ b, float* y,
                                                         int64_t ldy, int rows, int C, float eps) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const int lane = threadIdx.x & 63;
    float v[ln_per_lane<CPL>()];
    ln_load<CPL>(v, x + (int64_t)row * ldx, C, lane);
    ln_vals<CPL>(v, w, b, C, eps, lane);
    ln_store<CPL>(v, y + (int64_t)row * ldy, C, lane);
}

// y1 = LN1(x), y2 = LN2(y1): the second LayerNorm from the first's registers (the same floats
// it stores, so y2 is bitwise what layer_norm_kernel gives on y1), one read of x instead of two
// launches.  The local stack's final norm and the global context's query norm (attention.py).
template <int CPL>
__global__ __launch_bounds__(256) void layer_norm_pair_kernel(const float* __restrict__ x, int64_t ldx,
                                                              const float* __restrict__ w1,
                                                              const float* __restrict__ b1, float eps1,
                                                              float* __restrict__ y1, int64_t ldy1,
                                                              const float* __restrict__ w2,
                                                              const float* __restrict__ b2, float eps2,
                                                              float* __restrict__ y2, int64_t ldy2, int rows, int C) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const int lane = threadIdx.x & 63;
    float v[ln_per_lane<CPL>()];
    ln_load<CPL>(v, x + (int64_t)row * ldx, C, lane);
    ln_vals<CPL>(v, w1, b1, C, eps1, lane);
    ln_store<CPL>(v, y1 + (int64_t)row * ldy1, C, lane);
    ln_vals<CPL>(v, w2, b2, C, eps2, lane);
    ln_store<CPL>(v, y2 + (int64_t)row * ldy2, C, lane);
}

// LayerNorm of every row, then F.adaptive_avg_pool1d over time (vasr_adaptive_pool_f32's windows and
// in-order sums): the global SSM stack's final norm followed by the second pooling level
// (attention.py).  One wave per (utterance, bin); the window's rows are loaded G at a time before
// they are normalised (ln_vals, layer_norm_kernel's own arithmetic) and added in row order, so the
// result is bitwise the LayerNorm launch + the pooling launch.  lens / ks as adaptive_pool_kernel.
template <int CPL>
__global__ __launch_bounds__(256) void ln_adaptive_pool_kernel(const float* __restrict__ x,
                                                               const float* __restrict__ w,
                                                               const float* __restrict__ bias, float eps,
                                                               float* __restrict__ out, int B, int L, int C, int K,
                                                               const int32_t* __restrict__ lens,
                                                               const int32_t* __restrict__ ks) {
    constexpr int PL = ln_per_lane<CPL>();
    constexpr int G = CPL > 0 ? 8 : 1;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= B * K) return;
    const int lane = threadIdx.x & 63;
    const int b = row / K, i = row - b * K;
    const int Lb = lens ? lens[b] : L, Kb = ks ? ks[b] : K;
    float acc[PL];
#pragma unroll
    for (int k = 0; k < PL; ++k) acc[k] = 0.f;
    float* o = out + (int64_t)row * C;
    if (i >= Kb) {
        ln_store<CPL>(acc, o, C, lane);
        return;
    }
    const int s = (int)(((int64_t)i * Lb) / Kb);
    const int e = (int)(((int64_t)(i + 1) * Lb + Kb - 1) / Kb);
    const float* xb = x + (int64_t)b * L * C;
    for (int t0 = s; t0 < e; t0 += G) {
        float v[G][PL];
#pragma unroll
        for (int j = 0; j < G; ++j)
            if (t0 + j < e) ln_load<CPL>(v[j], xb + (int64_t)(t0 + j) * C, C, lane);
#pragma unroll
        for (int j = 0; j < G; ++j)
            if (t0 + j < e) {  // wave-uniform
                ln_vals<CPL>(v[j], w, bias, C, eps, lane);
#pragma unroll
                for (int k = 0; k < PL; ++k) acc[k] += v[j][k];
            }
    }
#pragma unroll
    for (int k = 0; k < PL; ++k) acc[k] = acc[k] / (float)(e - s);
    ln_store<CPL>(acc, o, C, lane);
}

// TT: output rows per block -- 16 for full-chip launches (1024 blocks at B = 32, L = 501: 4 per
// CU), 8 below 1024 blocks of 16, 4 below 128 (graph-timed at L = 501, bitwise the same outputs:
// B = 1 2.74 / 3.18 / 4.09 us at 4 / 8 / 16 rows, B = 16 5.69 / 5.28 / 5.65, B = 32 9.11 / 8.39 /
// 8.31; 32 rows slower everywhere.  Measured and dropped (patch in profiles/r05at/): a wave-tiled
// form with the causal window in registers (no LDS, no barrier: 8.13 vs 8.35 us at B = 32, slower
// below) and LayerNorm with 2 / 4 rows per wave (5.8 / 6.2 vs 5.5 us at B = 32))
constexpr int kMaxC = 256;   // LDS row capacity
constexpr int kMaxK = 8;

// Phase 1: the 4 waves layer-norm rows t0-(Kc-1) .. t0+TT-1 into LDS (zero rows before t=0).
// Phase 2: thread c owns channel c for all TT rows: taps and bias in registers, a sliding
// window of the last Kc LN values, one LDS read and one coalesced store per output.
// KC: the conv width as a compile-time constant (the model's 4) so the taps, the window and
// the history rows unroll without runtime guards; KC = 0 is the generic path (Kc <= kMaxK at
// run time).  A runtime Kc turned every tap load and window read into its own guarded basic
// block with a wait, serialising ~8 global-load latencies per thread (13.5 -> 4 us at B = 16).
// CPT: floats per lane of a row as a compile-time constant (C = 64 * CPT; the model's 192 is 3),
// 0 = generic (C <= kMaxC, guarded columns).  The channel's taps and bias are loaded before
// phase 1 (C <= kMaxC = 256 threads: one channel per thread), so their latency overlaps the
// row loads instead of following the barrier.
//
// PRE (C = 64 * CPT only): x is the row before a LayerNorm of its own (pre_w, pre_b, pre_eps: the
// temporal binding's norm, model.py), applied to every tile row in registers before norm1 with
// layer_norm_kernel's own arithmetic (ln_vals), and the block's own rows of it stored to xo (the
// SSM block's residual input): bitwise the LayerNorm launch + this kernel on its output.
template <int KC, int CPT, int TT, bool PRE = false>
__global__ __launch_bounds__(256) void ln_dwconv_kernel(const float* __restrict__ x,
                                                        const float* __restrict__ ln_w,
                                                        const float* __restrict__ ln_b,
                                                        const float* __restrict__ cw,
                                                        const float* __restrict__ cb, float* __restrict__ y,
                                                        int L, int C, int Kc_rt, float eps,
                                                        const float* __restrict__ pre_w = nullptr,
                                                        const float* __restrict__ pre_b = nullptr, float pre_eps = 0.f,
                                                        float* __restrict__ xo = nullptr) {
    static_assert(!PRE || CPT > 0, "the pre-norm needs C = 64 * CPT");
    const int Kc = KC > 0 ? KC : Kc_rt;
    constexpr int KM = KC > 0 ? KC : kMaxK;
    __shared__ float tile[(TT + KM - 1) * kMaxC];
    const int b = blockIdx.y;
    const int t0 = blockIdx.x * TT;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nrows = min(TT, L - t0) + Kc - 1;
    const float* xb = x + (int64_t)b * L * C;
    // Each wave normalises rows wave, wave + 4, ...: all of its row loads are issued before
    // the first reduction, so the rows' load latencies and butterfly chains overlap.
    constexpr int RPW = (TT + KM - 1 + 3) / 4;
    constexpr int CPL = CPT > 0 ? CPT : kMaxC / 64;
    const int c_own = threadIdx.x;  // phase-2 channel (C <= 256)
    float w[KM];
    float bias = 0.f;
    if (c_own < C) {
#pragma unroll
        for (int j = 0; j < KM; ++j) w[j] = (KC > 0 || j < Kc) ? cw[c_own * Kc + j] : 0.f;
        bias = cb[c_own];
    }
    float lw[CPL], lb[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
        const int col = c * 64 + lane;
        lw[c] = (CPT > 0 || col < C) ? ln_w[col] : 0.f;
        lb[c] = (CPT > 0 || col < C) ? ln_b[col] : 0.f;
    }
    float v[RPW][CPL];
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
        const int rr = wave + 4 * i;
        const int t = t0 - (Kc - 1) + rr;
        const bool ok = rr < nrows && t >= 0;
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const int col = c * 64 + lane;
            v[i][c] = (ok && (CPT > 0 || col < C)) ? xb[(int64_t)t * C + col] : 0.f;
        }
    }
    if constexpr (PRE) {
        float* xob = xo + (int64_t)b * L * C;
        // every row slot normalised (rows past the tile hold zeros: finite, never stored or used),
        // so the slots' reduction chains carry no branches between them and interleave
#pragma unroll
        for (int i = 0; i < RPW; ++i) ln_vals<CPT>(v[i], pre_w, pre_b, C, pre_eps, lane);
#pragma unroll
        for (int i = 0; i < RPW; ++i) {
            const int rr = wave + 4 * i;
            const int t = t0 - (Kc - 1) + rr;
            if (rr >= Kc - 1 && rr < nrows) ln_store<CPT>(v[i], xob + (int64_t)t * C, C, lane);  // own rows
        }
    }
    float mean[RPW], rstd[RPW];
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
        float sum = 0.f;
#pragma unroll
        for (int c = 0; c < CPL; ++c) sum += v[i][c];
        mean[i] = wave_sum(sum) / (float)C;
    }
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
        float q = 0.f;
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const float d = (CPT > 0 || c * 64 + lane < C) ? v[i][c] - mean[i] : 0.f;
            q = __builtin_fmaf(d, d, q);  // as ln_vals: the same rounding in every instantiation
        }
        rstd[i] = 1.0f / sqrtf(wave_sum(q) / (float)C + eps);
    }
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
        const int rr = wave + 4 * i;
        if (rr >= nrows) continue;
        const int t = t0 - (Kc - 1) + rr;
        float* dst = tile + rr * C;
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const int col = c * 64 + lane;
            if (CPT > 0 || col < C) dst[col] = t < 0 ? 0.f : (v[i][c] - mean[i]) * rstd[i] * lw[c] + lb[c];
        }
    }
    __syncthreads();
    float* yb = y + (int64_t)b * L * C;
    const int rows = min(TT, L - t0);
    if (c_own < C) {
        const int c = c_own;
        float win[KM];
#pragma unroll
        for (int j = 0; j < KM; ++j) win[j] = (j < Kc - 1) ? tile[j * C + c] : 0.f;
        if (KC > 0 && rows == TT) {
            // full tile: every LN row read up front, outputs in straight-line code
            float lv[TT];
#pragma unroll
            for (int tt = 0; tt < TT; ++tt) lv[tt] = tile[(tt + KM - 1) * C + c];
#pragma unroll
            for (int tt = 0; tt < TT; ++tt) {
                float acc = 0.f;
#pragma unroll
                for (int j = 0; j < KM; ++j) {
                    const int r = tt + j - (KM - 1);  // LN row tt + j of the tile
                    acc = __builtin_fmaf(r < 0 ? win[j + tt] : lv[r], w[j], acc);  // one rounding per tap (every path)
                }
                yb[(int64_t)(t0 + tt) * C + c] = acc + bias;
            }
            return;
        }
        for (int tt = 0; tt < rows; ++tt) {
            // window = LN rows tt .. tt + Kc - 1 of the tile (inputs t - Kc + 1 .. t)
            const float v = tile[(tt + Kc - 1) * C + c];
            float acc = 0.f;
#pragma unroll
            for (int j = 0; j < KM; ++j) {
                if (j < Kc - 1) acc = __builtin_fmaf(win[j], w[j], acc);
                else if (j == Kc - 1) acc = __builtin_fmaf(v, w[j], acc);
            }
#pragma unroll
            for (int j = 0; j + 1 < KM; ++j) {
                if (j < Kc - 2) win[j] = win[j + 1];
                else if (j == Kc - 2) win[j] = v;
            }
            yb[(int64_t)(t0 + tt) * C + c] = acc + bias;
        }
    }
}

__global__ void add_table_kernel(const float* __restrict__ x, const float* __restrict__ table, float* __restrict__ out,
                                 int64_t n, int64_t per_batch) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = x[i] + table[i % per_batch];
}

}  // namespace
}  // namespace vasr

VASR_API int vasr_add_table_f32(const float* x, const float* table, float* out, int B, int L, int C, void* stream) {
    using namespace vasr;
    VASR_CHECK_ARG(x && table && out && B >= 0 && L >= 0 && C >= 0, "vasr_add_table_f32: bad arguments");
    const int64_t n = (int64_t)B * L * C;
    if (n == 0) return VASR_OK;
    const int blocks = (int)((n + 255) / 256 < 2048 ? (n + 255) / 256 : 2048);
    hipLaunchKernelGGL(add_table_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), x, table, out, n,
                       (int64_t)L * C);
    return launch_status("vasr_add_table_f32");
}

VASR_API int vasr_layer_norm_f32(const float* x, int64_t ldx, const float* w, const float* b, float* y,
                                 int64_t ldy, int rows, int C, float eps, void* stream) {
    using namespace vasr;
    VASR_CHECK_ARG(x && w && b && y, "vasr_layer_norm_f32: null pointer");
    VASR_CHECK_ARG(C > 0 && C <= 64 * kMaxPerLane && rows >= 0, "vasr_layer_norm_f32: bad shape rows=%d C=%d", rows, C);
    if (rows == 0) return VASR_OK;
    const dim3 grid((rows + 3) / 4), block(256);
    hipStream_t s = as_stream(stream);
    switch (C) {
        case 192: hipLaunchKernelGGL(layer_norm_kernel<3>, grid, block, 0, s, x, ldx, w, b, y, ldy, rows, C, eps); break;
        case 384: hipLaunchKernelGGL(layer_norm_kernel<6>, grid, block, 0, s, x, ldx, w, b, y, ldy, rows, C, eps); break;
        default: hipLaunchKernelGGL(layer_norm_kernel<0>, grid, block, 0, s, x, ldx, w, b, y, ldy, rows, C, eps); break;
    }
    return launch_status("vasr_layer_norm_f32");
}

VASR_API int vasr_layer_norm_pair_f32(const float* x, int64_t ldx, const float* w1, const float* b1, float eps1,
                                      float* y1, int64_t ldy1, const float* w2, const float* b2, float eps2, float* y2,
                                      int64_t ldy2, int rows, int C, void* stream) {
    using namespace vasr;
    VASR_CHECK_ARG(x && w1 && b1 && y1 && w2 && b2 && y2, "vasr_layer_norm_pair_f32: null pointer");
    VASR_CHECK_ARG(C > 0 && C <= 64 * kMaxPerLane && rows >= 0, "vasr_layer_norm_pair_f32: bad shape rows=%d C=%d",
                   rows, C);
    VASR_CHECK_ARG(y1 != y2, "vasr_layer_norm_pair_f32: y1 and y2 must differ");
    if (rows == 0) return VASR_OK;
    const dim3 grid((rows + 3) / 4), block(256);
    hipStream_t s = as_stream(stream);
#define VASR_LN2(CPL)                                                                                                \
    hipLaunchKernelGGL(layer_norm_pair_kernel<CPL>, grid, block, 0, s, x, ldx, w1, b1, eps1, y1, ldy1, w2, b2, eps2, \
                       y2, ldy2, rows, C)
    switch (C) {
        case 192: VASR_LN2(3); break;
        case 384: VASR_LN2(6); break;
        default: VASR_LN2(0); break;
    }
#undef VASR_LN2
    return launch_status("vasr_layer_norm_pair_f32");
}

VASR_API int vasr_ln_dwconv_prenorm_f32(const float* x, const float* pre_w, const float* pre_b, float pre_eps,
                                        float* xo, const float* ln_w, const float* ln_b, const float* conv_w,
                                        const float* conv_b, float* y, int B, int L, int C, int Kc, float eps,
                                        void* stream) {
    using namespace vasr;
    VASR_CHECK_ARG(x && pre_w && pre_b && xo && ln_w && ln_b && conv_w && conv_b && y,
                   "vasr_ln_dwconv_prenorm_f32: null pointer");
    VASR_CHECK_ARG(x != y && x != xo && xo != y, "vasr_ln_dwconv_prenorm_f32: x, xo and y must be distinct");
    VASR_CHECK_ARG(C == 192 && Kc == 4 && B >= 0 && L >= 0,
                   "vasr_ln_dwconv_prenorm_f32: C = 192 and Kc = 4 only (C=%d Kc=%d)", C, Kc);
    if (B == 0 || L == 0) return VASR_OK;
    const dim3 block(256);
    hipStream_t s = as_stream(stream);
    const int n16 = B * ((L + 15) / 16);
    const int tt = option(VASR_OPT_DW_ROWS) ? option(VASR_OPT_DW_ROWS) : n16 < 128 ? 4 : n16 < 1024 ? 8 : 16;
#define VASR_DWP(TT)                                                                                              \
    hipLaunchKernelGGL((ln_dwconv_kernel<4, 3, TT, true>), dim3((L + TT - 1) / TT, B), block, 0, s, x, ln_w, ln_b, \
                       conv_w, conv_b, y, L, C, Kc, eps, pre_w, pre_b, pre_eps, xo)
    if (tt == 4) VASR_DWP(4); else if (tt == 8) VASR_DWP(8); else VASR_DWP(16);
#undef VASR_DWP
    return launch_status("vasr_ln_dwconv_prenorm_f32");
}

VASR_API int vasr_ln_adaptive_pool_f32(const float* x, const float* w, const float* b, float eps, float* out, int B,
                                       int L, int C, int K, const int32_t* lens, const int32_t* ks, void* stream) {
    using namespace vasr;
    VASR_CHECK_ARG(x && w && b && out, "vasr_ln_adaptive_pool_f32: null pointer");
    VASR_CHECK_ARG((lens == nullptr) == (ks == nullptr), "vasr_ln_adaptive_pool_f32: lens and ks go together");
    VASR_CHECK_ARG(B >= 0 && L >= 1 && C >= 1 && C <= 64 * kMaxPerLane && K >= 1 && K <= L,
                   "vasr_ln_adaptive_pool_f32: need 1 <= K <= L and C <= %d (K=%d L=%d C=%d)", 64 * kMaxPerLane, K, L,
                   C);
    if (B == 0) return VASR_OK;
    const dim3 grid((unsigned)(((int64_t)B * K + 3) / 4)), block(256);
    hipStream_t s = as_stream(stream);
    switch (C) {
        case 192:
            hipLaunchKernelGGL(ln_adaptive_pool_kernel<3>, grid, block, 0, s, x, w, b, eps, out, B, L, C, K, lens, ks);
            break;
        default:
            hipLaunchKernelGGL(ln_adaptive_pool_kernel<0>, grid, block, 0, s, x, w, b, eps, out, B, L, C, K, lens, ks);
            break;
    }
    return launch_status("vasr_ln_adaptive_pool_f32");
}

VASR_API int vasr_ln_dwconv_f32(const float* x, const float* ln_w, const float* ln_b, const float* conv_w,
                                const float* conv_b, float* y, int B, int L, int C, int Kc, float eps,
                                void* stream) {
    using namespace vasr;
    VASR_CHECK_ARG(x && ln_w && ln_b && conv_w && conv_b && y, "vasr_ln_dwconv_f32: null pointer");
    VASR_CHECK_ARG(x != y, "vasr_ln_dwconv_f32: in-place not supported");
    VASR_CHECK_ARG(C > 0 && C <= kMaxC && Kc >= 1 && Kc <= kMaxK && B >= 0 && L >= 0,
                   "vasr_ln_dwconv_f32: unsupported shape C=%d Kc=%d", C, Kc);
    if (B == 0 || L == 0) return VASR_OK;
    const dim3 block(256);
    hipStream_t s = as_stream(stream);
    const int n16 = B * ((L + 15) / 16);  // workgroups at 16 rows
    const int tt = option(VASR_OPT_DW_ROWS) ? option(VASR_OPT_DW_ROWS) : n16 < 128 ? 4 : n16 < 1024 ? 8 : 16;
#define VASR_DW(KC, CPT, TT)                                                                                     \
    hipLaunchKernelGGL((ln_dwconv_kernel<KC, CPT, TT>), dim3((L + TT - 1) / TT, B), block, 0, s, x, ln_w, ln_b, \
                       conv_w, conv_b, y, L, C, Kc, eps)
#define VASR_DW_TT(KC, CPT) \
    if (tt == 4) VASR_DW(KC, CPT, 4); else if (tt == 8) VASR_DW(KC, CPT, 8); else VASR_DW(KC, CPT, 16)
    if (Kc == 4 && C == 192) {
        VASR_DW_TT(4, 3);
    } else if (Kc == 4) {
        VASR_DW_TT(4, 0);
    } else {
        VASR_DW_TT(0, 0);
    }
#undef VASR_DW_TT
#undef VASR_DW
    return launch_status("vasr_ln_dwconv_f32");
}
