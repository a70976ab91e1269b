// Split-bf16 fp32 GEMM with LDS-resident weight panels (the model's K = 192 / 384 GEMMs).
//
// The tile kernel (gemm_x3.hip) streams both operands through a two-stage LDS ring and
// waits for every stage: its loads, MFMAs and stores serialise per block.  Here each block
// owns one 64-column panel of the split weight planes for the WHOLE of K (72 KiB at K = 192,
// 144 KiB at K = 384), loaded once, and its waves walk 32-row slabs of A:
//  * A never touches LDS: each lane loads its own MFMA fragment rows (8 consecutive k per
//    k-step, 2 x 16 B) straight into a register ring of R chunks x KC k-steps, R - 1 chunks
//    ahead, and the ring runs on across slab boundaries, so the next slab's operands are in
//    flight while this slab finishes and its epilogue stores drain;
//  * W fragments are conflict-free linear ds_read_b128 of the panel;
//  * the epilogue's per-column constants (bias, fake-quant parameters) are loaded once per
//    block, and per-element aux rows (residual, positional table) are issued before the next
//    slab's prefetch, so no epilogue load waits behind the prefetch.
// The MFMA sequence per output element (k-steps in order, the six split products in the tile
// kernel's order) is the tile kernel's, so the two engines agree bit for bit
// (tests/test_gemm_panel.py).
//
// Measured (profiles/r01_gemm_panel.txt): NOT faster than the tile kernel on the model's shapes
// except x_proj at M = 16032 (-14 %); slower for N = 192 (3 panels leave most waves idle) and
// at the bench's 16-clip M = 8016.  An MFMA-only ablation of this kernel already takes 26 us
// for in_proj (vs a 14 us issue bound), so the per-wave serialisation the panels were meant
// to remove is not the binding limit.  Kept as an opt-in engine (VASR_GEMM_PANEL=1: 4 waves
// per SIMD, 2: 2 waves per SIMD with a deeper ring) for further work; the default is tiles.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "gemm_common.h"
#include "gemm_split.h"

namespace vasr {
namespace {

using namespace gemm;

#ifndef VASR_PANEL_ABLATE
#define VASR_PANEL_ABLATE 0  // diagnostic builds only: 1 no MFMA, 2 no C stores, 4 no A loads in the
#endif                       // loop, 8 no W LDS reads in the loop, 16 no A split

constexpr int TN = 2;  // 32-column MFMA tiles per panel (64 columns)
// Configurations (KS = K / 16; NW waves per block; BPC blocks per CU; R chunks of KC k-steps
// in the A register ring; PIPE: W fragments read one k-step ahead and aux rows preloaded — for
// 2 waves per SIMD, where nothing else hides those latencies; at 4 waves per SIMD the register
// budget (128) takes plain in-step reads instead).
template <int KS, int NW, int BPC, int R, int KC, bool PIPE, int EPI>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(NW * BPC / 4, NW * BPC / 4)))
void gemm_panel_kernel(GemmParams p, int np, int groups) {
    constexpr int CPS = KS / KC;
    static_assert(KS % KC == 0 && CPS % R == 0, "a slab is a whole number of ring turns");
    constexpr int PANEL = TN * KS * 3 * 1024;  // [TN][KS][3 planes][64 lanes][16 B]
    constexpr int PIECES = PANEL / 16;
    constexpr int PER_T = PIECES / (64 * NW);
    static_assert(PIECES % (64 * NW) == 0, "whole 16-B pieces per thread");
    constexpr bool kAux = false;  // aux preload (32 VGPRs) spills at 2 waves per SIMD: read in the epilogue
    __shared__ __attribute__((aligned(16))) char wl[PANEL];
    __shared__ float4 col_q[32 * TN];  // per-column fake-quant parameters
    __shared__ float col_b[32 * TN];   // per-column bias

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // slab indices stay scalar
    const int r = lane & 31, h = lane >> 5;
    const int panel = (int)blockIdx.x % np, grp = (int)blockIdx.x / np;
    const int n0 = panel * 32 * TN;
    const int NT = (p.N + 31) / 32;

    // 1. the weight panel (tiles past N re-read the last tile: finite, never stored)
    const float4* __restrict__ wsrc = reinterpret_cast<const float4*>(p.Wx);
    float4 wv[PER_T];
#pragma unroll
    for (int i = 0; i < PER_T; ++i) {
        const int idx = tid + i * 64 * NW;
        const int tl = idx / (KS * 192);
        const int nt = min(n0 / 32 + tl, NT - 1);
        wv[i] = wsrc[(int64_t)nt * KS * 192 + (idx - tl * KS * 192)];
    }

    // 2. A fragments: lane (r, h) holds row r of the slab, k = 16 ks + 8 h .. +7.  Rows past M
    //    re-read row M-1 (finite, never stored).
    const int Sb = (p.M + 31) / 32;
    const int S = Sb * p.batch;
    const int stride = groups * NW;
    float4 ra[R][KC][2];
    auto row_ptr = [&](int slab) {
        const int bz = slab / Sb;
        const int m = min((slab - bz * Sb) * 32 + r, p.M - 1);
        return p.A + (int64_t)bz * p.stride_a + (int64_t)m * p.lda;
    };
    // K == 16 * KS (host check): fragment k offsets are immediates off one row pointer
    auto kofs = [&](int ks) { return ks * 16 + 8 * h; };
    // Every load below is unconditional (past the last slab a wave re-reads a valid one), so
    // the compiler's vmcnt bookkeeping sees one straight-line count and never drains the ring.
    int s = grp * NW + wave;
    {
        const float* ar = row_ptr(min(s, S - 1));
#pragma unroll
        for (int c = 0; c < R - 1; ++c)
#pragma unroll
            for (int j = 0; j < KC; ++j) {
                const float* src = ar + kofs(c * KC + j);
                ra[c][j][0] = *reinterpret_cast<const float4*>(src);
                ra[c][j][1] = *reinterpret_cast<const float4*>(src + 4);
            }
    }
#pragma unroll
    for (int i = 0; i < PER_T; ++i) reinterpret_cast<float4*>(wl)[tid + i * 64 * NW] = wv[i];
    // 3. per-column epilogue constants, read from LDS in the epilogue (no vector-memory wait)
    if (tid < 32 * TN) {
        const int col = n0 + tid;
        const bool ok = col < p.N;
        col_b[tid] = (p.bias && ok) ? p.bias[col] : 0.0f;
        col_q[tid] = (p.qp && ok) ? p.qp[col] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __syncthreads();

    // W fragments of one k-step: [plane][tn]; read one k-step ahead of their MFMAs
    auto read_w = [&](int ks, bf16x8 (&fw)[3][TN]) {
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
                fw[pl][tn] = *reinterpret_cast<const bf16x8*>(wl + ((tn * KS + ks) * 3 + pl) * 1024 + lane * 16);
    };
    bf16x8 fwc[3][TN];
    if constexpr (PIPE) read_w(0, fwc);

    for (; s < S; s += stride) {
        const int sn = s + stride;
        const float* ar = row_ptr(s);
        const float* arn = row_ptr(sn < S ? sn : s);
        const int bz = s / Sb;
        const int m0 = (s - bz * Sb) * 32;
        floatx16 acc[1][TN];
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[0][tn][i] = 0.f;
        float ax[TN][16];

#pragma unroll
        for (int kc = 0; kc < CPS; ++kc) {
            if constexpr (kAux) {
                if (kc == CPS - R + 1) {  // before the first load of the next slab
                    const float* auxb = p.aux + (int64_t)bz * p.stride_aux;
#pragma unroll
                    for (int tn = 0; tn < TN; ++tn) {
                        const int col = min(n0 + tn * 32 + r, p.N - 1);
#pragma unroll
                        for (int i = 0; i < 16; ++i) {
                            const int row = min(m0 + (i & 3) + 8 * (i >> 2) + 4 * h, p.M - 1);
                            ax[tn][i] = auxb[(int64_t)row * p.ld_aux + col];
                        }
                    }
                }
            }
            // prefetch chunk kc + R - 1 of this slab, or the head of the next one
            if constexpr (!(VASR_PANEL_ABLATE & 4)) {
                const int cp = kc + R - 1;
                const float* src_row = cp < CPS ? ar : arn;
                const int cc = cp < CPS ? cp : cp - CPS;
#pragma unroll
                for (int j = 0; j < KC; ++j) {
                    const float* src = src_row + kofs(cc * KC + j);
                    ra[cp % R][j][0] = *reinterpret_cast<const float4*>(src);
                    ra[cp % R][j][1] = *reinterpret_cast<const float4*>(src + 4);
                }
            }
#pragma unroll
            for (int j = 0; j < KC; ++j) {
                const int ks = kc * KC + j;
                bf16x8 fw[3][TN];
                if constexpr (PIPE) {
#pragma unroll
                    for (int pl = 0; pl < 3; ++pl)
#pragma unroll
                        for (int tn = 0; tn < TN; ++tn) fw[pl][tn] = fwc[pl][tn];
                    if constexpr (!(VASR_PANEL_ABLATE & 8))
                        read_w(ks + 1 < KS ? ks + 1 : 0, fwc);  // next k-step (or the next slab's first)
                } else {
                    read_w(ks, fw);
                }
                // pin the split to its k-step: without this the compiler hoists the splits of
                // whole chunks to the loop head, waiting for (draining) the prefetch ring
                float4 x0 = ra[kc % R][j][0], x1 = ra[kc % R][j][1];
                asm volatile("" : "+v"(x0.x), "+v"(x0.y), "+v"(x0.z), "+v"(x0.w));
                asm volatile("" : "+v"(x1.x), "+v"(x1.y), "+v"(x1.z), "+v"(x1.w));
                bf16x8 hi, mid, lo;
                if constexpr (VASR_PANEL_ABLATE & 16) {
                    hi = mid = lo = bf16x8{(__bf16)x0.x, (__bf16)x0.y, (__bf16)x0.z, (__bf16)x0.w,
                                           (__bf16)x1.x, (__bf16)x1.y, (__bf16)x1.z, (__bf16)x1.w};
                } else {
                    split8(x0, x1, hi, mid, lo);
                }
                // the tile kernel's order: small terms first, then hi*hi
#pragma unroll
                for (int tn = 0; tn < TN; ++tn) {
                    if constexpr (VASR_PANEL_ABLATE & 1) {
                        acc[0][tn][0] += (float)hi[0] * (float)fw[0][tn][1] + (float)lo[1] * (float)fw[2][tn][0] +
                                         (float)mid[2] * (float)fw[1][tn][3];
                        continue;
                    }
                    floatx16 c = acc[0][tn];
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(lo, fw[0][tn], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(hi, fw[2][tn], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(mid, fw[1][tn], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(mid, fw[0][tn], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(hi, fw[1][tn], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(hi, fw[0][tn], c, 0, 0, 0);
                    acc[0][tn] = c;
                }
                // keep the scheduler from hoisting later k-steps' LDS reads (register pressure)
                __builtin_amdgcn_sched_barrier(0);
            }
        }

        // 4. epilogue (gemm_common.h's arithmetic, constants preloaded)
        if constexpr (EPI == VASR_EPI_ARGMAX) {
            unsigned long long* __restrict__ keys =
                reinterpret_cast<unsigned long long*>(p.C) + (int64_t)bz * p.stride_c;
            const int s0 = n0 / 32;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                unsigned long long key = 0ull;
#pragma unroll
                for (int tn = 0; tn < TN; ++tn) {
                    const int col = n0 + tn * 32 + r;
                    if (col >= p.N) continue;
                    float v = acc[0][tn][i];
                    if (p.bias) v = v + col_b[tn * 32 + r];
                    if (p.qp) v = fake_quant(v, col_q[tn * 32 + r]);
                    const unsigned u = __float_as_uint(v);
                    const unsigned ord = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
                    const unsigned long long k = ((unsigned long long)ord << 32) | (0xFFFFFFFFu - (unsigned)col);
                    key = k > key ? k : key;
                }
                key = max_u64_over_32_lanes(key);  // lanes r = 16..31 hold it
                const int row = m0 + (i & 3) + 8 * (i >> 2) + 4 * h;
                const int slot = r - (32 - TN);
                if (slot >= 0 && row < p.M && (s0 + slot) * 32 < p.N)
                    keys[(int64_t)row * p.ldc + s0 + slot] = slot == 0 ? key : 0ull;
            }
        } else {
            float* __restrict__ Cb = p.C + (int64_t)bz * p.stride_c;
            const float* __restrict__ abase =
                kAux || !(EPI == VASR_EPI_RESIDUAL || EPI == VASR_EPI_GELU_PE)
                    ? nullptr
                    : p.aux + (int64_t)bz * p.stride_aux + (int64_t)m0 * p.ld_aux;
            const bool has_b = p.bias != nullptr;
            // an opaque 0 in the row strides keeps the 32 per-element offsets from being hoisted
            // out of the slab loop (32 VGPRs held across the main loop)
            int opaque_zero = 0;
            asm volatile("" : "+s"(opaque_zero));
            // QP / GUARD as template arguments: the per-element work is branch-free
            auto store = [&](auto qp_c, auto guard_c) {
                constexpr bool QP = decltype(qp_c)::value, GUARD = decltype(guard_c)::value;
#pragma unroll
                for (int tn = 0; tn < TN; ++tn) {
                    const int col = n0 + tn * 32 + r;
                    if (GUARD && col >= p.N) continue;
                    const float b = col_b[tn * 32 + r];
                    float4 q;
                    if constexpr (QP) q = col_q[tn * 32 + r];
                    const bool sp = col >= p.n_out;
                    float* __restrict__ cbase = Cb + (int64_t)m0 * p.ldc;  // wave-uniform
                    const int ldc = (int)p.ldc + opaque_zero;
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const int rr = (i & 3) + 8 * (i >> 2) + 4 * h;
                        if (GUARD && m0 + rr >= p.M) continue;
                        float v = acc[0][tn][i];
                        v = has_b ? v + b : v;
                        if constexpr (QP) v = fake_quant(v, q);
                        if constexpr (EPI == VASR_EPI_GELU) {
                            v = gelu_fast(v);
                        } else if constexpr (EPI == VASR_EPI_SOFTPLUS_FROM) {
                            v = sp ? softplus20_fast(v) : v;
                        } else if constexpr (EPI == VASR_EPI_RESIDUAL || EPI == VASR_EPI_GELU_PE) {
                            float a;
                            if constexpr (kAux) a = ax[tn][i];
                            else a = abase[(unsigned)(rr * ((int)p.ld_aux + opaque_zero) + col)];
                            v = (EPI == VASR_EPI_GELU_PE ? gelu_fast(v) : v) + a;
                        }
                        const unsigned off = (unsigned)(rr * ldc + col);  // 32-bit lane offset
                        if constexpr (VASR_PANEL_ABLATE & 2) {
                            if (v == 1.2345f) cbase[off] = v;
                        } else {
                            cbase[off] = v;
                        }
                    }
                }
            };
            using T = std::true_type;
            using F = std::false_type;
            const bool full = m0 + 32 <= p.M && n0 + 32 * TN <= p.N;
            if (p.qp) {
                if (full) store(T{}, F{}); else store(T{}, T{});
            } else {
                if (full) store(F{}, F{}); else store(F{}, T{});
            }
        }
    }
}

template <int KS, int NW, int BPC, int R, int KC, bool PIPE>
int launch_panel(const GemmParams& p, int epi, hipStream_t st) {
    const int np = (p.N + 32 * TN - 1) / (32 * TN);
    const long S = (long)((p.M + 31) / 32) * p.batch;
    const long want = (S + NW - 1) / NW;
    const int groups = (int)std::max(1L, std::min(want, (long)(kCUs * BPC / np)));
    const dim3 grid(np * groups), block(64 * NW);
#define VASR_P(E) \
    hipLaunchKernelGGL((gemm_panel_kernel<KS, NW, BPC, R, KC, PIPE, E>), grid, block, 0, st, p, np, groups)
    switch (epi) {
        case VASR_EPI_NONE: VASR_P(VASR_EPI_NONE); break;
        case VASR_EPI_GELU: VASR_P(VASR_EPI_GELU); break;
        case VASR_EPI_SOFTPLUS_FROM: VASR_P(VASR_EPI_SOFTPLUS_FROM); break;
        case VASR_EPI_RESIDUAL: VASR_P(VASR_EPI_RESIDUAL); break;
        case VASR_EPI_GELU_PE: VASR_P(VASR_EPI_GELU_PE); break;
        case VASR_EPI_ARGMAX: VASR_P(VASR_EPI_ARGMAX); break;
        default: set_error("vasr_linear_x3_f32 (panel): epilogue %d", epi); return VASR_EINVAL;
    }
#undef VASR_P
    return launch_status("vasr_linear_x3_f32 (panel)");
}

int g_panel_enabled = -1;  // -1: from VASR_GEMM_PANEL (default 0: measured slower, see header)

}  // namespace

namespace gemm {

bool try_panel_x3(const GemmParams& p, int epi, hipStream_t st, int* rc) {
    if (g_panel_enabled < 0) {
        const char* e = std::getenv("VASR_GEMM_PANEL");
        g_panel_enabled = e ? std::atoi(e) : 0;
    }
    if (!g_panel_enabled || p.K != p.Kp || p.K % 16 != 0) return false;
    if (epi != VASR_EPI_NONE && epi != VASR_EPI_GELU && epi != VASR_EPI_SOFTPLUS_FROM && epi != VASR_EPI_RESIDUAL &&
        epi != VASR_EPI_GELU_PE && epi != VASR_EPI_ARGMAX)
        return false;
    const int ks = p.Kp / 16;
    if (g_panel_enabled == 2) {  // 2 waves per SIMD, deep ring, pipelined W reads
        if (ks == 12) return *rc = launch_panel<12, 4, 2, 3, 4, true>(p, epi, st), true;
        if (ks == 24) return *rc = launch_panel<24, 8, 1, 3, 4, true>(p, epi, st), true;
        return false;
    }
    // 4 waves per SIMD (16 per CU): 72 KiB panels x 2 blocks of 8 waves, or 144 KiB x 1 of 16
    if (ks == 12) return *rc = launch_panel<12, 8, 2, 2, 2, false>(p, epi, st), true;
    if (ks == 24) return *rc = launch_panel<24, 16, 1, 2, 2, false>(p, epi, st), true;
    return false;
}

}  // namespace gemm
}  // namespace vasr

VASR_API int vasr_set_x3_engine(int engine) {
    using namespace vasr;
    if (g_panel_enabled < 0) {
        const char* e = std::getenv("VASR_GEMM_PANEL");
        g_panel_enabled = e ? std::atoi(e) : 0;
    }
    const int prev = g_panel_enabled;
    if (engine >= 0 && engine <= 2) g_panel_enabled = engine;
    return prev;
}
