// fp32 GEMM with fused epilogues on the gfx950 f32-input MFMA (v_mfma_f32_32x32x2_f32).
//
// C[b] = epi(A[b] (M x K, row stride lda) * W^T + bias), W row-major [N][K] (nn.Linear).
//
// Tiling: 256 threads = 4 waves laid out WM x WN; each wave owns a (32*TM) x 64 tile,
// i.e. TM x 2 MFMA 32x32 accumulators (16 f32 each).  The block tile BM x BN =
// (WM*32*TM) x (WN*64) walks K in BK = 32 steps through one LDS buffer with register
// prefetch of the next step.  Each lane (r = lane&31, h = lane>>5) supplies k-slot h of
// every MFMA; over the 16 k-steps of a BK tile lane half h covers k = h*16 .. h*16+15,
// so A and W fragments are read as contiguous float4s (ds_read_b128).  Rows are padded
// to 36 floats: every ds_read_b128 lane group then hits 16 distinct 4-bank slots.
// Tile decode, epilogues and the tile cost model: gemm_common.h.
#include "gemm_common.h"

namespace vasr {
namespace {

using namespace gemm;

constexpr int BK = 32;
constexpr int SK = BK + 4;  // padded LDS row (floats)

template <int WM, int WN, int TM, int TN, int EPI>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmParams p) {
    constexpr int BM = WM * 32 * TM;
    constexpr int BN = WN * 32 * TN;
    static_assert(TN % 2 == 0 || (EPI != VASR_EPI_PAIR_POWER && EPI != VASR_EPI_PAIR_FUSION), "pairs need even TN");
    constexpr int A_LOADS = BM * (BK / 4) / 256;  // float4 per thread
    constexpr int W_LOADS = BN * (BK / 4) / 256;
    static_assert(A_LOADS >= 1 && W_LOADS >= 1, "tile too small");

    __shared__ __attribute__((aligned(16))) float smem[(BM + BN) * SK];
    float* As = smem;
    float* Ws = smem + BM * SK;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wr = wave / WN;
    const int wc = wave % WN;
    const int r = lane & 31;
    const int h = lane >> 5;

    const Tile t = decode_tile<BM, BN>(p);
    const int m0 = t.m0, n0 = t.n0;
    const float* __restrict__ A = p.A + (int64_t)t.bz * p.stride_a;
    const float* __restrict__ W = p.W;

    float4 ra[A_LOADS], rw[W_LOADS];

    auto load_tile = [&](int k0) {
#pragma unroll
        for (int i = 0; i < A_LOADS; ++i) {
            const int q = tid + 256 * i;
            const int row = q >> 3, c = (q & 7) * 4;
            const int gm = m0 + row, gk = k0 + c;
            ra[i] = (gm < p.M && gk < p.K) ? *reinterpret_cast<const float4*>(A + (int64_t)gm * p.lda + gk)
                                           : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int i = 0; i < W_LOADS; ++i) {
            const int q = tid + 256 * i;
            const int row = q >> 3, c = (q & 7) * 4;
            const int gn = n0 + row, gk = k0 + c;
            rw[i] = (gn < p.N && gk < p.K) ? *reinterpret_cast<const float4*>(W + (int64_t)gn * p.ldw + gk)
                                           : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto store_tile = [&]() {
#pragma unroll
        for (int i = 0; i < A_LOADS; ++i) {
            const int q = tid + 256 * i;
            *reinterpret_cast<float4*>(As + (q >> 3) * SK + (q & 7) * 4) = ra[i];
        }
#pragma unroll
        for (int i = 0; i < W_LOADS; ++i) {
            const int q = tid + 256 * i;
            *reinterpret_cast<float4*>(Ws + (q >> 3) * SK + (q & 7) * 4) = rw[i];
        }
    };

    floatx16 acc[TM][TN];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[tm][tn][i] = 0.f;

    const int nk = (p.K + BK - 1) / BK;
    load_tile(0);
    store_tile();
    __syncthreads();

    const float* a_base = As + (wr * 32 * TM + r) * SK + h * 16;
    const float* w_base = Ws + (wc * 32 * TN + r) * SK + h * 16;

    for (int kt = 0; kt < nk; ++kt) {
        if (kt + 1 < nk) load_tile((kt + 1) * BK);
#pragma unroll
        for (int kh = 0; kh < 2; ++kh) {
            float4 fa[TM][2], fw[TN][2];
#pragma unroll
            for (int tm = 0; tm < TM; ++tm) {
                fa[tm][0] = *reinterpret_cast<const float4*>(a_base + tm * 32 * SK + kh * 8);
                fa[tm][1] = *reinterpret_cast<const float4*>(a_base + tm * 32 * SK + kh * 8 + 4);
            }
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                fw[tn][0] = *reinterpret_cast<const float4*>(w_base + tn * 32 * SK + kh * 8);
                fw[tn][1] = *reinterpret_cast<const float4*>(w_base + tn * 32 * SK + kh * 8 + 4);
            }
#pragma unroll
            for (int s = 0; s < 8; ++s) {
#pragma unroll
                for (int tm = 0; tm < TM; ++tm) {
                    const float av = reinterpret_cast<const float*>(&fa[tm][s >> 2])[s & 3];
#pragma unroll
                    for (int tn = 0; tn < TN; ++tn) {
                        const float bv = reinterpret_cast<const float*>(&fw[tn][s >> 2])[s & 3];
                        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[tm][tn], 0, 0, 0);
                    }
                }
            }
        }
        __syncthreads();
        if (kt + 1 < nk) {
            store_tile();
            __syncthreads();
        }
    }

    epilogue<BM, BN, TM, TN, EPI>(p, t, acc, wr, wc, r, h);
}

template <int WM, int WN, int TM, int TN>
int launch_cfg(const GemmParams& p, int batch, int epi, hipStream_t s) {
    constexpr int BM = WM * 32 * TM;
    constexpr int BN = WN * 32 * TN;
    const int tiles = ((p.N + BN - 1) / BN) * ((p.M + BM - 1) / BM);
    dim3 grid(tiles, batch);
    dim3 block(256);
#define VASR_L(E) hipLaunchKernelGGL((gemm_f32_kernel<WM, WN, TM, TN, E>), grid, block, 0, s, p)
    switch (epi) {
        case VASR_EPI_NONE: VASR_L(VASR_EPI_NONE); break;
        case VASR_EPI_GELU: VASR_L(VASR_EPI_GELU); break;
        case VASR_EPI_SOFTPLUS_FROM: VASR_L(VASR_EPI_SOFTPLUS_FROM); break;
        case VASR_EPI_RESIDUAL: VASR_L(VASR_EPI_RESIDUAL); break;
        case VASR_EPI_GELU_PE: VASR_L(VASR_EPI_GELU_PE); break;
        case VASR_EPI_PAIR_POWER:
            if constexpr (TN % 2 == 0) { VASR_L(VASR_EPI_PAIR_POWER); break; }
            set_error("vasr_linear_f32: paired epilogue needs a TN=2 tile"); return VASR_EINVAL;
        case VASR_EPI_ARGMAX: VASR_L(VASR_EPI_ARGMAX); break;
        case VASR_EPI_PAIR_FUSION:
            if constexpr (TN % 2 == 0) { VASR_L(VASR_EPI_PAIR_FUSION); break; }
            set_error("vasr_linear_f32: paired epilogue needs a TN=2 tile"); return VASR_EINVAL;
        default: set_error("vasr_linear_f32: unknown epilogue %d", epi); return VASR_EINVAL;
    }
#undef VASR_L
    return launch_status("vasr_linear_f32");
}

constexpr TileCfg kCfgs[] = {
    {2, 2, 2, 2, 3},  // 128 x 128
    {2, 2, 1, 2, 4},  //  64 x 128
    {4, 1, 1, 2, 4},  // 128 x  64
    {2, 2, 1, 1, 7},  //  64 x  64
};

}  // namespace
}  // namespace vasr

VASR_API int vasr_linear_f32(const vasr_gemm_args* a, void* stream) {
    using namespace vasr;
    GemmParams p;
    if (int rc = check_args(a, "vasr_linear_f32", p)) return rc;
    VASR_CHECK_ARG(a->ln_w == nullptr, "vasr_linear_f32: the row-LayerNorm prologue is an x3 / bf16 engine feature");
    VASR_CHECK_ARG(a->W != nullptr, "vasr_linear_f32: null W");
    VASR_CHECK_ARG(a->ldw % 4 == 0 && (reinterpret_cast<uintptr_t>(a->W) & 15) == 0,
                   "vasr_linear_f32: W must be 16-byte aligned with ldw %% 4 == 0");
    if (a->M == 0) return VASR_OK;
    const int epi = a->epilogue;
    const bool pair = epi == VASR_EPI_PAIR_POWER || epi == VASR_EPI_PAIR_FUSION;
    hipStream_t s = as_stream(stream);
    switch (pick_cfg(kCfgs, 4, a->M, a->N, a->batch, pair)) {
        case 0: return launch_cfg<2, 2, 2, 2>(p, a->batch, epi, s);
        case 1: return launch_cfg<2, 2, 1, 2>(p, a->batch, epi, s);
        case 2: return launch_cfg<4, 1, 1, 2>(p, a->batch, epi, s);
        default: return launch_cfg<2, 2, 1, 1>(p, a->batch, epi, s);
    }
}
