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
//
// The "pair" epilogues rely on the two 32-column MFMA tiles of a wave (tn = 0, 1)
// holding two views of the same 32 output columns in the same lane and register:
// PAIR_POWER puts DFT cos|sin rows side by side (|X|^2 in-register); PAIR_FUSION puts
// the gate and global_proj rows side by side (gated fusion in-register).
#include "vasr_internal.h"

namespace vasr {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

#ifndef VASR_GEMM_XCD
#define VASR_GEMM_XCD 1   // XCD-aware tile order (diagnostic builds may turn it off)
#endif

constexpr int BK = 32;
constexpr int SK = BK + 4;  // padded LDS row (floats)

struct GemmParams {
    const float* A;
    int64_t lda, stride_a;
    const float* W;
    int64_t ldw;
    const float* bias;
    float* C;
    int64_t ldc, stride_c;
    int M, N, K;
    const float* aux;
    int64_t ld_aux, stride_aux;
    const float* aux2;
    int n_out;
};

template <int WM, int WN, int TM, int TN, int EPI>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmParams p) {
    constexpr int BM = WM * 32 * TM;
    constexpr int BN = WN * 32 * TN;
    static_assert(TN == 2 || (EPI != VASR_EPI_PAIR_POWER && EPI != VASR_EPI_PAIR_FUSION), "pairs need TN=2");
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

    // Tile decode.  The grid is 1-D; blocks id, id + 8, id + 16, ... are dealt to the same XCD
    // (round-robin dispatch), so each such group gets a contiguous, M-major run of tiles: all
    // N tiles of an A row panel then run on one XCD and share its L2.
    const int tiles_n = (p.N + BN - 1) / BN;
    const int tiles_m = (p.M + BM - 1) / BM;
    const int tiles = tiles_n * tiles_m * (int)gridDim.y;
    int w = blockIdx.x + (int)blockIdx.y * (int)gridDim.x;
    if (VASR_GEMM_XCD) {
        const int q8 = tiles / 8, r8 = tiles % 8, xg = w % 8;
        w = (xg < r8 ? xg * (q8 + 1) : r8 * (q8 + 1) + (xg - r8) * q8) + w / 8;
    }
    const int per_batch = tiles_n * tiles_m;
    const int bz = w / per_batch;
    const int wr_ = w - bz * per_batch;
    const int m0 = (wr_ / tiles_n) * BM;
    const int n0 = (wr_ % tiles_n) * BN;
    const float* __restrict__ A = p.A + (int64_t)bz * p.stride_a;
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

    // ---------------------------------------------------------------- epilogue
    float* __restrict__ Cb = p.C + (int64_t)bz * p.stride_c;
    const float* __restrict__ auxb = p.aux ? p.aux + (int64_t)bz * p.stride_aux : nullptr;

    if constexpr (EPI == VASR_EPI_PAIR_POWER || EPI == VASR_EPI_PAIR_FUSION) {
        const int col = (n0 + wc * 32 * TN) / 2 + r;  // output column of this lane
        if (col >= p.n_out) return;
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int row = m0 + wr * 32 * TM + tm * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
                if (row >= p.M) continue;
                const float v0 = acc[tm][0][i];
                const float v1 = acc[tm][TN - 1][i];
                float out;
                if constexpr (EPI == VASR_EPI_PAIR_POWER) {
                    out = v0 * v0 + v1 * v1;
                } else {
                    // aux: local-side partial products in the same paired layout.
                    const int pc = n0 + wc * 32 * TN + r;  // paired column of half 0
                    const float* ar = auxb + (int64_t)row * p.ld_aux;
                    const float gate = sigmoidf_((ar[pc] + v0) + p.bias[pc]);
                    const float lt = ar[pc + 32] + p.aux2[col];
                    const float gt = v1 + p.bias[pc + 32];
                    out = gate * lt + (1.0f - gate) * gt;
                }
                Cb[(int64_t)row * p.ldc + col] = out;
            }
        }
    } else {
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int col = n0 + wc * 32 * TN + tn * 32 + r;
                if (col >= p.N) continue;
                const float bv = p.bias ? p.bias[col] : 0.0f;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int row = m0 + wr * 32 * TM + tm * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
                    if (row >= p.M) continue;
                    float v = acc[tm][tn][i];
                    if (p.bias) v = v + bv;
                    if constexpr (EPI == VASR_EPI_GELU) {
                        v = gelu_erf(v);
                    } else if constexpr (EPI == VASR_EPI_SOFTPLUS_FROM) {
                        if (col >= p.n_out) v = softplus20(v);
                    } else if constexpr (EPI == VASR_EPI_RESIDUAL) {
                        v = v + auxb[(int64_t)row * p.ld_aux + col];
                    } else if constexpr (EPI == VASR_EPI_GELU_PE) {
                        v = gelu_erf(v) + auxb[(int64_t)row * p.ld_aux + col];
                    }
                    Cb[(int64_t)row * p.ldc + col] = v;
                }
            }
        }
    }
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
            if constexpr (TN == 2) { VASR_L(VASR_EPI_PAIR_POWER); break; }
            set_error("vasr_linear_f32: paired epilogue needs a TN=2 tile"); return VASR_EINVAL;
        case VASR_EPI_PAIR_FUSION:
            if constexpr (TN == 2) { VASR_L(VASR_EPI_PAIR_FUSION); break; }
            set_error("vasr_linear_f32: paired epilogue needs a TN=2 tile"); return VASR_EINVAL;
        default: set_error("vasr_linear_f32: unknown epilogue %d", epi); return VASR_EINVAL;
    }
#undef VASR_L
    return launch_status("vasr_linear_f32");
}

// Tile configurations: {WM, WN, TM, TN, blocks per CU the kernel's VGPR/LDS use admits}.
struct TileCfg {
    int wm, wn, tm, tn, occ;
    int bm() const { return wm * 32 * tm; }
    int bn() const { return wn * 32 * tn; }
};
constexpr TileCfg kCfgs[] = {
    {2, 2, 2, 2, 3},  // 128 x 128
    {2, 2, 1, 2, 4},  //  64 x 128
    {4, 1, 1, 2, 4},  // 128 x  64
    {2, 2, 1, 1, 7},  //  64 x  64
};
constexpr int kCUs = 256;

// Pick the tile that minimises (rounds of resident blocks) x (blocks sharing a CU) x tile area:
// at M = 16032 the grids are only one or two rounds deep, so wave quantisation and CU
// balance, not per-tile efficiency, decide the time (measured in tools/gemm_variants_run.py).
int pick_cfg(int M, int N, int batch, bool pair) {
    int best = -1;
    double best_cost = 0;
    for (int i = 0; i < 4; ++i) {
        const TileCfg& c = kCfgs[i];
        if (pair && c.tn != 2) continue;
        const long tiles = (long)((M + c.bm() - 1) / c.bm()) * ((N + c.bn() - 1) / c.bn()) * batch;
        const long per_cu = (tiles + kCUs - 1) / kCUs;
        const long rounds = (per_cu + c.occ - 1) / c.occ;
        const double cost = (double)rounds * (double)(per_cu < c.occ ? per_cu : c.occ) * c.bm() * c.bn();
        if (best < 0 || cost < best_cost * 0.999) {
            best = i;
            best_cost = cost;
        }
    }
    return best;
}

}  // namespace
}  // namespace vasr

VASR_API int vasr_linear_f32(const vasr_gemm_args* a, void* stream) {
    using namespace vasr;
    VASR_CHECK_ARG(a != nullptr, "vasr_linear_f32: null args");
    VASR_CHECK_ARG(a->A && a->W && a->C, "vasr_linear_f32: null A/W/C");
    VASR_CHECK_ARG(a->M >= 0 && a->N > 0 && a->K > 0 && a->batch >= 1, "vasr_linear_f32: bad shape M=%d N=%d K=%d batch=%d",
                   a->M, a->N, a->K, a->batch);
    VASR_CHECK_ARG(a->K % 4 == 0 && a->lda % 4 == 0 && a->ldw % 4 == 0 && a->stride_a % 4 == 0,
                   "vasr_linear_f32: K, lda, ldw, stride_a must be multiples of 4 (K=%d lda=%lld)", a->K,
                   (long long)a->lda);
    VASR_CHECK_ARG((reinterpret_cast<uintptr_t>(a->A) & 15) == 0 && (reinterpret_cast<uintptr_t>(a->W) & 15) == 0,
                   "vasr_linear_f32: A and W must be 16-byte aligned");
    const int epi = a->epilogue;
    const bool pair = epi == VASR_EPI_PAIR_POWER || epi == VASR_EPI_PAIR_FUSION;
    if (pair) {
        VASR_CHECK_ARG(a->N % 64 == 0 && a->n_out > 0 && a->n_out <= a->N / 2,
                       "vasr_linear_f32: paired epilogue needs N %% 64 == 0 and 0 < n_out <= N/2");
    }
    if (epi == VASR_EPI_RESIDUAL || epi == VASR_EPI_GELU_PE || epi == VASR_EPI_PAIR_FUSION)
        VASR_CHECK_ARG(a->aux != nullptr, "vasr_linear_f32: epilogue %d needs aux", epi);
    if (epi == VASR_EPI_PAIR_FUSION)
        VASR_CHECK_ARG(a->aux2 != nullptr && a->bias != nullptr, "vasr_linear_f32: fusion needs bias and aux2");
    if (a->M == 0) return VASR_OK;

    GemmParams p;
    p.A = a->A; p.lda = a->lda; p.stride_a = a->stride_a;
    p.W = a->W; p.ldw = a->ldw; p.bias = a->bias;
    p.C = a->C; p.ldc = a->ldc; p.stride_c = a->stride_c;
    p.M = a->M; p.N = a->N; p.K = a->K;
    p.aux = a->aux; p.ld_aux = a->ld_aux; p.stride_aux = a->stride_aux;
    p.aux2 = a->aux2; p.n_out = a->n_out;
    hipStream_t s = as_stream(stream);

    switch (pick_cfg(a->M, a->N, a->batch, pair)) {
        case 0: return launch_cfg<2, 2, 2, 2>(p, a->batch, epi, s);
        case 1: return launch_cfg<2, 2, 1, 2>(p, a->batch, epi, s);
        case 2: return launch_cfg<4, 1, 1, 2>(p, a->batch, epi, s);
        default: return launch_cfg<2, 2, 1, 1>(p, a->batch, epi, s);
    }
}
