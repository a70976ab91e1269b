// fp32 GEMM on the bf16 matrix cores by exact operand splitting ("bf16x3").
//
// Every fp32 operand x is written as x = hi + mid + lo with hi = bf16(x),
// mid = bf16(x - hi), lo = bf16(x - hi - mid) (round-to-nearest-even; each residual is exact
// in fp32).  hi carries 8 significant bits and each residual at least 8 more, so the three
// terms hold all 24 bits of x.  The product a*b is accumulated as the six terms
//   hi*hi + hi*mid + mid*hi + mid*mid + hi*lo + lo*hi
// on v_mfma_f32_32x32x16_bf16 (bf16 products are exact in fp32, accumulation in fp32);
// the three dropped terms are below 2^-25 |a||b| together, under the 2^-24 rounding of an
// fp32 product, so the result is an fp32 GEMM to within accumulation order.  Six bf16
// MFMAs (32 cycles each per 32x32x16) replace eight f32 MFMAs (64 cycles per 32x32x2) per
// 16 k-steps: 2.67x the f32-input MFMA rate (MI355X_MICROARCH.md, cycle constants).
//
// Weights are split once (vasr_split_weights_bf16x3) into planes [3][N][Kp] bf16.  The
// activation tile is split on its way into LDS.  LDS holds, per k-tile of 32, three planes
// for A (BM rows) and three for W (BN rows), 64 B per row, 16-B chunk c of row r stored at
// chunk c ^ ((r >> 2) & 3): every ds_read_b128 lane group of the operand reads (lanes
// r = 0..31 of one row block, one chunk) then hits 16 distinct 16-B slots of the 256-B bank
// row (conflict-free; MI355X_MICROARCH.md §LDS lane groups).
//
// Operand maps (cdna_hip_programming.md §3): lane (r = lane & 31, h = lane >> 5) supplies
// A[row r][k = 8h + j] and B[k = 8h + j][col r], j = 0..7, i.e. chunk 2s + h of k-step s.
// The accumulator layout equals the f32-input MFMA's, so gemm_common.h's epilogues apply.
#include "gemm_common.h"

namespace vasr {
namespace {

using namespace gemm;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

#ifndef VASR_X3_ABLATE
#define VASR_X3_ABLATE 0  // diagnostic builds only: 1 no MFMA, 2 no C stores, 4 no A split,
#endif                    // 8 no global loads after the first k-tile

constexpr int BK = 32;      // fp32 k per LDS tile (two MFMA k-steps)
constexpr int ROWB = 64;    // bytes per LDS row per plane (32 bf16)

__device__ __forceinline__ int swz(int row, int chunk) { return row * ROWB + 16 * (chunk ^ ((row >> 2) & 3)); }

__device__ __forceinline__ void split4(const float4& x, bf16x4& hi, bf16x4& mid, bf16x4& lo) {
    const float v[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const __bf16 a = (__bf16)v[j];
        const float r1 = v[j] - (float)a;
        const __bf16 b = (__bf16)r1;
        const float r2 = r1 - (float)b;
        hi[j] = a;
        mid[j] = b;
        lo[j] = (__bf16)r2;
    }
}

template <int WM, int WN, int TM, int TN, int EPI>
__global__ __launch_bounds__(256) void gemm_x3_kernel(GemmParams p) {
    constexpr int BM = WM * 32 * TM;
    constexpr int BN = WN * 32 * TN;
    static_assert(TN == 2 || (EPI != VASR_EPI_PAIR_POWER && EPI != VASR_EPI_PAIR_FUSION), "pairs need TN=2");
    constexpr int A_LOADS = BM * (BK / 4) / 256;      // float4 of A per thread per tile
    constexpr int W_LOADS = 3 * BN * (BK / 8) / 256;  // 16-B bf16 chunks of W per thread per tile
    static_assert(A_LOADS >= 1 && W_LOADS >= 1 && (3 * BN * 4) % 256 == 0, "tile too small");
    constexpr int A_PLANE = BM * ROWB, W_PLANE = BN * ROWB;

    __shared__ __attribute__((aligned(16))) char smem[3 * (A_PLANE + W_PLANE)];
    char* As = smem;
    char* Ws = smem + 3 * A_PLANE;

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
    const uint16_t* __restrict__ Wx = p.Wx;
    const int64_t plane_stride = (int64_t)p.N * p.Kp;

    float4 ra[A_LOADS];
    uint4 rw[W_LOADS];

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
            const int q = tid + 256 * i;  // (plane, row, chunk)
            const int pl = q / (BN * 4), rem = q % (BN * 4);
            const int row = rem >> 2, c = rem & 3;
            const int gn = n0 + row;
            rw[i] = gn < p.N ? *reinterpret_cast<const uint4*>(Wx + pl * plane_stride + (int64_t)gn * p.Kp + k0 + c * 8)
                             : make_uint4(0, 0, 0, 0);
        }
    };
    auto store_tile = [&]() {
#pragma unroll
        for (int i = 0; i < A_LOADS; ++i) {
            const int q = tid + 256 * i;
            const int row = q >> 3, c4 = q & 7;  // float4 c4 = half (c4 & 1) of chunk c4 >> 1
            const int off = swz(row, c4 >> 1) + 8 * (c4 & 1);
            bf16x4 hi, mid, lo;
            if constexpr (VASR_X3_ABLATE & 4) {
                hi = bf16x4{(__bf16)ra[i].x, (__bf16)ra[i].y, (__bf16)ra[i].z, (__bf16)ra[i].w};
                mid = hi;
                lo = hi;
            } else {
                split4(ra[i], hi, mid, lo);
            }
            *reinterpret_cast<bf16x4*>(As + off) = hi;
            *reinterpret_cast<bf16x4*>(As + A_PLANE + off) = mid;
            *reinterpret_cast<bf16x4*>(As + 2 * A_PLANE + off) = lo;
        }
#pragma unroll
        for (int i = 0; i < W_LOADS; ++i) {
            const int q = tid + 256 * i;
            const int pl = q / (BN * 4), rem = q % (BN * 4);
            *reinterpret_cast<uint4*>(Ws + pl * W_PLANE + swz(rem >> 2, rem & 3)) = rw[i];
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

    const int a_row = wr * 32 * TM + r;
    const int w_row = wc * 32 * TN + r;

    for (int kt = 0; kt < nk; ++kt) {
        if (kt + 1 < nk && !((VASR_X3_ABLATE & 8) && kt > 0)) load_tile((kt + 1) * BK);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int chunk = 2 * s + h;
            bf16x8 fa[3][TM], fw[3][TN];
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
                for (int tm = 0; tm < TM; ++tm)
                    fa[pl][tm] = *reinterpret_cast<const bf16x8*>(As + pl * A_PLANE + swz(a_row + tm * 32, chunk));
#pragma unroll
                for (int tn = 0; tn < TN; ++tn)
                    fw[pl][tn] = *reinterpret_cast<const bf16x8*>(Ws + pl * W_PLANE + swz(w_row + tn * 32, chunk));
            }
            // small terms first, then the leading hi*hi term
            if constexpr (VASR_X3_ABLATE & 1) {
#pragma unroll
                for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                    for (int tn = 0; tn < TN; ++tn) acc[tm][tn][0] += (float)fa[0][tm][0] * (float)fw[2][tn][1];
                continue;
            }
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int tn = 0; tn < TN; ++tn) {
                    floatx16 c = acc[tm][tn];
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2][tm], fw[0][tn], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][tm], fw[2][tn], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1][tm], fw[1][tn], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1][tm], fw[0][tn], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][tm], fw[1][tn], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][tm], fw[0][tn], c, 0, 0, 0);
                    acc[tm][tn] = c;
                }
        }
        __syncthreads();
        if (kt + 1 < nk) {
            store_tile();
            __syncthreads();
        }
    }

    if constexpr (VASR_X3_ABLATE & 2) {  // keep every accumulator live, store nothing
        float sum = 0.f;
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
#pragma unroll
            for (int tn = 0; tn < TN; ++tn)
#pragma unroll
                for (int i = 0; i < 16; ++i) sum += acc[tm][tn][i];
        if (sum != 1.2345f) return;
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
#define VASR_L(E) hipLaunchKernelGGL((gemm_x3_kernel<WM, WN, TM, TN, E>), grid, block, 0, s, p)
    switch (epi) {
        case VASR_EPI_NONE: VASR_L(VASR_EPI_NONE); break;
        case VASR_EPI_GELU: VASR_L(VASR_EPI_GELU); break;
        case VASR_EPI_SOFTPLUS_FROM: VASR_L(VASR_EPI_SOFTPLUS_FROM); break;
        case VASR_EPI_RESIDUAL: VASR_L(VASR_EPI_RESIDUAL); break;
        case VASR_EPI_GELU_PE: VASR_L(VASR_EPI_GELU_PE); break;
        case VASR_EPI_PAIR_POWER:
            if constexpr (TN == 2) { VASR_L(VASR_EPI_PAIR_POWER); break; }
            set_error("vasr_linear_x3_f32: paired epilogue needs a TN=2 tile"); return VASR_EINVAL;
        case VASR_EPI_PAIR_FUSION:
            if constexpr (TN == 2) { VASR_L(VASR_EPI_PAIR_FUSION); break; }
            set_error("vasr_linear_x3_f32: paired epilogue needs a TN=2 tile"); return VASR_EINVAL;
        default: set_error("vasr_linear_x3_f32: unknown epilogue %d", epi); return VASR_EINVAL;
    }
#undef VASR_L
    return launch_status("vasr_linear_x3_f32");
}

// occ: min(waves per SIMD from VGPR+AGPR use, 160 KiB / LDS per block)
constexpr TileCfg kCfgs[] = {
    {2, 2, 2, 2, 2},  // 128 x 128: 200 regs, 48 KiB
    {2, 2, 1, 2, 3},  //  64 x 128: 132 regs, 36 KiB
    {4, 1, 1, 2, 3},  // 128 x  64
    {2, 2, 1, 1, 5},  //  64 x  64:  82 regs, 24 KiB
};

// [3][N][Kp] planes; thread per 8 consecutive k of one row.
__global__ void split_weights_kernel(const float* __restrict__ W, int64_t ldw, int N, int K, int Kp,
                                     uint16_t* __restrict__ out) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int cpr = Kp / 8;
    if (q >= (int64_t)N * cpr) return;
    const int n = (int)(q / cpr), k0 = (int)(q % cpr) * 8;
    bf16x8 hi, mid, lo;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float x = k0 + j < K ? W[(int64_t)n * ldw + k0 + j] : 0.0f;
        const __bf16 a = (__bf16)x;
        const float r1 = x - (float)a;
        const __bf16 b = (__bf16)r1;
        hi[j] = a;
        mid[j] = b;
        lo[j] = (__bf16)(r1 - (float)b);
    }
    const int64_t plane = (int64_t)N * Kp, base = (int64_t)n * Kp + k0;
    *reinterpret_cast<bf16x8*>(out + base) = hi;
    *reinterpret_cast<bf16x8*>(out + plane + base) = mid;
    *reinterpret_cast<bf16x8*>(out + 2 * plane + base) = lo;
}

}  // namespace
}  // namespace vasr

VASR_API int64_t vasr_split_weights_elems(int N, int K) {
    if (N <= 0 || K <= 0) return 0;
    return 3 * (int64_t)N * ((K + 31) / 32 * 32);
}

VASR_API int vasr_split_weights_bf16x3(const float* W, int64_t ldw, int N, int K, uint16_t* out, void* stream) {
    using namespace vasr;
    VASR_CHECK_ARG(W && out, "vasr_split_weights_bf16x3: null pointer");
    VASR_CHECK_ARG(N > 0 && K > 0 && ldw >= K, "vasr_split_weights_bf16x3: bad shape N=%d K=%d ldw=%lld", N, K,
                   (long long)ldw);
    VASR_CHECK_ARG((reinterpret_cast<uintptr_t>(out) & 15) == 0, "vasr_split_weights_bf16x3: out must be 16-byte aligned");
    const int Kp = (K + 31) / 32 * 32;
    const int64_t n = (int64_t)N * (Kp / 8);
    hipLaunchKernelGGL(split_weights_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), W, ldw,
                       N, K, Kp, out);
    return launch_status("vasr_split_weights_bf16x3");
}

VASR_API int vasr_linear_x3_f32(const vasr_gemm_args* a, const uint16_t* w_split, void* stream) {
    using namespace vasr;
    GemmParams p;
    if (int rc = check_args(a, "vasr_linear_x3_f32", p)) return rc;
    VASR_CHECK_ARG(w_split != nullptr && (reinterpret_cast<uintptr_t>(w_split) & 15) == 0,
                   "vasr_linear_x3_f32: w_split must be a 16-byte aligned device pointer");
    if (a->M == 0) return VASR_OK;
    p.Wx = w_split;
    p.Kp = (a->K + 31) / 32 * 32;
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
