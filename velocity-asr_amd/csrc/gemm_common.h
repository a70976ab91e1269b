// Pieces of the GEMM (gemm_x3.hip: split-bf16 and bf16 MFMA main loops): parameters, the
// XCD-aware tile decode, the fused epilogues and argument checks.  The 32x32 accumulator
// map of v_mfma_f32_32x32x16_bf16 is the one the epilogues index.
#pragma once

#include "vasr_internal.h"

namespace vasr {
namespace gemm {

typedef float floatx16 __attribute__((ext_vector_type(16)));

#ifndef VASR_GEMM_XCD
#define VASR_GEMM_XCD 1   // XCD-aware tile order (diagnostic builds may turn it off)
#endif

struct GemmParams {
    const float* A;
    int64_t lda, stride_a;
    const float* W;
    int64_t ldw;
    const uint16_t* Wx;  // split-bf16 planes [3][N][Kp] (gemm_x3 only)
    int Kp;
    const float* bias;
    float* C;
    int64_t ldc, stride_c;
    int M, N, K;
    const float* aux;
    int64_t ld_aux, stride_aux;
    const float* aux2;
    int n_out;
    const float4* qp;  // per-column activation fake-quant {scale, zp, qmin, qmax} or null
    int batch;
};

struct Tile {
    int bz, m0, n0;
};

// The grid is 1-D; blocks id, id + 8, id + 16, ... are dealt to the same XCD (round-robin
// dispatch), so each such group gets a contiguous, M-major run of tiles: all N tiles of an
// A row panel then run on one XCD and share its L2.
template <int BM, int BN>
__device__ __forceinline__ Tile decode_tile(const GemmParams& p) {
    const int tiles_n = (p.N + BN - 1) / BN;
    const int tiles_m = (p.M + BM - 1) / BM;
    const int tiles = tiles_n * tiles_m * (int)gridDim.y;
    int w = blockIdx.x + (int)blockIdx.y * (int)gridDim.x;
    if (VASR_GEMM_XCD) {
        const int q8 = tiles / 8, r8 = tiles % 8, xg = w % 8;
        w = (xg < r8 ? xg * (q8 + 1) : r8 * (q8 + 1) + (xg - r8) * q8) + w / 8;
    }
    const int per_batch = tiles_n * tiles_m;
    Tile t;
    t.bz = w / per_batch;
    const int wr_ = w - t.bz * per_batch;
    t.m0 = (wr_ / tiles_n) * BM;
    t.n0 = (wr_ % tiles_n) * BN;
    return t;
}

// Max of a 64-bit key over the 32 lanes r = 0..31 of each wave half, all in DPP (no LDS
// round trips): xor 1, xor 2 (quad_perm), the half-row and row mirrors complete each 16-lane
// row; row_bcast15 then hands row 0's (2's) result to row 1 (3), whose lanes (r = 16..31)
// all end with the max of the 32.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ unsigned long long dpp_u64(unsigned long long v) {
    const int lo = __builtin_amdgcn_update_dpp((int)(unsigned)v, (int)(unsigned)v, CTRL, ROWMASK, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(unsigned)(v >> 32), (int)(unsigned)(v >> 32), CTRL, ROWMASK, 0xF,
                                               false);
    return ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo;
}

__device__ __forceinline__ unsigned long long max_u64_over_32_lanes(unsigned long long k) {
    unsigned long long o;
    o = dpp_u64<0xB1, 0xF>(k);  // quad_perm [1,0,3,2]
    k = o > k ? o : k;
    o = dpp_u64<0x4E, 0xF>(k);  // quad_perm [2,3,0,1]
    k = o > k ? o : k;
    o = dpp_u64<0x141, 0xF>(k);  // row_half_mirror
    k = o > k ? o : k;
    o = dpp_u64<0x140, 0xF>(k);  // row_mirror
    k = o > k ? o : k;
    o = dpp_u64<0x142, 0xA>(k);  // row_bcast15 into rows 1 and 3 (rows 0, 2 keep their own value)
    return o > k ? o : k;
}

// Accumulator element i of MFMA tile (tm, tn) of wave (wr, wc), lane (r, h) is
// C[m0 + wr*32*TM + tm*32 + (i&3) + 8*(i>>2) + 4*h][n0 + wc*32*TN + tn*32 + r].
//
// The "pair" epilogues rely on each pair of 32-column MFMA tiles of a wave (tn = 2tp, 2tp+1)
// holding two views of the same 32 output columns in the same lane and register: PAIR_POWER
// puts DFT cos|sin rows side by side (|X|^2 in-register); PAIR_FUSION puts the gate and
// global_proj rows side by side (gated fusion in-register).
//
// GUARD = false for tiles wholly inside M x N: no per-element bounds branches.
template <int TM, int TN, int EPI, bool GUARD>
__device__ __forceinline__ void epilogue_body(const GemmParams& p, const Tile& t, floatx16 (&acc)[TM][TN], int wr,
                                              int wc, int r, int h, unsigned long long* scr) {
    float* __restrict__ Cb = p.C + (int64_t)t.bz * p.stride_c;
    const float* __restrict__ auxb = p.aux ? p.aux + (int64_t)t.bz * p.stride_aux : nullptr;
    const int m0 = t.m0, n0 = t.n0;

    if constexpr (EPI == VASR_EPI_PAIR_POWER || EPI == VASR_EPI_PAIR_FUSION) {
#pragma unroll
        for (int tp = 0; tp < TN / 2; ++tp) {
            const int col = (n0 + wc * 32 * TN) / 2 + tp * 32 + r;  // output column of this lane
            if (GUARD && col >= p.n_out) continue;
            const int pc = n0 + wc * 32 * TN + tp * 64 + r;  // paired column of half 0
            float bg = 0.f, bgl = 0.f, b2 = 0.f;
            float4 qg, qgl, ql;
            if constexpr (EPI == VASR_EPI_PAIR_FUSION) {
                bg = p.bias[pc];
                bgl = p.bias[pc + 32];
                b2 = p.aux2[col];
                if (p.qp) {
                    qg = p.qp[pc];
                    qgl = p.qp[pc + 32];
                    ql = p.qp[2 * p.n_out + col];
                }
            }
#pragma unroll
            for (int tm = 0; tm < TM; ++tm) {
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int row = m0 + wr * 32 * TM + tm * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
                    if (GUARD && row >= p.M) continue;
                    const float v0 = acc[tm][2 * tp][i];
                    const float v1 = acc[tm][2 * tp + 1][i];
                    float out;
                    if constexpr (EPI == VASR_EPI_PAIR_POWER) {
                        out = v0 * v0 + v1 * v1;
                    } else {
                        // aux: local-side partial products in the same paired layout.
                        const float* ar = auxb + (int64_t)row * p.ld_aux;
                        float gp = (ar[pc] + v0) + bg;
                        float lt = ar[pc + 32] + b2;
                        float gt = v1 + bgl;
                        if (p.qp) {
                            gp = fake_quant(gp, qg);
                            lt = fake_quant(lt, ql);
                            gt = fake_quant(gt, qgl);
                        }
                        const float gate = sigmoid_fast(gp);
                        out = gate * lt + (1.0f - gate) * gt;
                    }
                    Cb[(int64_t)row * p.ldc + col] = out;
                }
            }
        }
    } else if constexpr (EPI == VASR_EPI_ARGMAX) {
        // per row: this lane's best over its TN columns (ascending, strict > keeps the first),
        // then the 32-lane max of order-preserving (value, ~index) keys; the wave's TN x 32
        // columns form slots s0 .. s0+TN-1 of 32 columns: slot s0 gets the key, the others 0,
        // so every slot of the row is written (plain stores, no atomics, no zero-init)
        unsigned long long* __restrict__ keys =
            reinterpret_cast<unsigned long long*>(p.C) + (int64_t)t.bz * p.stride_c;
        const int s0 = (n0 + wc * 32 * TN) / 32;
        float bv[TN];
        float4 qc[TN];
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int col = n0 + wc * 32 * TN + tn * 32 + r;
            const bool ok = !GUARD || col < p.N;
            bv[tn] = (p.bias && ok) ? p.bias[col] : 0.0f;
            if (p.qp) qc[tn] = ok ? p.qp[col] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
            unsigned long long kl[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                unsigned long long key = 0ull;
#pragma unroll
                for (int tn = 0; tn < TN; ++tn) {
                    const int col = n0 + wc * 32 * TN + tn * 32 + r;
                    if (GUARD && col >= p.N) continue;
                    float v = acc[tm][tn][i];
                    if (p.bias) v = v + bv[tn];
                    if (p.qp) v = fake_quant(v, qc[tn]);
                    const unsigned u = __float_as_uint(v);
                    const unsigned ord = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
                    const unsigned long long k = ((unsigned long long)ord << 32) | (0xFFFFFFFFu - (unsigned)col);
                    key = k > key ? k : key;
                }
                kl[i] = key;
            }
            if (scr) {
                // transpose through LDS: lane (r, h) writes its 16 row keys to column r of the
                // wave's 32 rows (rows padded to 33 entries: conflict-free column reads), then
                // lane (r, h) reduces half h of row r and the halves meet across h
#pragma unroll
                for (int i = 0; i < 16; ++i) scr[((i & 3) + 8 * (i >> 2) + 4 * h) * 33 + r] = kl[i];
                __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
                __builtin_amdgcn_wave_barrier();
                unsigned long long key = 0ull;
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const unsigned long long k = scr[r * 33 + 16 * h + j];
                    key = k > key ? k : key;
                }
                const unsigned long long o = __shfl_xor(key, 32, 64);
                key = o > key ? o : key;
                __builtin_amdgcn_s_waitcnt(0xC07F);
                __builtin_amdgcn_wave_barrier();  // all reads done before the next tm overwrites scr
                const int row = m0 + wr * 32 * TM + tm * 32 + r;
                if (!GUARD || row < p.M) {
#pragma unroll
                    for (int sl = h; sl < TN; sl += 2)  // h = 0 writes the key slot, h = 1 the zero slots
                        if (!GUARD || (s0 + sl) * 32 < p.N) keys[(int64_t)row * p.ldc + s0 + sl] = sl == 0 ? key : 0ull;
                }
            } else {
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int row = m0 + wr * 32 * TM + tm * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
                    const unsigned long long key = max_u64_over_32_lanes(kl[i]);  // lanes r = 16..31 hold it
                    const int slot = r - (32 - TN);  // lanes r = 32-TN .. 31 write slots s0 .. s0+TN-1
                    if (slot >= 0 && (!GUARD || row < p.M) && (!GUARD || (s0 + slot) * 32 < p.N))
                        keys[(int64_t)row * p.ldc + s0 + slot] = slot == 0 ? key : 0ull;
                }
            }
        }
    } else {
#pragma unroll
        for (int tm = 0; tm < TM; ++tm) {
#pragma unroll
            for (int tn = 0; tn < TN; ++tn) {
                const int col = n0 + wc * 32 * TN + tn * 32 + r;
                if (GUARD && col >= p.N) continue;
                const float bv = p.bias ? p.bias[col] : 0.0f;
                float4 qc;
                if (p.qp) qc = p.qp[col];
                // softplus columns: decided per 32-column MFMA tile (wave-uniform) where possible
                const int cbase = n0 + wc * 32 * TN + tn * 32;
                const bool sp_all = cbase >= p.n_out, sp_none = cbase + 32 <= p.n_out;
                const bool sp = col >= p.n_out;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int row = m0 + wr * 32 * TM + tm * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
                    if (GUARD && row >= p.M) continue;
                    float v = acc[tm][tn][i];
                    if (p.bias) v = v + bv;
                    if (p.qp) v = fake_quant(v, qc);
                    if constexpr (EPI == VASR_EPI_GELU) {
                        v = gelu_fast(v);
                    } else if constexpr (EPI == VASR_EPI_SOFTPLUS_FROM) {
                        if (sp_all) v = softplus20_fast(v);
                        else if (!sp_none) v = sp ? softplus20_fast(v) : v;
                    } else if constexpr (EPI == VASR_EPI_RESIDUAL) {
                        v = v + auxb[(int64_t)row * p.ld_aux + col];
                    } else if constexpr (EPI == VASR_EPI_GELU_PE) {
                        v = gelu_fast(v) + auxb[(int64_t)row * p.ld_aux + col];
                    }
                    Cb[(int64_t)row * p.ldc + col] = v;
                }
            }
        }
    }
}

// scr: optional per-wave LDS scratch of 32 x 33 uint64 for the ARGMAX row reduction (the
// staging LDS is free once the main loop is done); null selects the DPP reduction.
template <int BM, int BN, int TM, int TN, int EPI>
__device__ __forceinline__ void epilogue(const GemmParams& p, const Tile& t, floatx16 (&acc)[TM][TN], int wr,
                                         int wc, int r, int h, unsigned long long* scr = nullptr) {
    const int ncols = (EPI == VASR_EPI_PAIR_POWER || EPI == VASR_EPI_PAIR_FUSION) ? 2 * p.n_out : p.N;
    if (t.m0 + BM <= p.M && t.n0 + BN <= ncols)
        epilogue_body<TM, TN, EPI, false>(p, t, acc, wr, wc, r, h, scr);
    else
        epilogue_body<TM, TN, EPI, true>(p, t, acc, wr, wc, r, h, scr);
}



// Tile configurations: {WM, WN, TM, TN, blocks per CU the kernel's VGPR/LDS use admits}.
struct TileCfg {
    int wm, wn, tm, tn, occ;
    int bm() const { return wm * 32 * tm; }
    int bn() const { return wn * 32 * tn; }
};
constexpr int kCUs = 256;

// Argument checks common to both GEMM entry points; fills p (W / Wx left to the caller).
inline int check_args(const vasr_gemm_args* a, const char* fn, GemmParams& p) {
    VASR_CHECK_ARG(a != nullptr, "%s: null args", fn);
    VASR_CHECK_ARG(a->A && a->C, "%s: null A/C", fn);
    VASR_CHECK_ARG(a->M >= 0 && a->N > 0 && a->K > 0 && a->batch >= 1, "%s: bad shape M=%d N=%d K=%d batch=%d", fn,
                   a->M, a->N, a->K, a->batch);
    VASR_CHECK_ARG(a->K % 4 == 0 && a->lda % 4 == 0 && a->stride_a % 4 == 0,
                   "%s: K, lda, stride_a must be multiples of 4 (K=%d lda=%lld)", fn, a->K, (long long)a->lda);
    VASR_CHECK_ARG((reinterpret_cast<uintptr_t>(a->A) & 15) == 0, "%s: A must be 16-byte aligned", fn);
    const int epi = a->epilogue;
    VASR_CHECK_ARG(epi >= VASR_EPI_NONE && epi <= VASR_EPI_ARGMAX, "%s: unknown epilogue %d", fn, epi);
    if (epi == VASR_EPI_ARGMAX)
        VASR_CHECK_ARG((reinterpret_cast<uintptr_t>(a->C) & 7) == 0 && a->ldc >= (a->N + 31) / 32,
                       "%s: argmax keys must be 8-byte aligned with ldc >= ceil(N / 32) slots", fn);
    const bool pair = epi == VASR_EPI_PAIR_POWER || epi == VASR_EPI_PAIR_FUSION;
    if (pair)
        VASR_CHECK_ARG(a->N % 64 == 0 && a->n_out > 0 && a->n_out <= a->N / 2,
                       "%s: paired epilogue needs N %% 64 == 0 and 0 < n_out <= N/2", fn);
    if (epi == VASR_EPI_RESIDUAL || epi == VASR_EPI_GELU_PE || epi == VASR_EPI_PAIR_FUSION)
        VASR_CHECK_ARG(a->aux != nullptr, "%s: epilogue %d needs aux", fn, epi);
    if (epi == VASR_EPI_PAIR_FUSION)
        VASR_CHECK_ARG(a->aux2 != nullptr && a->bias != nullptr, "%s: fusion needs bias and aux2", fn);
    VASR_CHECK_ARG(!(a->qparams && epi == VASR_EPI_PAIR_POWER), "%s: qparams not allowed with PAIR_POWER", fn);
    VASR_CHECK_ARG((reinterpret_cast<uintptr_t>(a->qparams) & 15) == 0, "%s: qparams must be 16-byte aligned", fn);
    p.A = a->A; p.lda = a->lda; p.stride_a = a->stride_a;
    p.W = a->W; p.ldw = a->ldw; p.Wx = nullptr; p.Kp = 0;
    p.bias = a->bias;
    p.C = a->C; p.ldc = a->ldc; p.stride_c = a->stride_c;
    p.M = a->M; p.N = a->N; p.K = a->K;
    p.aux = a->aux; p.ld_aux = a->ld_aux; p.stride_aux = a->stride_aux;
    p.aux2 = a->aux2; p.n_out = a->n_out;
    p.qp = reinterpret_cast<const float4*>(a->qparams);
    p.batch = a->batch;
    return VASR_OK;
}

}  // namespace gemm

// gemm_rows.hip: launches the A-rows-stationary split GEMM when the shape suits it (batch 1,
// K = 128 / 192, unpaired epilogue) and the engine option allows; returns true with the launch
// status in *rc, false when the tile kernel should run.
bool try_rows_x3(const gemm::GemmParams& p, int batch, int epi, hipStream_t s, int* rc);

}  // namespace vasr
