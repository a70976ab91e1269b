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
// Staging: both operands go global -> LDS by LDS-DMA (global_load_lds_dwordx4, 1 KiB per
// wave-instruction, no VGPRs) into two double-buffer sets that are distinct LDS objects (the
// k loop is unrolled by two), so the compiler does not drain the in-flight prefetch before the
// current buffer's reads; one barrier per k-tile of 32.
//  * A stays fp32 in LDS, [BM][32] with 16-B chunk c of row r at position c ^ f(r),
//    f(r) = ((r >> 1) & 3) ^ (((r >> 3) & 1) << 2): every ds_read_b128 lane group of the
//    fragment read (16 rows, one chunk) then hits 16 distinct 16-B slots of the 256-B bank row
//    (MI355X_MICROARCH.md §LDS lane groups).  LDS-DMA writes lane-linearly, so the swizzle is
//    applied to the source address.  Each wave splits its fragments after the read (VALU that
//    runs in the MFMA shadow).
//  * W is split once (vasr_split_weights_bf16x3) into a fragment-native layout
//    [N/32][Kp/16][3 planes][64 lanes][8 bf16]: one k-step of one plane of one 32-column tile
//    is 1 KiB in lane order, so LDS-DMA and the ds_read_b128 fragment reads are both linear.
//
// Operand maps (cdna_hip_programming.md §3): lane (r = lane & 31, h = lane >> 5) supplies
// A[row r][k = 8h + j] and B[k = 8h + j][col r], j = 0..7.  The accumulator layout equals the
// f32-input MFMA's, so gemm_common.h's epilogues apply.
#include <cstdlib>
#include <type_traits>

#include "gemm_common.h"
#include "gemm_split.h"

namespace vasr {
namespace {

using namespace gemm;

#ifndef VASR_X3_ABLATE
#define VASR_X3_ABLATE 0  // diagnostic builds only: 1 no MFMA, 2 no C stores, 4 no A split,
#endif                    // 8 no LDS-DMA after the first stage, 16 no per-stage barrier

typedef __attribute__((address_space(3))) void lds_void;

constexpr int BK = 32;  // fp32 k per stage (two MFMA k-steps)

__device__ __forceinline__ int a_swz(int r) { return ((r >> 1) & 3) ^ (((r >> 3) & 1) << 2); }

// LDS-DMA of 16 B per lane into dst_base + 16*lane, issued from inline asm: the compiler then
// does not track it, so it adds no waits of its own before reads of other ring slots (its
// tracking loses the slot distinction across the loop back edge and drains the ring).  The
// kernel orders these loads itself: counted vmcnt + barrier before a slot is read.  Extra
// untracked vector-memory operations can only make the compiler's own vmcnt waits stricter.
#ifndef VASR_X3_STAGE
#define VASR_X3_STAGE 0  // diagnostic builds only: 1 compiler LDS-DMA builtin, 2 register staging
#endif
__device__ __forceinline__ void glds16(const void* src, void* dst_base) {
    if constexpr (VASR_X3_STAGE == 1) {
        __builtin_amdgcn_global_load_lds(src, (lds_void*)dst_base, 16, 0, 0);
    } else if constexpr (VASR_X3_STAGE == 2) {
        const float4 v = *reinterpret_cast<const float4*>(src);
        reinterpret_cast<float4*>(dst_base)[threadIdx.x & 63] = v;
    } else {
    const unsigned lds = (unsigned)(uintptr_t)(lds_void*)dst_base;
    // M0 is compiler-reserved: saved and restored inside the statement, and the SALU write of M0
    // needs one wait state before the LDS-DMA reads it (s_nop 0)
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "s"(lds), "v"(src) : "memory");
    }
}

// vmcnt(n) with lgkmcnt / expcnt left open (gfx9 s_waitcnt encoding).
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    if constexpr (VASR_X3_STAGE == 2)
        __builtin_amdgcn_s_waitcnt(0);  // register staging: its LDS writes, before the barrier
    else
        __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// P = 3: the split-bf16 fp32 GEMM described above.  P = 1: the bf16 GEMM of a bf16 model
// (vasr_linear_bf16): W is one bf16 plane, A is rounded to bf16 (RNE) at the fragment read,
// one MFMA per k-step, fp32 accumulation — same staging, same epilogues.
// Blocks per CU the register allocation targets: as many as the LDS ring admits (<= 160 KiB).
template <int WM, int WN, int TM, int TN, int RING, int P>
constexpr int x3_occ() {
    constexpr int lds = RING * (WM * 32 * TM * 128 + WN * TN * 2048 * P);
#ifdef VASR_GEMM_OCC_CAP
    constexpr int cap = VASR_GEMM_OCC_CAP;
#else
    constexpr int cap = 2;
#endif
    return 163840 / lds >= cap ? cap : (163840 / lds >= 1 ? 163840 / lds : 1);
}

template <int WM, int WN, int TM, int TN, int RING, int EPI, int P>
__global__ __launch_bounds__(256, (x3_occ<WM, WN, TM, TN, RING, P>())) void gemm_x3_kernel(GemmParams p) {
    constexpr int BM = WM * 32 * TM;
    constexpr int BN = WN * 32 * TN;
    static_assert(WM * WN == 4, "4 waves");
    static_assert(P == 1 || P == 3, "planes");
    static_assert(TN % 2 == 0 || (EPI != VASR_EPI_PAIR_POWER && EPI != VASR_EPI_PAIR_FUSION), "pairs need even TN");
    constexpr int A_BYTES = BM * BK * 4;            // fp32 [BM][32]
    constexpr int W_BYTES = (BN / 32) * 2 * P * 1024;  // [BN/32][2 k-steps][P planes][64][16 B]
    constexpr int A_INSTR = A_BYTES / 1024, W_INSTR = W_BYTES / 1024;
    static_assert(A_INSTR % 4 == 0 && W_INSTR % 4 == 0, "whole LDS-DMA pieces per wave");

    // RING stages, each one distinct LDS object [A | W] (unused ones are 16-B stubs).  One object
    // per stage keeps the count of distinct LDS-DMA targets small enough for the compiler's
    // waitcnt tracking to tell them apart (it then waits for nothing before a stage's reads).
    static_assert(RING >= 2 && RING <= 4, "ring depth");
    constexpr int STAGE = A_BYTES + W_BYTES;
    __shared__ __attribute__((aligned(16))) char s0[STAGE];
    __shared__ __attribute__((aligned(16))) char s1[STAGE];
    __shared__ __attribute__((aligned(16))) char s2[RING > 2 ? STAGE : 16];
    __shared__ __attribute__((aligned(16))) char s3[RING > 3 ? STAGE : 16];
    constexpr int GL = (A_INSTR + W_INSTR) / 4;  // LDS-DMA instructions per wave per stage

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
    const char* __restrict__ Wf = reinterpret_cast<const char*>(p.Wx);
    const int KS = p.Kp / 16;
    const int NT = (p.N + 31) / 32;
    const int nk = p.Kp / BK;

    // LDS-DMA sources.  A piece j = rows 8j .. 8j+7 of the tile; lane -> (row 8j + lane/8,
    // position lane%8) holding chunk position ^ f(row).  f(row) depends on the lane and on the
    // parity of j only, so a lane's byte offset inside a piece takes two values; the piece and
    // k-tile bases are wave-uniform.  Rows past M re-read row M-1 and chunks past K re-read
    // chunk 0 (finite data; the W planes are zero there and those rows are never stored).
    const int wave_u = __builtin_amdgcn_readfirstlane(wave);
    const int prow = lane >> 3, ppos = lane & 7;
    const int csw = ppos ^ ((prow >> 1) & 3);
    const int a_off[2] = {csw * 16, (csw ^ 4) * 16};  // chunk byte offset in the row, j even / odd
    const bool m_full = m0 + BM <= p.M;
    const char* __restrict__ Ab = reinterpret_cast<const char*>(A);
    const int64_t lda_b = p.lda * 4;
    auto issue = [&](int kt, char* abuf, char* wbuf) {
        if ((VASR_X3_ABLATE & 8) && kt > 0) return;
        const int k0b = kt * BK * 4;
        const bool k_full = (kt + 1) * BK <= p.K;
#pragma unroll
        for (int jj = 0; jj < A_INSTR / 4; ++jj) {
            const int j = jj * 4 + wave_u;
            int off = a_off[j & 1];
            if (!k_full && k0b + off >= p.K * 4) off = 0;
            const char* src;
            if (m_full) {
                src = Ab + (int64_t)(m0 + j * 8) * lda_b + k0b + prow * lda_b + off;
            } else {
                const int gm = min(m0 + j * 8 + prow, p.M - 1);
                src = Ab + (int64_t)gm * lda_b + k0b + off;
            }
            glds16(src, abuf + j * 1024);
        }
#pragma unroll
        for (int jj = 0; jj < W_INSTR / 4; ++jj) {
            const int j = jj * 4 + wave_u;
            const int tnl = j / (2 * P), rem = j - tnl * (2 * P);  // rem = k-step * P + plane
            const int nt = min(n0 / 32 + tnl, NT - 1);
            const char* src = Wf + ((int64_t)(nt * KS + 2 * kt) * P + rem) * 1024 + lane * 16;
            glds16(src, wbuf + j * 1024);
        }
    };

    floatx16 acc[TM][TN];
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[tm][tn][i] = 0.f;

    const int fr = a_swz(r);
    // One stage = two MFMA k-steps.  All fragment reads of the stage are issued first, then
    // step 0's A fragments are split and its MFMAs issued; step 1's split is independent VALU
    // work the scheduler places in the shadow of step 0's MFMAs.
    auto compute = [&](const char* abuf, const char* wbuf) {
        float4 xa[2][TM][2];
        bf16x8 fw[2][P][TN];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int c0 = 4 * s + 2 * h;
#pragma unroll
            for (int tm = 0; tm < TM; ++tm) {
                const char* rowp = abuf + (wr * 32 * TM + tm * 32 + r) * (BK * 4);
                xa[s][tm][0] = *reinterpret_cast<const float4*>(rowp + 16 * (c0 ^ fr));
                xa[s][tm][1] = *reinterpret_cast<const float4*>(rowp + 16 * ((c0 + 1) ^ fr));
            }
#pragma unroll
            for (int tn = 0; tn < TN; ++tn)
#pragma unroll
                for (int pl = 0; pl < P; ++pl)
                    fw[s][pl][tn] = *reinterpret_cast<const bf16x8*>(
                        wbuf + (((wc * TN + tn) * 2 + s) * P + pl) * 1024 + lane * 16);
        }
        bf16x8 fa[2][P][TM];
        auto split_step = [&](int s) {
#pragma unroll
            for (int tm = 0; tm < TM; ++tm) {
                if constexpr (P == 1) {
                    const float4 x0 = xa[s][tm][0], x1 = xa[s][tm][1];
                    const bf16x8 v = {(__bf16)x0.x, (__bf16)x0.y, (__bf16)x0.z, (__bf16)x0.w,
                                      (__bf16)x1.x, (__bf16)x1.y, (__bf16)x1.z, (__bf16)x1.w};
                    fa[s][0][tm] = v;
                } else if constexpr (VASR_X3_ABLATE & 4) {
                    const float4 x0 = xa[s][tm][0], x1 = xa[s][tm][1];
                    const bf16x8 v = {(__bf16)x0.x, (__bf16)x0.y, (__bf16)x0.z, (__bf16)x0.w,
                                      (__bf16)x1.x, (__bf16)x1.y, (__bf16)x1.z, (__bf16)x1.w};
                    fa[s][0][tm] = v;
                    fa[s][P - 1][tm] = v;
                    fa[s][P / 2][tm] = v;
                } else {
                    split8(xa[s][tm][0], xa[s][tm][1], fa[s][0][tm], fa[s][P / 2][tm], fa[s][P - 1][tm]);
                }
            }
        };
        auto mfma_step = [&](int s) {
            if constexpr (VASR_X3_ABLATE & 1) {
#pragma unroll
                for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                    for (int tn = 0; tn < TN; ++tn) acc[tm][tn][0] += (float)fa[s][0][tm][0] * (float)fw[s][P - 1][tn][1];
                return;
            }
            if constexpr (P == 1) {
#pragma unroll
                for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                    for (int tn = 0; tn < TN; ++tn)
                        acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][0][tm], fw[s][0][tn], acc[tm][tn],
                                                                              0, 0, 0);
                return;
            } else {
            // small terms first, then the leading hi*hi term
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int tn = 0; tn < TN; ++tn) {
                    floatx16 c = acc[tm][tn];
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][2][tm], fw[s][0][tn], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][0][tm], fw[s][2][tn], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][1][tm], fw[s][1][tn], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][1][tm], fw[s][0][tn], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][0][tm], fw[s][1][tn], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][0][tm], fw[s][0][tn], c, 0, 0, 0);
                    acc[tm][tn] = c;
                }
            }
        };
        split_step(0);
        mfma_step(0);
        split_step(1);
        mfma_step(1);
    };

    // Ring pipeline: stage kt lives in slot kt % RING; up to RING-1 stages are in flight.  Each
    // step waits for its own stage with a counted vmcnt (the LDS-DMA instructions per wave and
    // stage are a compile-time count, and nothing else touches the vector-memory counter in the
    // loop), then a raw barrier publishes it block-wide and certifies that every wave is done
    // reading the slot the step refills.
    auto slot = [&](auto Ic) -> char* {
        constexpr int I = decltype(Ic)::value;
        if constexpr (I == 0) return s0;
        else if constexpr (I == 1) return s1;
        else if constexpr (I == 2) return s2;
        else return s3;
    };
    // Every step issues exactly GL LDS-DMA instructions (past the last stage it re-loads stage
    // nk-1 into the slot it frees, which nothing reads again), so one wait count serves all
    // steps: vmcnt((RING-2)*GL) leaves the RING-2 younger stages in flight.  The prologue fills
    // RING-1 stages the same way.
    auto step = [&](auto Ic, int kt) {
        constexpr int I = decltype(Ic)::value;
        constexpr int NEXT = (I + RING - 1) % RING;
        wait_vmcnt<(RING - 2) * GL>();
        if constexpr (!(VASR_X3_ABLATE & 16)) __builtin_amdgcn_s_barrier();
        char* nb = slot(std::integral_constant<int, NEXT>());
        issue(min(kt + RING - 1, nk - 1), nb, nb + A_BYTES);
        char* cb = slot(Ic);
        compute(cb, cb + A_BYTES);
    };

    issue(0, s0, s0 + A_BYTES);
    if constexpr (RING > 2) issue(min(1, nk - 1), s1, s1 + A_BYTES);
    if constexpr (RING > 3) issue(min(2, nk - 1), s2, s2 + A_BYTES);
    for (int kt = 0; kt < nk; kt += RING) {
        step(std::integral_constant<int, 0>(), kt);
        if (kt + 1 >= nk) break;
        step(std::integral_constant<int, 1>(), kt + 1);
        if constexpr (RING > 2) {
            if (kt + 2 >= nk) break;
            step(std::integral_constant<int, 2>(), kt + 2);
        }
        if constexpr (RING > 3) {
            if (kt + 3 >= nk) break;
            step(std::integral_constant<int, 3>(), kt + 3);
        }
    }
    // Drain this wave's LDS-DMA (the last step re-loads a stage nothing reads) before the epilogue
    // may reuse the staging LDS and before the workgroup exits: the DMA is inline asm, untracked by
    // the compiler, so __syncthreads() alone would not wait for it.  (Not the cause of the r04
    // concurrent-stream STFT perturbation -- that one stays with register staging, profiles/r04l;
    // see the Makefile's stft.hip rule.)
    __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) expcnt(0) lgkmcnt(0)
    __syncthreads();

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
    // ARGMAX: each wave gets 32 x 33 uint64 of the (now idle) staging LDS, two waves per slot
    unsigned long long* scr = nullptr;
    if constexpr (EPI == VASR_EPI_ARGMAX && STAGE >= 2 * 32 * 33 * 8)  // else: the DPP reduction
        scr = reinterpret_cast<unsigned long long*>(wave < 2 ? s0 : s1) + (wave & 1) * 32 * 33;
    epilogue<BM, BN, TM, TN, EPI>(p, t, acc, wr, wc, r, h, scr);
}

template <int WM, int WN, int TM, int TN, int RING, int P>
int launch_cfg(const GemmParams& p, int batch, int epi, hipStream_t s) {
    constexpr int BM = WM * 32 * TM;
    constexpr int BN = WN * 32 * TN;
    const int tiles = ((p.N + BN - 1) / BN) * ((p.M + BM - 1) / BM);
    dim3 grid(tiles, batch);
    dim3 block(256);
#define VASR_L(E) hipLaunchKernelGGL((gemm_x3_kernel<WM, WN, TM, TN, RING, E, P>), grid, block, 0, s, p)
    switch (epi) {
        case VASR_EPI_NONE: VASR_L(VASR_EPI_NONE); break;
        case VASR_EPI_GELU: VASR_L(VASR_EPI_GELU); break;
        case VASR_EPI_SOFTPLUS_FROM: VASR_L(VASR_EPI_SOFTPLUS_FROM); break;
        case VASR_EPI_RESIDUAL: VASR_L(VASR_EPI_RESIDUAL); break;
        case VASR_EPI_GELU_PE: VASR_L(VASR_EPI_GELU_PE); break;
        case VASR_EPI_PAIR_POWER:
            if constexpr (TN % 2 == 0) { VASR_L(VASR_EPI_PAIR_POWER); break; }
            set_error("vasr_linear_x3_f32: paired epilogue needs an even TN"); return VASR_EINVAL;
        case VASR_EPI_ARGMAX: VASR_L(VASR_EPI_ARGMAX); break;
        case VASR_EPI_PAIR_FUSION:
            if constexpr (TN % 2 == 0) { VASR_L(VASR_EPI_PAIR_FUSION); break; }
            set_error("vasr_linear_x3_f32: paired epilogue needs an even TN"); return VASR_EINVAL;
        default: set_error("vasr_linear_x3_f32: unknown epilogue %d", epi); return VASR_EINVAL;
    }
#undef VASR_L
    return launch_status("vasr_linear_x3_f32");
}


// Tile shapes, largest first.  Measured (tools/gemm_variant_sweep.py, M = 16032): the
// 128 x 128 tile has the best main loop (1.0 : 0.89 for 128 x 64 : 0.76 for 64 x 64 at long K)
// and wins whenever it still yields about two tiles per CU; below that the CU balance of the
// smaller tiles wins.  occ: min(waves per SIMD from the register use, 160 KiB / LDS per block).
#ifndef VASR_X3_RING
#define VASR_X3_RING 2  // deeper rings (3, 4) measured slower: they cost a block per CU
#endif
constexpr int RING_SMALL = VASR_X3_RING;                      // 64 x 64 tiles
constexpr int RING_BIG = VASR_X3_RING > 3 ? 3 : VASR_X3_RING;  // larger tiles
#ifndef VASR_BF16_RING
#define VASR_BF16_RING 2
#endif
constexpr int RING_B16 = VASR_BF16_RING;  // bf16 (one plane): a stage is 24 KiB at 128 x 128
constexpr TileCfg kCfgs[] = {
    {2, 2, 2, 2, 2},  // 128 x 128
    {4, 1, 1, 2, 2},  // 128 x  64
    {2, 2, 1, 1, 4},  //  64 x  64
};

// Tiles a launch needs before a larger tile shape is taken: 1.9 per CU for 128 x 128, 1.4 per
// CU for 128 x 64 (FFN1 at the bench's 16-clip M = 8016: 378 tiles of 128 x 64 measured 1-1.5 %
// faster end to end than 756 of 64 x 64; N = 192 at 189 tiles stays on 64 x 64, 4 % faster).
// VASR_X3_MIN_TILES overrides both (read once; diagnostic).
static long x3_min_tiles(int cfg) {
    static const long v = [] {
        const char* e = std::getenv("VASR_X3_MIN_TILES");
        return e ? std::atol(e) : 0L;
    }();
    if (v > 0) return v;
    return cfg == 0 ? 19L * kCUs / 10 : 14L * kCUs / 10;
}

int pick_x3(int M, int N, int batch, bool pair) {
    for (int i = 0; i < 2; ++i) {
        // N <= 192 (three 64-column tiles or fewer): 64 x 64 tiles at any M (the temporal binding and
        // the fusion's out_proj at M = 16032: 15.7 vs 16.7 and 12.9 vs 13.9 us for 128 x 64,
        // profiles/r06an/)
        if (i == 1 && N <= 192 && !pair) break;
        const TileCfg& c = kCfgs[i];
        const long tiles = (long)((M + c.bm() - 1) / c.bm()) * ((N + c.bn() - 1) / c.bn()) * batch;
        const bool exact_n = N % c.bn() == 0 || N > 4 * c.bn();  // little padding waste
        if (tiles >= x3_min_tiles(i) && exact_n) return i;
    }
    return pair ? 1 : 2;  // paired epilogues need an even TN
}

// Fragment-native planes [NT][KS][3][64][8] (NT = ceil(N/32), KS = Kp/16): element (n, k)
// sits in tile n/32, k-step k/16, lane 32*((k%16)/8) + n%32, slot k%8.  One thread per 8
// consecutive k of one (padded) row; rows >= N and k >= K are zero.
__global__ void split_weights_kernel(const float* __restrict__ W, int64_t ldw, int N, int K, int Kp,
                                     uint16_t* __restrict__ out) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int cpr = Kp / 8;
    const int NT = (N + 31) / 32;
    if (q >= (int64_t)NT * 32 * cpr) return;
    const int n = (int)(q / cpr), k0 = (int)(q % cpr) * 8;
    bf16x8 hi, mid, lo;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float x = (n < N && k0 + j < K) ? W[(int64_t)n * ldw + k0 + j] : 0.0f;
        __bf16 a, b, c;
        split1(x, a, b, c);
        hi[j] = a;
        mid[j] = b;
        lo[j] = c;
    }
    const int KS = Kp / 16;
    const int lane = 32 * ((k0 % 16) / 8) + n % 32;
    const int64_t base = ((int64_t)(n / 32) * KS + k0 / 16) * 3 * 512 + lane * 8;
    *reinterpret_cast<bf16x8*>(out + base) = hi;
    *reinterpret_cast<bf16x8*>(out + base + 512) = mid;
    *reinterpret_cast<bf16x8*>(out + base + 1024) = lo;
}

// One bf16 plane in the same fragment-native layout [NT][KS][64][8] from a bf16 (N, K) matrix.
__global__ void pack_bf16_kernel(const uint16_t* __restrict__ W, int64_t ldw, int N, int K, int Kp,
                                 uint16_t* __restrict__ out) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int cpr = Kp / 8;
    const int NT = (N + 31) / 32;
    if (q >= (int64_t)NT * 32 * cpr) return;
    const int n = (int)(q / cpr), k0 = (int)(q % cpr) * 8;
    uint16_t v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (n < N && k0 + j < K) ? W[(int64_t)n * ldw + k0 + j] : (uint16_t)0;
    const int KS = Kp / 16;
    const int lane = 32 * ((k0 % 16) / 8) + n % 32;
    uint16_t* dst = out + ((int64_t)(n / 32) * KS + k0 / 16) * 512 + lane * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) dst[j] = v[j];
}

}  // namespace
}  // namespace vasr

VASR_API int64_t vasr_split_weights_elems(int N, int K) {
    if (N <= 0 || K <= 0) return 0;
    return 3 * (int64_t)((N + 31) / 32 * 32) * ((K + 31) / 32 * 32);
}

VASR_API int vasr_split_weights_bf16x3(const float* W, int64_t ldw, int N, int K, uint16_t* out, void* stream) {
    using namespace vasr;
    VASR_CHECK_ARG(W && out, "vasr_split_weights_bf16x3: null pointer");
    VASR_CHECK_ARG(N > 0 && K > 0 && ldw >= K, "vasr_split_weights_bf16x3: bad shape N=%d K=%d ldw=%lld", N, K,
                   (long long)ldw);
    VASR_CHECK_ARG((reinterpret_cast<uintptr_t>(out) & 15) == 0, "vasr_split_weights_bf16x3: out must be 16-byte aligned");
    const int Kp = (K + 31) / 32 * 32;
    const int64_t n = (int64_t)((N + 31) / 32 * 32) * (Kp / 8);
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
    int rc;
    if (try_rows_x3(p, a->batch, epi, s, &rc)) return rc;
#ifdef VASR_X3_FORCE_CFG
    const int cfg = VASR_X3_FORCE_CFG;  // diagnostic builds only
#else
    const int cfg = pick_x3(a->M, a->N, a->batch, pair);
#endif
    switch (cfg) {
        case 0: return launch_cfg<2, 2, 2, 2, RING_BIG, 3>(p, a->batch, epi, s);
        case 1: return launch_cfg<4, 1, 1, 2, RING_BIG, 3>(p, a->batch, epi, s);
        default: return launch_cfg<2, 2, 1, 1, RING_SMALL, 3>(p, a->batch, epi, s);
    }
}

VASR_API int64_t vasr_pack_weights_bf16_elems(int N, int K) {
    if (N <= 0 || K <= 0) return 0;
    return (int64_t)((N + 31) / 32 * 32) * ((K + 31) / 32 * 32);
}

VASR_API int vasr_pack_weights_bf16(const uint16_t* W, int64_t ldw, int N, int K, uint16_t* out, void* stream) {
    using namespace vasr;
    VASR_CHECK_ARG(W && out, "vasr_pack_weights_bf16: null pointer");
    VASR_CHECK_ARG(N > 0 && K > 0 && ldw >= K, "vasr_pack_weights_bf16: bad shape N=%d K=%d ldw=%lld", N, K,
                   (long long)ldw);
    VASR_CHECK_ARG((reinterpret_cast<uintptr_t>(out) & 15) == 0, "vasr_pack_weights_bf16: out must be 16-byte aligned");
    const int Kp = (K + 31) / 32 * 32;
    const int64_t n = (int64_t)((N + 31) / 32 * 32) * (Kp / 8);
    hipLaunchKernelGGL(pack_bf16_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), W, ldw, N,
                       K, Kp, out);
    return launch_status("vasr_pack_weights_bf16");
}

VASR_API int vasr_linear_bf16(const vasr_gemm_args* a, const uint16_t* w_packed, void* stream) {
    using namespace vasr;
    GemmParams p;
    if (int rc = check_args(a, "vasr_linear_bf16", p)) return rc;
    VASR_CHECK_ARG(w_packed != nullptr && (reinterpret_cast<uintptr_t>(w_packed) & 15) == 0,
                   "vasr_linear_bf16: w_packed must be a 16-byte aligned device pointer");
    if (a->M == 0) return VASR_OK;
    p.Wx = w_packed;
    p.Kp = (a->K + 31) / 32 * 32;
    const int epi = a->epilogue;
    const bool pair = epi == VASR_EPI_PAIR_POWER || epi == VASR_EPI_PAIR_FUSION;
    hipStream_t s = as_stream(stream);
#ifdef VASR_BF16_FORCE_CFG
    const int cfg = VASR_BF16_FORCE_CFG;  // diagnostic builds only
#else
    const int cfg = pick_x3(a->M, a->N, a->batch, pair);
#endif
    switch (cfg) {
        case 0: return launch_cfg<2, 2, 2, 2, RING_B16, 1>(p, a->batch, epi, s);
        case 1: return launch_cfg<4, 1, 1, 2, RING_B16, 1>(p, a->batch, epi, s);
        default: return launch_cfg<2, 2, 1, 1, RING_B16, 1>(p, a->batch, epi, s);
    }
}
