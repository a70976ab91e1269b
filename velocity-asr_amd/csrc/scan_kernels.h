// Selective-SSM scan + D skip + SiLU gate (reference velocity_asr/ssm.py:119-129): the kernels.
// Included by scan_n{16,32,64,128}.hip, one translation unit per state dim (they compile in
// parallel); scan.hip holds the C ABI entry points.
//
// mode 0 reproduces the reference's DEFAULT scan_mode="parallel": _associative_scan
// (ssm.py:216-295), a Blelloch up/down sweep over the time axis padded to a power of two
// whose down-sweep combine re-uses the already-updated right operand and whose result is
// the EXCLUSIVE prefix.  Instead of materialising (B, P, Di, N) arrays
// the kernel streams time and keeps, per state lane, a binary-counter stack of aligned
// blocks: (la, lb) = the block's up-sweep composite, (ca, cb) = the down-sweep prefix right
// after the block.  Pushing element t merges it with its left siblings exactly as the
// up-sweep does and derives (ca, cb) exactly as the down-sweep does, so every float
// operation of the reference tree is performed once, in the same order (the numpy oracle's
// associative_scan_stream is bitwise equal to the literal tree; see oracle/velocity_ref.py).
// The only deviation from the reference arithmetic is exp: dA = exp2(dt * A*log2e) on the
// hardware v_exp_f32 (a few ULP) instead of torch's CPU exp.  Contraction is disabled so
// a*b + c stays two roundings as in the reference.
//
// mode 1 is the true recurrence of scan_mode="sequential" (ssm.py:134-171).
//
// Work decomposition (MI355X): one workgroup = (utterance b, DPB consecutive channels d),
// 4 waves.  G = N/4 lanes share one channel and each lane owns 4 state indices n, held as
// two float2 pairs so the state algebra issues as packed v_pk_mul/v_pk_add_f32 (two lanes'
// worth of fp32 per instruction: the f32 vector peak); tiny launches use G = N/2 lanes with
// 2 state indices each (scan_body.inc is compiled for both layouts).  Per time step each lane leaves its
// partial y = sum_n h C in an LDS tile; the chunk's gated outputs are reduced and written
// from LDS as coalesced row segments.  Time runs in 16-step chunks: x, dt, z, B, C slices
// are staged to LDS (double-buffered, register prefetch of the next chunk); the four
// in-chunk stack levels are compile-time registers (step i's push/merge pattern is a
// constant, full chunks carry no per-step guards); chunk-sized blocks form the upper stack,
// merged once per chunk.  Launches of at most two waves per SIMD run 32-step chunks (five
// in-chunk levels; see launch_n).  Blocks are remapped so all channel blocks of one utterance share
// an XCD (its 4 MiB L2 then serves the B/C slices and the 64-B row segments they share).
#pragma once

#include <type_traits>

#include "gate.h"
#include "vasr_internal.h"

namespace vasr {
namespace {

typedef __attribute__((address_space(3))) void lds_void;

#ifdef VASR_SCAN_STAMPS
// Diagnostic builds only (tools/diag/scan_clock.py): per workgroup of the streaming kernel {XCC id,
// s_memtime and s_memrealtime at entry and exit} -- the shader clock the launch ran at.
__device__ int64_t* g_scan_stamps;
#endif

#ifndef VASR_SCAN_ABLATE
#define VASR_SCAN_ABLATE 0  // diagnostic builds only (tools/scan_ablate.sh): 1 no exp,
#endif                      // 4 no B/C LDS reads, 8 no chunk staging after the first,
                            // 16 no tree update, 32 no gated-output pass, 64 no block barriers
#ifndef VASR_SCAN_WAVES
#define VASR_SCAN_WAVES 3   // waves per SIMD the register allocator targets
#endif
#ifndef VASR_SCAN_WAVES_NPL2
#define VASR_SCAN_WAVES_NPL2 4  // the same for the 2-states-per-lane layout
#endif
#ifndef VASR_SCAN_WAVES_TC32
#define VASR_SCAN_WAVES_TC32 2  // the 32-step-chunk kernel (VASR_SCAN_T=32): one more stack level
#endif
#ifndef VASR_SCAN_FASTSTAGE
#define VASR_SCAN_FASTSTAGE 1  // 0: every chunk's staging addresses from the clamped index path
#endif
#ifndef VASR_SCAN_PRIO
#define VASR_SCAN_PRIO 4  // wave priority between the blocks sharing a CU (ssm_scan_kernel): 0 off, 1 time
                          // phases, 2 chunk-index rotation, 3 fewer chunks first (quarters), 5 = 3 with the last
                          // quarter by youth, 4 = 5 at >= 3 blocks per CU else 2
#endif
#ifndef VASR_SCAN_PRIO_ROT
#define VASR_SCAN_PRIO_ROT 3  // priorities 0 .. ROT-1 rotated by chunk index where fewer than 3 blocks share a CU
#endif
#ifndef VASR_SCAN_PRIO_SHIFT
#define VASR_SCAN_PRIO_SHIFT 13  // rotation period: 2^SHIFT shader cycles per priority phase
#endif
#ifndef VASR_SCAN_UPPER_REG
#define VASR_SCAN_UPPER_REG 5  // upper-stack levels held in registers (the rest in LDS)
#endif
#ifndef VASR_SCAN_PACKED
#define VASR_SCAN_PACKED 1  // 1: state pairs as float2 vectors (v_pk_*_f32); 0: scalar pairs
#endif

// A pair of state values.  Packed v_pk_mul/add_f32 issue at half the rate of their scalar
// forms on gfx950 (no FLOP gain) but halve the instruction count; measured 4 % faster than
// scalar pairs here (tools/scan_ablate.sh), so packed is the default.
#if VASR_SCAN_PACKED
typedef float f2 __attribute__((ext_vector_type(2)));
#else
struct f2 {
    float x, y;
};
__device__ __forceinline__ f2 operator*(f2 a, f2 b) { return f2{a.x * b.x, a.y * b.y}; }
__device__ __forceinline__ f2 operator+(f2 a, f2 b) { return f2{a.x + b.x, a.y + b.y}; }
#endif

constexpr int T = 16;    // time steps per chunk (the chunk-parallel form; the streaming kernel's TC)
constexpr int TP = T + 1;  // padded row of the per-channel partial-sum tile
constexpr int NW = 4;    // waves per block

constexpr int ctz_c(int v) { return v & 1 ? 0 : 1 + ctz_c(v >> 1); }
constexpr int trailing_ones(int v) { return v & 1 ? 1 + trailing_ones(v >> 1) : 0; }
// Level of the stack entry right below a new block at level j after step i (count i+1),
// or -1 when the entry below is the upper (chunk-level) stack.
// lg = in-chunk stack levels (log2 of the chunk length).
constexpr int below_level(int i, int j, int lg = 4) {
    return ((i + 1) >> (j + 1)) == 0 ? -1
           : (j + 1 + ctz_c((i + 1) >> (j + 1)) < lg ? j + 1 + ctz_c((i + 1) >> (j + 1)) : -1);
}

template <int CTRL>
__device__ __forceinline__ float dpp_mov(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}

// lane ^ 16 within each 32-lane half (ds_swizzle bit mode: and 0x1F, or 0, xor 0x10); DPP
// cannot cross a 16-lane row
__device__ __forceinline__ float swz_xor16(float x) {
    return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(x), 0x401F));
}

// Sum over aligned groups of G lanes (G in {4, 8, 16, 32}); every lane gets the sum.
template <int G>
__device__ __forceinline__ float group_sum(float v) {
    v += dpp_mov<0xB1>(v);                          // quad_perm [1,0,3,2]
    v += dpp_mov<0x4E>(v);                          // quad_perm [2,3,0,1]
    if constexpr (G >= 8) v += dpp_mov<0x141>(v);   // row_half_mirror
    if constexpr (G >= 16) v += dpp_mov<0x140>(v);  // row_mirror
    if constexpr (G >= 32) v += swz_xor16(v);
    return v;
}

// partner exchange of a butterfly level: a DPP control, or -1 for lane ^ 16
template <int CTRL>
__device__ __forceinline__ float xchg(float x) {
    if constexpr (CTRL < 0) return swz_xor16(x);
    else return dpp_mov<CTRL>(x);
}

constexpr int log2_c(int v) { return v <= 1 ? 0 : 1 + log2_c(v >> 1); }

// Cross-lane reduction of 8 per-step partial sums over the G lanes of a channel, as a
// transposing butterfly: each level halves the values a lane holds by exchanging the half it
// gives away with its partner (DPP), so the 8 sums cost 7 exchanges and no wait states
// (independent chains) instead of 8 dependent group_sum chains.  Partner masks xor 15, 7,
// 2, 1 (row_mirror, row_half_mirror, quad_perm) keep partners in the same step subset.
// Returns in v[0 .. S_f) the sums of steps j + S_f * (g >> (log2 G - nsplit)).
template <int G>
struct HalfReduce {
    static constexpr int LG = log2_c(G);
    static constexpr int NSPLIT = LG < 3 ? LG : 3;
    static constexpr int SF = 8 >> NSPLIT;
    static __device__ __forceinline__ int step(int j, int g) { return j + SF * (g >> (LG - NSPLIT)); }
};

// One exchange of a level: lanes with sel = 0 get lo + partner's lo, lanes with sel = 1 get
// hi + partner's hi (the partner has the other sel).  Where sel is a whole DPP row or bank of
// the lane index, two bank-/row-masked DPP adds do it (each writes only its half of the lanes);
// the lane ^ 16 exchange is one v_permlane16_swap (rows 1 / 3 of lo trade places with rows 0 / 2
// of hi) and one add; other levels select with v_cndmask first (3 VALU instead of 2).  The
// sums are the same pairs, so every variant gives the same bits.
template <int CTRL, int SELBIT>
__device__ __forceinline__ float exchange_add(float lo, float hi, bool sel) {
    if constexpr (CTRL == -1) {
        static_assert(SELBIT == 4, "lane ^ 16: sel = bit 4");
        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(lo), __float_as_uint(hi), false, false);
        return __uint_as_float(r[0]) + __uint_as_float(r[1]);
    } else if constexpr ((CTRL == 0x140 && SELBIT == 3) || (CTRL == 0x141 && SELBIT == 2)) {
        float s;
        // banks (4-lane groups of a row) with sel = 0 / 1; s_nop 1: the VALU -> DPP read wait states
        if constexpr (CTRL == 0x140)
            asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %1, %1 row_mirror row_mask:0xf bank_mask:0x3\n\t"
                         "v_add_f32_dpp %0, %2, %2 row_mirror row_mask:0xf bank_mask:0xc"
                         : "=&v"(s) : "v"(lo), "v"(hi));
        else
            asm volatile("s_nop 1\n\tv_add_f32_dpp %0, %1, %1 row_half_mirror row_mask:0xf bank_mask:0x5\n\t"
                         "v_add_f32_dpp %0, %2, %2 row_half_mirror row_mask:0xf bank_mask:0xa"
                         : "=&v"(s) : "v"(lo), "v"(hi));
        return s;
    } else {
        const float keep = sel ? hi : lo;
        const float send = sel ? lo : hi;
        return keep + xchg<CTRL>(send);
    }
}

template <int CTRL, int S, int SELBIT = 0>
__device__ __forceinline__ void butterfly_level(float (&v)[8], int g) {
    if constexpr (S >= 2) {
        const bool sel = (g >> SELBIT) & 1;
#pragma unroll
        for (int j = 0; j < S / 2; ++j) v[j] = exchange_add<CTRL, SELBIT>(v[j], v[j + S / 2], sel);
    } else {
        v[0] = v[0] + xchg<CTRL>(v[0]);
    }
}

template <int G>
__device__ __forceinline__ void reduce_half(float (&v)[8], int g) {
    if constexpr (G == 32) {
        butterfly_level<-1, 8, 4>(v, g);     // v_permlane16_swap: lane ^ 16
        butterfly_level<0x140, 4, 3>(v, g);  // row_mirror: lane ^ 15
        butterfly_level<0x141, 2, 2>(v, g);  // row_half_mirror: lane ^ 7
        butterfly_level<0x4E, 1>(v, g);      // quad_perm [2,3,0,1]: lane ^ 2
        butterfly_level<0xB1, 1>(v, g);      // quad_perm [1,0,3,2]: lane ^ 1
    } else if constexpr (G == 16) {
        butterfly_level<0x140, 8, 3>(v, g);  // row_mirror: lane ^ 15
        butterfly_level<0x141, 4, 2>(v, g);  // row_half_mirror: lane ^ 7
        butterfly_level<0x4E, 2, 1>(v, g);   // quad_perm [2,3,0,1]: lane ^ 2
        butterfly_level<0xB1, 1>(v, g);      // quad_perm [1,0,3,2]: lane ^ 1
    } else if constexpr (G == 8) {
        butterfly_level<0x141, 8, 2>(v, g);
        butterfly_level<0x4E, 4, 1>(v, g);
        butterfly_level<0xB1, 2, 0>(v, g);
    } else {
        static_assert(G == 4, "G in {4, 8, 16, 32}");
        butterfly_level<0x4E, 8, 1>(v, g);
        butterfly_level<0xB1, 4, 0>(v, g);
    }
}

// Reduce the partial sums of steps [8*HALF, 8*HALF + 8) and store them to the channel's row
// of the partial-sum tile ([DPB][TC + 1] floats; TC = chunk length).
template <int G, int HALF, int TC = T>
__device__ __forceinline__ void flush_half(float (&yv)[TC], float* yp, int dl, int g) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = yv[HALF * 8 + j];
    reduce_half<G>(v, g);
#pragma unroll
    for (int j = 0; j < HalfReduce<G>::SF; ++j) yp[dl * (TC + 1) + HALF * 8 + HalfReduce<G>::step(j, g)] = v[j];
}

// a * b + c: two roundings as in the reference tree (modes 0), or one fused multiply-add
// (mode 2: v_pk_fma_f32, a third fewer state-update instructions)
template <bool FMA>
__device__ __forceinline__ f2 mad2(f2 a, f2 b, f2 c) {
#pragma clang fp contract(off)
    if constexpr (FMA) {
#if VASR_SCAN_PACKED
        return __builtin_elementwise_fma(a, b, c);
#else
        return f2{__builtin_fmaf(a.x, b.x, c.x), __builtin_fmaf(a.y, b.y, c.y)};
#endif
    } else {
        return a * b + c;
    }
}

// x + y as one scalar v_add_f32 (used where needed: at N = 128).  Left to itself the compiler
// forms the sum of a pair's two halves there as v_pk_add_f32 with the second source's dwords swapped (op_sel:[0,1]
// op_sel_hi:[1,0]): a packed-fp32 form that returned wrong values in a half-wave beside MFMA kernels
// of another stream (profiles/r05e-r05f); tests/test_host.py checks every shipped kernel.
__device__ __forceinline__ float add_f32(float x, float y) {
    float r;
    asm("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
    return r;
}

__device__ __forceinline__ f2 exp2v(f2 v) {
    f2 r;
    r.x = __builtin_amdgcn_exp2f(v.x);
    r.y = __builtin_amdgcn_exp2f(v.y);
    return r;
}

// The kernel body for each lane layout (scan_body.inc): npl4 = 4 state indices per lane
// (G = N/4 lanes per channel), npl2 = 2 per lane (twice the waves for the same work).
// (npl2 first: the chunk-parallel launcher of either layout uses npl2's block-level kernel)
namespace npl2 {
constexpr int NPL = 2;
#include "scan_body.inc"
}  // namespace npl2
namespace npl4 {
constexpr int NPL = 4;
#include "scan_body.inc"
}  // namespace npl4

}  // namespace
}  // namespace vasr

namespace vasr {
// Per-state-dim launchers (scan_n<N>.hip): two = 2 state indices per lane (npl2), else 4.
#define VASR_SCAN_LAUNCHERS(NN)                                                                                    \
    int scan_streaming_n##NN(bool two, int mode, const float* xz, int64_t ld_xz, const float* dt, int64_t ld_dt,   \
                             const float* bc, int64_t ld_bc, const float* A2, const float* D, float* out,           \
                             int64_t ld_out, int B, int L, int Di, hipStream_t s);                                  \
    int scan_chunked_n##NN(bool two, int mode, const float* xz, int64_t ld_xz, const float* dt, int64_t ld_dt,     \
                           const float* bc, int64_t ld_bc, const float* A2, const float* D, float* out,             \
                           int64_t ld_out, int B, int L, int Di, float* ws_a, float* ws_b, hipStream_t s);          \
    int scan_ungated_n##NN(bool two, int mode, const float* x, int64_t ld_x, const float* dt, int64_t ld_dt,        \
                           const float* bc, int64_t ld_bc, const float* A2, const float* D, float* out,             \
                           int64_t ld_out, int B, int L, int Di, hipStream_t s);
VASR_SCAN_LAUNCHERS(16)
VASR_SCAN_LAUNCHERS(32)
VASR_SCAN_LAUNCHERS(64)
VASR_SCAN_LAUNCHERS(128)
#undef VASR_SCAN_LAUNCHERS
// One-launch time-split form (2 state indices per lane; N <= 64)
#define VASR_SCAN_SPLIT_LAUNCHER(NN)                                                                               \
    int scan_split_n##NN(int mode, const float* xz, int64_t ld_xz, const float* dt, int64_t ld_dt, const float* bc, \
                         int64_t ld_bc, const float* A2, const float* D, float* out, int64_t ld_out, int B, int L,   \
                         int Di, hipStream_t s);
VASR_SCAN_SPLIT_LAUNCHER(16)
VASR_SCAN_SPLIT_LAUNCHER(32)
VASR_SCAN_SPLIT_LAUNCHER(64)
#undef VASR_SCAN_SPLIT_LAUNCHER
}  // namespace vasr
