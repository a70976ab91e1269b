// The tail of an SSMBlock as ONE kernel (reference ssm.py:415-425, SSMBlock._forward_impl):
//
//     x1  = out_proj(g) + x               (ssm.py:130 out_proj, :419 residual)
//     h   = LayerNorm_2(x1)               (:422)
//     f   = GELU(ffn.0(h))                (:394-397)
//     out = ffn.3(f) + x1                 (:398-400, :425)
//
// for D = 192, E = 384 (d_model, FFN width / d_inner).  The unfused form is three GEMM launches
// plus a LayerNorm launch that write and re-read x1 (D floats per token) and the FFN
// intermediate (E floats per token) through HBM; here one workgroup owns 32 token rows and
// keeps everything on chip: the scan output tile g (32 x 384 fp32) staged once by LDS-DMA,
// x1 in registers (and in LDS for the LayerNorm), h and f in LDS as the next product's A
// operand.  HBM traffic per token: g in (1536 B), x in (768 B), out (768 B) -- the weights
// (1.3 MB of split planes for the three matrices) stream from L2, the same for every row tile.
//
// Arithmetic: the split-bf16 fp32 GEMM of gemm_x3.hip (x = hi + mid + lo, six bf16 products,
// small terms first), on v_mfma_f32_16x16x32_bf16 (K = 32 per instruction); LayerNorm with the
// float operations of vasr_layer_norm_f32; the same bias / GELU / residual epilogues.  The
// result is an fp32 computation of the block tail; it differs from the unfused launches only
// in the MFMA accumulation grouping (32 k per instruction here, 16 there).
//
// Work decomposition: 4 waves (one per SIMD), 32 token rows (16 for small launches, see
// tail_rows); each output 32 x 192 is 2 x 12
// tiles of 16 x 16 and wave w owns column tiles 3w .. 3w + 2 of both row tiles (FFN1's 32 x 384
// runs as two 192-column halves with the same map), so no two waves need the same weight
// fragment: weights go global -> VGPRs straight from their fragment-native split planes, each
// wave prefetching PD 32-k steps ahead (the 36 steps of the three products form one stream:
// prefetch runs across the product boundaries).  A operands sit in LDS already split into
// their three bf16 planes (each element split once per block, not once per wave), 16-B chunk c
// of row r at c ^ (r & 15) (384-wide) or c ^ (r & 7) (192-wide): conflict-free fragment reads.
// LDS: 72 KiB for the 384-wide planes (g, then f; the fp32 x1 scratch of the LayerNorm lives
// there in between) + 36 KiB for the 192-wide planes of h.
#include <cstdlib>

#include "gate.h"
#include "ssm_fused.h"

namespace vasr {
namespace {

using namespace fused;
using gemm::split8;

constexpr int NSTAGES = 36;      // out_proj 12 k-steps, FFN1 2 halves x 6, FFN2 12
// weight prefetch distance (steps): 3 for the split planes (9 fragments a step), 6 for one
// bf16 plane (3 fragments a step); 2, 4 and 5 measured within 1 us of 3 (tools/tailpd_ab.sh)
#ifndef VASR_TAIL_PD
#define VASR_TAIL_PD 3
#endif
#ifndef VASR_TAIL_PD16
#define VASR_TAIL_PD16 2  // the 16-row form (two waves per SIMD: 256 registers, no spills at 2)
#endif
#ifndef VASR_TAIL_PD12
#define VASR_TAIL_PD12 4  // 12 waves (one column tile each), 16 rows: 154 registers (5: 168, within 0.3 us)
#endif
// Diagnostic ablations (tools/build_variant_lib.sh -DVASR_TAIL_ABLATE=<bits>; results wrong):
// 1 = no weight loads after the prologue's, 2 = no MFMAs (one add per tile keeps the loads
// live), 4 = no A-fragment LDS reads in the steps
#ifndef VASR_TAIL_ABLATE
#define VASR_TAIL_ABLATE 0
#endif
#ifndef VASR_TAIL_PD21
#define VASR_TAIL_PD21 2  // 32 rows, 12 waves: 168 registers with the A fragments pipelined (3: spills)
#endif
template <int NP, int RT = 2, int CT = 3>
constexpr int pd_of() {
    if constexpr (NP == 1) return CT == 3 ? 6 : 8;
    if constexpr (CT == 1) return RT == 1 ? VASR_TAIL_PD12 : VASR_TAIL_PD21;
    if constexpr (CT == 2) return 3;
    return RT == 1 ? VASR_TAIL_PD16 : VASR_TAIL_PD;
}

struct TailParams {
    const float* g;
    int64_t ldg;
    const float* x;
    int64_t ldx;
    const uint16_t* wo;  // out_proj (D x E) in the 16x16x32 fragment layout, 3 planes
    const float* ln_w;
    const float* ln_b;
    float ln_eps;
    const uint16_t* w1;  // ffn.0 (E x D)
    const float* b1;
    const uint16_t* w2;  // ffn.3 (D x E)
    const float* b2;
    float* out;
    int64_t ldo;
    int M;
};

// RT = 16-row tiles per workgroup: 2 (32 rows, one block per CU) or 1 (16 rows, half the LDS,
// two blocks per CU: twice the weight stream per row, two waves per SIMD to hide it).
// CT = 16-column output tiles per wave: 3 (4 waves), or 2 / 1 (6 / 12 waves: the block's
// weight stream split over more waves, each with a deeper prefetch -- the small-M forms, where
// one block per CU leaves the registers for it)
template <int NP, int RT, int CT = 3>
struct TailCtx {
    static constexpr int NWV = 12 / CT;  // waves per workgroup
    static constexpr int PD = pd_of<NP, RT, CT>();
    static constexpr int RING = PD + 1;
    static constexpr int ROWS = 16 * RT;
    static constexpr int PE = ROWS * TE * 2;  // one bf16 plane of a 384-wide A tile
    static constexpr int PDB = ROWS * TD * 2;  // one bf16 plane of a 192-wide A tile
    const TailParams& P;
    char* R;   // 384-wide planes (g, f) / fp32 x1 scratch
    char* H;   // 192-wide planes (h)
    int lane, wave, r, q, m0;
    floatx4 acc[RT][CT];
    bf16x8 a[2][RT][NP];  // A fragments of this step and the next
    bf16x8 w[RING][CT][NP];  // [ring slot][column tile][plane]
    float x1[RT][CT][4];     // residual x, then x1 = out_proj(g) + x
    float bb1[2][CT], bb2[CT], lnw[3], lnb[3];
#ifdef VASR_TAIL_STAMPS
    uint64_t ts[13];  // diagnostic builds: s_memtime at the phase boundaries (wave 0)
#endif
};

#ifdef VASR_TAIL_STAMPS
// Diagnostic builds only (-DVASR_TAIL_STAMPS, tools/diag/tail_stamps.py): per workgroup of the gated
// tail, 16 int64: HW_ID | XCC << 32, s_memrealtime at entry and exit, s_memtime at 12 phase boundaries
// (slots 9-11: inside the tail steps, tools/diag/tail_stamps.py orders them).
__device__ int64_t* g_tail_stamps;
#define TAIL_STAMP(c, i) ((c).ts[i] = __builtin_amdgcn_s_memtime())
#else
#define TAIL_STAMP(c, i) ((void)0)
#endif

// weight fragments of step S for this wave: column tiles CT w .. CT w + CT - 1, NP planes, from the
// fragment layout [N/16][K/32][NP][64][8]
template <int S, int NP, int RT, int CT>
__device__ __forceinline__ void load_w(TailCtx<NP, RT, CT>& c) {
    const uint16_t* W;
    int nt0, ks, KS;
    if constexpr (S < 12) {
        W = c.P.wo, nt0 = 0, ks = S, KS = TE / 32;
    } else if constexpr (S < 24) {
        W = c.P.w1, nt0 = 12 * ((S - 12) / 6), ks = (S - 12) % 6, KS = TD / 32;
    } else {
        W = c.P.w2, nt0 = 0, ks = S - 24, KS = TE / 32;
    }
#pragma unroll
    for (int t = 0; t < CT; ++t) {
        const int nt = nt0 + CT * c.wave + t;
#pragma unroll
        for (int pl = 0; pl < NP; ++pl)
            c.w[S % TailCtx<NP, RT, CT>::RING][t][pl] =
                *reinterpret_cast<const bf16x8*>(W + ((int64_t)(nt * KS + ks) * NP + pl) * 512 + c.lane * 8);
    }
}

// the first PD steps' weights (prologue)
template <int S, int NP, int RT, int CT>
__device__ __forceinline__ void load_first(TailCtx<NP, RT, CT>& c) {
    load_w<S, NP, RT, CT>(c);
    if constexpr (S + 1 < TailCtx<NP, RT, CT>::PD) load_first<S + 1, NP, RT, CT>(c);
}

template <int S, int NP, int RT, int CT>
__device__ __forceinline__ void read_step_a(TailCtx<NP, RT, CT>& c, bf16x8 (&a)[RT][NP]) {
    using Ctx = TailCtx<NP, RT, CT>;
#pragma unroll
    for (int tm = 0; tm < RT; ++tm) {
        if constexpr ((VASR_TAIL_ABLATE & 4) != 0) {
#pragma unroll
            for (int pl = 0; pl < NP; ++pl) a[tm][pl] = c.w[(S + 1) % Ctx::RING][0][pl];
            continue;
        }
        if constexpr (S < 12 || S >= 24)
            read_a<NP, TE, Ctx::ROWS>(c.R, 16 * tm + c.r, S < 12 ? S : S - 24, c.q, a[tm]);
        else
            read_a<NP, TD, Ctx::ROWS>(c.H, 16 * tm + c.r, (S - 12) % 6, c.q, a[tm]);
    }
}

template <int S, int NP, int RT, int CT>
__device__ __forceinline__ void tail_step(TailCtx<NP, RT, CT>& c) {
    using Ctx = TailCtx<NP, RT, CT>;
    constexpr int PD = Ctx::PD;
    if constexpr (S + PD < NSTAGES && !(VASR_TAIL_ABLATE & 1)) load_w<S + PD, NP, RT, CT>(c);
    // keep the prefetch where it is: without this fence the scheduler sinks the loads next to
    // their use (to save registers) and the step then waits on them (measured: the weight
    // stream then ran at a third of the L2 rate)
    __builtin_amdgcn_sched_barrier(0);
    // A fragments of both row tiles, read one step ahead of their MFMAs: the next step's are
    // issued before this step's products (whose fragments were read a step earlier), so an LDS
    // round trip no longer sits in front of every step's first MFMA.  Steps 0, 12 and 24 start a
    // product whose A image is written at the end of the step before (LN at 11, f at 23): they
    // read their own.  Measured (graph-timed, profiles/r04ap, r04aq): the A reads were the
    // largest single cost of a step -- without them the M = 501 launch took 8.9 instead of 15.9
    // us -- and pipelining them took it to 13.4 us (12 waves), M = 16032 from 50 to 48 us;
    // bitwise the same outputs.
    constexpr bool first = S == 0 || S == 12 || S == 24;
    if constexpr (first) read_step_a<S, NP, RT, CT>(c, c.a[S & 1]);
    if constexpr (S + 1 < NSTAGES && S + 1 != 12 && S + 1 != 24) read_step_a<S + 1, NP, RT, CT>(c, c.a[(S + 1) & 1]);
    __builtin_amdgcn_sched_barrier(0);  // keep those reads ahead of this step's MFMAs
    auto& a = c.a[S & 1];
#pragma unroll
    for (int tm = 0; tm < RT; ++tm)
#pragma unroll
        for (int t = 0; t < CT; ++t) {
            if constexpr ((VASR_TAIL_ABLATE & 2) != 0) {
                c.acc[tm][t][0] += (float)c.w[S % Ctx::RING][t][0][0] + (float)a[tm][0][1];
                continue;
            }
            c.acc[tm][t] = mac_tile<NP>(a[tm], c.w[S % Ctx::RING][t], c.acc[tm][t]);
        }

    if constexpr (S == 11) {
        // x1 = out_proj(g) + x (registers, kept for the final residual) -> fp32 scratch in R
        // (the g planes are dead once every wave is past its last GEMM1 read)
        TAIL_STAMP(c, 9);
        lds_barrier();
        float* xs = reinterpret_cast<float*>(c.R);
#pragma unroll
        for (int tm = 0; tm < RT; ++tm)
#pragma unroll
            for (int t = 0; t < CT; ++t) {
                const int col = 16 * (CT * c.wave + t) + c.r;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    c.x1[tm][t][i] = c.acc[tm][t][i] + c.x1[tm][t][i];
                    xs[(16 * tm + 4 * c.q + i) * TD + col] = c.x1[tm][t][i];
                }
                c.acc[tm][t] = floatx4{0.f, 0.f, 0.f, 0.f};
            }
        lds_barrier();
        TAIL_STAMP(c, 10);
        // h = LayerNorm_2(x1): one wave per row with vasr_layer_norm_f32's operations, each
        // value split into the three planes of H
        for (int rr = c.wave; rr < Ctx::ROWS; rr += Ctx::NWV) {
            float v[3];
            float sum = 0.f;
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                v[i] = xs[rr * TD + c.lane + 64 * i];
                sum += v[i];
            }
            const float mean = wave_sum(sum) / (float)TD;
            float qs = 0.f;
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const float d = v[i] - mean;
                qs += d * d;
            }
            const float var = wave_sum(qs) / (float)TD;
            const float rstd = 1.0f / sqrtf(var + c.P.ln_eps);
#pragma unroll
            for (int i = 0; i < 3; ++i)
                split_store<NP>(c.H, Ctx::PDB, poff<TD>(rr, c.lane + 64 * i), __builtin_fmaf((v[i] - mean) * rstd, c.lnw[i], c.lnb[i]));
        }
        lds_barrier();  // h complete; the scratch in R is free for f
        TAIL_STAMP(c, 5);
    } else if constexpr (S == 17 || S == 23) {
        // f = GELU(ffn.0(h) + b1), FFN1 column half hh, split into the planes of R
        constexpr int hh = S == 17 ? 0 : 1;
#pragma unroll
        for (int tm = 0; tm < RT; ++tm)
#pragma unroll
            for (int t = 0; t < CT; ++t) {
                const int col = TD * hh + 16 * (CT * c.wave + t) + c.r;
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    split_store<NP>(c.R, Ctx::PE, poff<TE>(16 * tm + 4 * c.q + i, col),
                                gelu_fast(c.acc[tm][t][i] + c.bb1[hh][t]));
                c.acc[tm][t] = floatx4{0.f, 0.f, 0.f, 0.f};
            }
        if constexpr (S == 17) TAIL_STAMP(c, 11);
        if constexpr (S == 23) {
            lds_barrier();  // f complete before FFN2 reads it
            TAIL_STAMP(c, 6);
        }
    }
    if constexpr (S + 1 < NSTAGES) tail_step<S + 1, NP, RT, CT>(c);
}

template <int NP, int RT, int CT = 3>
__global__ __launch_bounds__(64 * (12 / CT), RT == 1 && CT == 3 ? 2 : 1) void ssm_tail_kernel(TailParams P) {
    using Ctx = TailCtx<NP, RT, CT>;
    constexpr int NT = 64 * Ctx::NWV;  // threads
    __shared__ __attribute__((aligned(16))) char R[NP * Ctx::PE];
    __shared__ __attribute__((aligned(16))) char H[NP * Ctx::PDB];
    Ctx c{P, R, H};
    c.lane = threadIdx.x & 63;
    c.wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    c.r = c.lane & 15;
    c.q = c.lane >> 4;
    c.m0 = blockIdx.x * Ctx::ROWS;
    // weights of the first PD steps, then the g tile (split once into R's planes), the residual
    // x and the epilogue constants: all of these loads are in flight together
    load_first<0, NP, RT, CT>(c);
    __builtin_amdgcn_sched_barrier(0);
    constexpr int UNITS = Ctx::ROWS * TE / 8;  // 8-float chunks of the g tile
    static_assert(UNITS % NT == 0, "whole g-tile staging rounds");
#pragma unroll
    for (int k = 0; k < UNITS / NT; ++k) {
        const int u = threadIdx.x + NT * k;
        const int rr = u / (TE / 8), ch = u - rr * (TE / 8);
        const float* src = P.g + (int64_t)min(c.m0 + rr, P.M - 1) * P.ldg + 8 * ch;
        const float4 v0 = *reinterpret_cast<const float4*>(src);
        const float4 v1 = *reinterpret_cast<const float4*>(src + 4);
        split_store8<NP>(R, Ctx::PE, rr * TE * 2 + ((ch ^ (rr & 15)) << 4), v0, v1);
    }
#pragma unroll
    for (int tm = 0; tm < RT; ++tm)
#pragma unroll
        for (int t = 0; t < CT; ++t) {
            const int col = 16 * (CT * c.wave + t) + c.r;
            c.bb2[t] = P.b2[col];
            c.bb1[0][t] = P.b1[col];
            c.bb1[1][t] = P.b1[TD + col];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = c.m0 + 16 * tm + 4 * c.q + i;
                c.x1[tm][t][i] = row < P.M ? P.x[(int64_t)row * P.ldx + col] : 0.0f;
            }
            c.acc[tm][t] = floatx4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        c.lnw[i] = P.ln_w[c.lane + 64 * i];
        c.lnb[i] = P.ln_b[c.lane + 64 * i];
    }
    lds_barrier();  // the g planes are complete
    tail_step<0, NP, RT, CT>(c);
    // out = ffn.3(f) + b2 + x1
#pragma unroll
    for (int tm = 0; tm < RT; ++tm)
#pragma unroll
        for (int t = 0; t < CT; ++t) {
            const int col = 16 * (CT * c.wave + t) + c.r;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = c.m0 + 16 * tm + 4 * c.q + i;
                if (row < P.M) P.out[(int64_t)row * P.ldo + col] = (c.acc[tm][t][i] + c.bb2[t]) + c.x1[tm][t][i];
            }
        }
}

// ---------------------------------------------------------------------------------------------
// The z-in-tail block: z = in_proj_z(u) is read only by the gate y * silu(z)
// (ssm.py:106, :129), so the projection GEMM leaves its 384 z columns out (its C stores are what
// bound it), the scan writes the ungated y + x D (vasr_ssm_scan_ungated_f32), and
// this kernel forms z itself before the tail:
//   z = u @ W_z^T      the rows / tile engines' exact product: per 32 x 32 chunk, 12 k-steps of
//                      the same six v_mfma_f32_32x32x16_bf16 split products in the same order
//                      (gemm_rows.hip), A = u split into its three planes, W_z in the
//                      vasr_split_weights_bf16x3 layout -- so z is bitwise the projection's z;
//   g = yD * silu(z)   the scan's gate (gate.h), into R's planes: bitwise the scan's g;
// then the 36 steps of ssm_tail_kernel.  One workgroup = 32 rows x 12 waves (the form of
// M > 4096): wave w owns z columns 32 w .. 32 w + 31, i.e. chunk w of W_z, all 32 rows.
typedef float floatx16 __attribute__((ext_vector_type(16)));

struct GateParams {
    const float* yd;      // (M, E) y + x D, row stride ldy
    int64_t ldy;
    const float* u;       // (M, D) the projection's input (ln_dwconv output), row stride ldu
    int64_t ldu;
    const uint16_t* wz;   // W_z = in_proj rows Di..2Di-1 as vasr_split_weights_bf16x3 planes
};

// g = y * silu(z) into R's NP planes, with contraction off for the product AND the split: left to the
// default (fp-contract=fast) the compiler forms the split's residual g - hi as one fma from the
// unrounded product, i.e. planes of a more exact g than the scan writes (1e-6 differences at the block
// output; the scan TU is built with -ffp-contract=off).  NP = 3 (fp32 model): z + 0.0f, as the
// projection's epilogue adds its zero bias to the z columns (the same sign of a zero); NP = 1 (bf16
// model): in_proj has no bias and the one plane is g rounded to bf16, as the bf16 tail's staging does.
template <int MODE, int NP>
__device__ __forceinline__ void gate_split_store(char* plane0, int plane_bytes, int off, float y, float z) {
#pragma clang fp contract(off)
    if constexpr (NP == 3) {
        const float v = y * silu_of<MODE>(z + 0.0f);
        const __bf16 hi = (__bf16)v;
        const float r1 = v - (float)hi;
        const __bf16 mid = (__bf16)r1;
        const __bf16 lo = (__bf16)(r1 - (float)mid);
        *reinterpret_cast<__bf16*>(plane0 + off) = hi;
        *reinterpret_cast<__bf16*>(plane0 + plane_bytes + off) = mid;
        *reinterpret_cast<__bf16*>(plane0 + 2 * plane_bytes + off) = lo;
    } else {
        *reinterpret_cast<__bf16*>(plane0 + off) = (__bf16)(y * silu_of<MODE>(z));
    }
}

// four consecutive columns of one row (one 8-B piece per plane): the same float operations per value
template <int MODE, int NP>
__device__ __forceinline__ void gate_split_store4(char* plane0, int plane_bytes, int off, const float4& y,
                                                  const floatx4& z) {
#pragma clang fp contract(off)
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    const float yy[4] = {y.x, y.y, y.z, y.w};
    bf16x4 hi, mid, lo;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if constexpr (NP == 3) {
            const float v = yy[i] * silu_of<MODE>(z[i] + 0.0f);
            hi[i] = (__bf16)v;
            const float r1 = v - (float)hi[i];
            mid[i] = (__bf16)r1;
            lo[i] = (__bf16)(r1 - (float)mid[i]);
        } else {
            hi[i] = (__bf16)(yy[i] * silu_of<MODE>(z[i]));
        }
    }
    *reinterpret_cast<bf16x4*>(plane0 + off) = hi;
    if constexpr (NP == 3) {
        *reinterpret_cast<bf16x4*>(plane0 + plane_bytes + off) = mid;
        *reinterpret_cast<bf16x4*>(plane0 + 2 * plane_bytes + off) = lo;
    }
}

// NP = 3: the fp32 model (split planes; z by the rows / tile engines' six products per k-step).
// NP = 1: the bf16 model (one bf16 plane; z by the bf16 tile engine's one product per k-step, A = u
// rounded to bf16, W_z as vasr_pack_weights_bf16's layout).
#ifndef VASR_TAILG_ZPD
#define VASR_TAILG_ZPD 2
#endif
// SWAP: z^T = W_z u^T (the same MFMAs with the operands exchanged: each output element is the same dot
// product of the same bf16 pairs in the same k order), so a lane holds 16 z columns of ONE token in
// four runs of four: y + x D arrives as four float4 loads and g leaves as one 8-B store per run and
// plane (instead of 16 scalar loads and 16 x NP two-byte stores); the u tile's loads go first
#ifndef VASR_TAILG_XCD
#define VASR_TAILG_XCD 1
#endif
#ifndef VASR_TAILG_SWAP
#define VASR_TAILG_SWAP 1
#endif
template <int MODE, int NP>
__global__ __launch_bounds__(768, 1) void ssm_tail_gated_kernel(TailParams P, GateParams G) {
    using Ctx = TailCtx<NP, 2, 1>;
    constexpr int NT = 768;
    constexpr int KSZ = TD / 16;  // z k-steps (16 k each)
    __shared__ __attribute__((aligned(16))) char R[NP * Ctx::PE];
    __shared__ __attribute__((aligned(16))) char H[NP * Ctx::PDB];
    Ctx c{P, R, H};
    c.lane = threadIdx.x & 63;
    c.wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    c.r = c.lane & 15;
    c.q = c.lane >> 4;
#if VASR_TAILG_XCD
    // XCD-aware tile order: workgroups id, id + 8, ... run on one XCD; give each such group a run of
    // consecutive row tiles, as the scan gives each XCD a run of consecutive utterances
    // (scan_body.inc), so a tile's y + x D rows were written through the same L2
    {
        const int nblk = (int)gridDim.x, id = (int)blockIdx.x;
        const int q8 = nblk / 8, r8 = nblk % 8, xg = id % 8;
        c.m0 = ((xg < r8 ? xg * (q8 + 1) : r8 * (q8 + 1) + (xg - r8) * q8) + id / 8) * Ctx::ROWS;
    }
#else
    c.m0 = blockIdx.x * Ctx::ROWS;
#endif
#ifdef VASR_TAIL_STAMPS
    const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
#endif
    TAIL_STAMP(c, 0);
    const int zr = c.lane & 31, zh = c.lane >> 5;  // 32x32x16 operand map: row / column zr, k half zh
    const int zcol = 32 * c.wave + zr;
    // W_z fragments of k-steps 0 .. ZPD-1 (chunk `wave` of the layout: [KSZ][NP][64 lanes][16 B])
    constexpr int ZPD = VASR_TAILG_ZPD;  // k-steps of W_z in flight
    const char* wzc = reinterpret_cast<const char*>(G.wz) + (int64_t)c.wave * KSZ * NP * 1024 + c.lane * 16;
    bf16x8 wf[ZPD + 1][NP];
    static_assert(Ctx::ROWS * TD / 8 == NT, "one 8-float chunk of u per thread");
    const int urr = threadIdx.x / (TD / 8), uch = threadIdx.x - urr * (TD / 8);
    float4 uv0, uv1;
#if VASR_TAILG_SWAP
    // the u tile's loads first: its LDS image is the first thing every wave waits for
    {
        const float* src = G.u + (int64_t)min(c.m0 + urr, P.M - 1) * G.ldu + 8 * uch;
        uv0 = *reinterpret_cast<const float4*>(src);
        uv1 = *reinterpret_cast<const float4*>(src + 4);
    }
#endif
#pragma unroll
    for (int ks = 0; ks < ZPD; ++ks)
#pragma unroll
        for (int pl = 0; pl < NP; ++pl) wf[ks][pl] = *reinterpret_cast<const bf16x8*>(wzc + (ks * NP + pl) * 1024);
#if VASR_TAILG_SWAP
    // y + x D of token zr at z columns 32 w + 8 j + 4 zh .. + 3 (j = 0..3)
    float4 yv4[4];
    {
        const int row = c.m0 + zr;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            yv4[j] = row < P.M ? *reinterpret_cast<const float4*>(G.yd + (int64_t)row * G.ldy + 32 * c.wave + 8 * j + 4 * zh)
                               : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#else
    // y + x D at this lane's z positions (rows (i & 3) + 8 (i >> 2) + 4 zh of the tile)
    float yv[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int row = c.m0 + (i & 3) + 8 * (i >> 2) + 4 * zh;
        yv[i] = row < P.M ? G.yd[(int64_t)row * G.ldy + zcol] : 0.0f;
    }
    {
        const float* src = G.u + (int64_t)min(c.m0 + urr, P.M - 1) * G.ldu + 8 * uch;
        uv0 = *reinterpret_cast<const float4*>(src);
        uv1 = *reinterpret_cast<const float4*>(src + 4);
    }
#endif
    // u tile -> H's NP planes (192-wide layout; rows past M repeat row M - 1, never stored)
    split_store8<NP>(H, Ctx::PDB, urr * TD * 2 + ((uch ^ (urr & 7)) << 4), uv0, uv1);
    lds_barrier();  // u planes complete
    TAIL_STAMP(c, 1);
    auto read_u = [&](int ks, bf16x8 (&a)[NP]) {
#pragma unroll
        for (int pl = 0; pl < NP; ++pl)
            a[pl] = *reinterpret_cast<const bf16x8*>(H + pl * Ctx::PDB + zr * TD * 2 + (((2 * ks + zh) ^ (zr & 7)) << 4));
    };
    bf16x8 af[2][NP];
    read_u(0, af[0]);
    floatx16 zc;
#pragma unroll
    for (int i = 0; i < 16; ++i) zc[i] = 0.f;
#pragma unroll
    for (int ks = 0; ks < KSZ; ++ks) {
        if (ks + ZPD < KSZ) {
#pragma unroll
            for (int pl = 0; pl < NP; ++pl)
                wf[(ks + ZPD) % (ZPD + 1)][pl] = *reinterpret_cast<const bf16x8*>(wzc + ((ks + ZPD) * NP + pl) * 1024);
        }
        if (ks + 1 < KSZ) read_u(ks + 1, af[(ks + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
        const bf16x8(&a)[NP] = af[ks & 1];
        const bf16x8(&w)[NP] = wf[ks % (ZPD + 1)];
#if VASR_TAILG_SWAP
#define ZMFMA(x, y) __builtin_amdgcn_mfma_f32_32x32x16_bf16(y, x, zc, 0, 0, 0)
#else
#define ZMFMA(x, y) __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, y, zc, 0, 0, 0)
#endif
        if constexpr (NP == 3) {
            // gemm_rows.hip's order: small terms first, then the leading hi * hi term
            zc = ZMFMA(a[2], w[0]);
            zc = ZMFMA(a[0], w[2]);
            zc = ZMFMA(a[1], w[1]);
            zc = ZMFMA(a[1], w[0]);
            zc = ZMFMA(a[0], w[1]);
        }
        zc = ZMFMA(a[0], w[0]);
#undef ZMFMA
        __builtin_amdgcn_sched_barrier(0);
    }
    // the first PD steps' weights of the tail's own stream, in flight during the gate
    TAIL_STAMP(c, 2);
    load_first<0, NP, 2, 1>(c);
    // g = (y + x D) * silu(z) into R's planes
#if VASR_TAILG_SWAP
#pragma unroll
    for (int j = 0; j < 4; ++j)
        gate_split_store4<MODE, NP>(R, Ctx::PE, poff<TE>(zr, 32 * c.wave + 8 * j + 4 * zh), yv4[j],
                                    floatx4{zc[4 * j], zc[4 * j + 1], zc[4 * j + 2], zc[4 * j + 3]});
#else
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int rl = (i & 3) + 8 * (i >> 2) + 4 * zh;
        gate_split_store<MODE, NP>(R, Ctx::PE, poff<TE>(rl, zcol), yv[i], zc[i]);
    }
#endif
#pragma unroll
    for (int tm = 0; tm < 2; ++tm) {
        const int col = 16 * c.wave + c.r;
        c.bb2[0] = P.b2[col];
        c.bb1[0][0] = P.b1[col];
        c.bb1[1][0] = P.b1[TD + col];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = c.m0 + 16 * tm + 4 * c.q + i;
            c.x1[tm][0][i] = row < P.M ? P.x[(int64_t)row * P.ldx + col] : 0.0f;
        }
        c.acc[tm][0] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        c.lnw[i] = P.ln_w[c.lane + 64 * i];
        c.lnb[i] = P.ln_b[c.lane + 64 * i];
    }
    TAIL_STAMP(c, 3);
    lds_barrier();  // the g planes are complete (and every wave is past its u reads: H is free for h)
    TAIL_STAMP(c, 4);
    tail_step<0, NP, 2, 1>(c);
    TAIL_STAMP(c, 7);
#pragma unroll
    for (int tm = 0; tm < 2; ++tm) {
        const int col = 16 * c.wave + c.r;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = c.m0 + 16 * tm + 4 * c.q + i;
            if (row < P.M) P.out[(int64_t)row * P.ldo + col] = (c.acc[tm][0][i] + c.bb2[0]) + c.x1[tm][0][i];
        }
    }
#ifdef VASR_TAIL_STAMPS
    TAIL_STAMP(c, 8);
    if (threadIdx.x == 0 && g_tail_stamps) {
        const uint64_t rt1 = __builtin_amdgcn_s_memrealtime();
        uint32_t xcc, hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        int64_t* o = g_tail_stamps + 16 * (int64_t)blockIdx.x;
        o[0] = (int64_t)hw | ((int64_t)(xcc & 0xF) << 32);
        o[1] = (int64_t)rt0;
        o[2] = (int64_t)rt1;
#pragma unroll
        for (int i = 0; i < 12; ++i) o[3 + i] = (int64_t)c.ts[i];
    }
#endif
}

// Fragment layout of v_mfma_f32_16x16x32_bf16's B operand, three split planes:
// [ceil(N/16)][Kp/32][3][64 lanes][8], lane l of (tile nt, step ks) holding
// W[16 nt + (l & 15)][32 ks + 8 (l >> 4) + j]; zero outside N x K.
__global__ void split_weights16_kernel(const float* __restrict__ W, int64_t ldw, int N, int K, int Kp,
                                       uint16_t* __restrict__ out) {
    const int64_t qd = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // one thread per 8 k of one row
    const int cpr = Kp / 8;
    const int NT = (N + 15) / 16;
    if (qd >= (int64_t)NT * 16 * cpr) return;
    const int n = (int)(qd / cpr), k0 = (int)(qd % cpr) * 8;
    bf16x8 hi, mid, lo;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float v = (n < N && k0 + j < K) ? W[(int64_t)n * ldw + k0 + j] : 0.0f;
        __bf16 a, b, c;
        gemm::split1(v, a, b, c);
        hi[j] = a;
        mid[j] = b;
        lo[j] = c;
    }
    const int KS = Kp / 32;
    const int ln = 16 * ((k0 % 32) / 8) + n % 16;
    const int64_t base = ((int64_t)(n / 16) * KS + k0 / 32) * 3 * 512 + ln * 8;
    *reinterpret_cast<bf16x8*>(out + base) = hi;
    *reinterpret_cast<bf16x8*>(out + base + 512) = mid;
    *reinterpret_cast<bf16x8*>(out + base + 1024) = lo;
}

// One bf16 plane (the bf16 model's own weights) in the same layout: [ceil(N/16)][Kp/32][64][8].
__global__ void pack_weights16_kernel(const uint16_t* __restrict__ W, int64_t ldw, int N, int K, int Kp,
                                      uint16_t* __restrict__ out) {
    const int64_t qd = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int cpr = Kp / 8;
    const int NT = (N + 15) / 16;
    if (qd >= (int64_t)NT * 16 * cpr) return;
    const int n = (int)(qd / cpr), k0 = (int)(qd % cpr) * 8;
    const int KS = Kp / 32;
    const int ln = 16 * ((k0 % 32) / 8) + n % 16;
    uint16_t* dst = out + ((int64_t)(n / 16) * KS + k0 / 32) * 512 + ln * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) dst[j] = (n < N && k0 + j < K) ? W[(int64_t)n * ldw + k0 + j] : (uint16_t)0;
}

// Rows per workgroup.  A block's time is set by its own weight stream and MFMA chain (23 us at
// 32 rows whatever M is, 21 us at 16), so 16-row blocks win while they still fit one per CU
// (M <= 4096: the global-context blocks, one utterance at a time); above that two 16-row blocks
// per CU duplicate the per-CU L2 -> VGPR weight stream: 33.2 vs 28.3 us at M = 8016,
// 135.5k vs 136.1k RTFx end to end (profiles/r02e/tail_rows.txt).  vasr_set_option(VASR_OPT_TAIL_ROWS,
// 16|32) (env VASR_TAIL_ROWS) forces one.
int tail_rows(int M) {
    if (const int r = option(VASR_OPT_TAIL_ROWS)) return r;
    return M <= 4096 ? 16 : 32;  // 256 CUs x 16 rows
}

// Waves per workgroup (12 / column tiles per wave).  At 32 rows, 12 waves of one column tile
// each take 23.3 vs 26.2 us at M = 8016 (profiles/r03m/tail.txt: the block's MFMA chain split
// three ways per SIMD).  16-row blocks too, graph-timed: 13.4 vs 15.8 us at M = 501, 13.7 vs
// 16.2 at M = 1024 (profiles/r04aq; round 2's "no gain" had timed the Python call path, which
// at these sizes is slower than the kernel).  vasr_set_option(VASR_OPT_TAIL_WAVES, 4|6|12) (env
// VASR_TAIL_WAVES) forces one.
int tail_waves(int M) {
    if (const int w = option(VASR_OPT_TAIL_WAVES)) return w;
    return 12;
}

template <int NP>
void launch_tail(const TailParams& p, hipStream_t s) {
    const int rows = tail_rows(p.M), waves = tail_waves(p.M);
    const dim3 grid((unsigned)((p.M + rows - 1) / rows)), block(64 * waves);
#define VASR_T(RT, CT) hipLaunchKernelGGL((ssm_tail_kernel<NP, RT, CT>), grid, block, 0, s, p)
    if (rows == 16) {
        if (waves == 12) VASR_T(1, 1);
        else if (waves == 6) VASR_T(1, 2);
        else VASR_T(1, 3);
    } else {
        if (waves == 12) VASR_T(2, 1);
        else if (waves == 6) VASR_T(2, 2);
        else VASR_T(2, 3);
    }
#undef VASR_T
}

int tail_args(const float* g, int64_t ldg, const float* x, int64_t ldx, const uint16_t* wo, const float* ln_w,
              const float* ln_b, const uint16_t* w1, const float* b1, const uint16_t* w2, const float* b2, float* out,
              int64_t ldo, int M, int D, int E, const char* fn) {
    VASR_CHECK_ARG(g && x && wo && ln_w && ln_b && w1 && b1 && w2 && b2 && out, "%s: null pointer", fn);
    VASR_CHECK_ARG(D == TD && E == TE, "%s: built for d_model %d, FFN width %d (got %d, %d)", fn, TD, TE, D, E);
    VASR_CHECK_ARG(M >= 0 && ldg >= E && ldx >= D && ldo >= D && ldg % 4 == 0,
                   "%s: bad shape M=%d ldg=%lld ldx=%lld ldo=%lld", fn, M, (long long)ldg, (long long)ldx,
                   (long long)ldo);
    VASR_CHECK_ARG(((reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(wo) | reinterpret_cast<uintptr_t>(w1) |
                     reinterpret_cast<uintptr_t>(w2)) & 15) == 0,
                   "%s: g and the weight planes must be 16-byte aligned", fn);
    return VASR_OK;
}

}  // namespace
}  // namespace vasr

VASR_API int64_t vasr_pack_weights16_bf16_elems(int N, int K) {
    if (N <= 0 || K <= 0) return 0;
    return (int64_t)((N + 15) / 16 * 16) * ((K + 31) / 32 * 32);
}

VASR_API int vasr_pack_weights16_bf16(const uint16_t* W, int64_t ldw, int N, int K, uint16_t* out, void* stream) {
    using namespace vasr;
    VASR_CHECK_ARG(W && out, "vasr_pack_weights16_bf16: null pointer");
    VASR_CHECK_ARG(N > 0 && K > 0 && ldw >= K, "vasr_pack_weights16_bf16: bad shape N=%d K=%d", N, K);
    VASR_CHECK_ARG((reinterpret_cast<uintptr_t>(out) & 15) == 0, "vasr_pack_weights16_bf16: out must be 16-B aligned");
    const int Kp = (K + 31) / 32 * 32;
    const int64_t n = (int64_t)((N + 15) / 16 * 16) * (Kp / 8);
    hipLaunchKernelGGL(pack_weights16_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), W,
                       ldw, N, K, Kp, out);
    return launch_status("vasr_pack_weights16_bf16");
}

VASR_API int vasr_ssm_block_tail_bf16(const float* g, int64_t ldg, const float* x, int64_t ldx, const uint16_t* wo16,
                                      const float* ln_w, const float* ln_b, float ln_eps, const uint16_t* w1_16,
                                      const float* b1, const uint16_t* w2_16, const float* b2, float* out, int64_t ldo,
                                      int M, int D, int E, void* stream) {
    using namespace vasr;
    if (int rc = tail_args(g, ldg, x, ldx, wo16, ln_w, ln_b, w1_16, b1, w2_16, b2, out, ldo, M, D, E,
                           "vasr_ssm_block_tail_bf16"))
        return rc;
    if (M == 0) return VASR_OK;
    const TailParams p{g, ldg, x, ldx, wo16, ln_w, ln_b, ln_eps, w1_16, b1, w2_16, b2, out, ldo, M};
    launch_tail<1>(p, as_stream(stream));
    return launch_status("vasr_ssm_block_tail_bf16");
}

VASR_API int64_t vasr_split_weights16_elems(int N, int K) {
    if (N <= 0 || K <= 0) return 0;
    return 3 * (int64_t)((N + 15) / 16 * 16) * ((K + 31) / 32 * 32);
}

VASR_API int vasr_split_weights16_bf16x3(const float* W, int64_t ldw, int N, int K, uint16_t* out, void* stream) {
    using namespace vasr;
    VASR_CHECK_ARG(W && out, "vasr_split_weights16_bf16x3: null pointer");
    VASR_CHECK_ARG(N > 0 && K > 0 && ldw >= K, "vasr_split_weights16_bf16x3: bad shape N=%d K=%d", N, K);
    VASR_CHECK_ARG((reinterpret_cast<uintptr_t>(out) & 15) == 0, "vasr_split_weights16_bf16x3: out must be 16-B aligned");
    const int Kp = (K + 31) / 32 * 32;
    const int64_t n = (int64_t)((N + 15) / 16 * 16) * (Kp / 8);
    hipLaunchKernelGGL(split_weights16_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), W, ldw,
                       N, K, Kp, out);
    return launch_status("vasr_split_weights16_bf16x3");
}

VASR_API int vasr_ssm_block_tail_f32(const float* g, int64_t ldg, const float* x, int64_t ldx, const uint16_t* wo16,
                                     const float* ln_w, const float* ln_b, float ln_eps, const uint16_t* w1_16,
                                     const float* b1, const uint16_t* w2_16, const float* b2, float* out, int64_t ldo,
                                     int M, int D, int E, void* stream) {
    using namespace vasr;
    if (int rc = tail_args(g, ldg, x, ldx, wo16, ln_w, ln_b, w1_16, b1, w2_16, b2, out, ldo, M, D, E,
                           "vasr_ssm_block_tail_f32"))
        return rc;
    if (M == 0) return VASR_OK;
    const TailParams p{g, ldg, x, ldx, wo16, ln_w, ln_b, ln_eps, w1_16, b1, w2_16, b2, out, ldo, M};
    launch_tail<3>(p, as_stream(stream));
    return launch_status("vasr_ssm_block_tail_f32");
}

VASR_API int vasr_ssm_block_tail_gated_f32(const float* yd, int64_t ldy, const float* u, int64_t ldu, const uint16_t* wz,
                                           int mode, const float* x, int64_t ldx, const uint16_t* wo16,
                                           const float* ln_w, const float* ln_b, float ln_eps, const uint16_t* w1_16,
                                           const float* b1, const uint16_t* w2_16, const float* b2, float* out,
                                           int64_t ldo, int M, int D, int E, void* stream) {
    using namespace vasr;
    if (int rc = tail_args(yd, ldy, x, ldx, wo16, ln_w, ln_b, w1_16, b1, w2_16, b2, out, ldo, M, D, E,
                           "vasr_ssm_block_tail_gated_f32"))
        return rc;
    VASR_CHECK_ARG(u && wz && ldu >= D && ldu % 4 == 0 && (reinterpret_cast<uintptr_t>(u) & 15) == 0 &&
                       (reinterpret_cast<uintptr_t>(wz) & 15) == 0,
                   "vasr_ssm_block_tail_gated_f32: u (16-B aligned rows, ldu >= D, ldu %% 4 == 0) and wz needed");
    VASR_CHECK_ARG(mode == 0 || mode == 2, "vasr_ssm_block_tail_gated_f32: mode must be 0 or 2 (the scan's gate)");
    if (M == 0) return VASR_OK;
    const TailParams p{yd, ldy, x, ldx, wo16, ln_w, ln_b, ln_eps, w1_16, b1, w2_16, b2, out, ldo, M};
    const GateParams gp{yd, ldy, u, ldu, wz};
    const dim3 grid((unsigned)((M + 31) / 32)), block(768);
    if (mode == 2) hipLaunchKernelGGL((ssm_tail_gated_kernel<2, 3>), grid, block, 0, as_stream(stream), p, gp);
    else hipLaunchKernelGGL((ssm_tail_gated_kernel<0, 3>), grid, block, 0, as_stream(stream), p, gp);
    return launch_status("vasr_ssm_block_tail_gated_f32");
}

#ifdef VASR_TAIL_STAMPS
VASR_API int vasr_diag_tail_stamps(void* buf) {  // diagnostic builds only
    return hipMemcpyToSymbol(HIP_SYMBOL(vasr::g_tail_stamps), &buf, sizeof(buf)) == hipSuccess ? VASR_OK : VASR_EINVAL;
}
#endif

VASR_API int vasr_ssm_block_tail_gated_bf16(const float* yd, int64_t ldy, const float* u, int64_t ldu, const uint16_t* wz,
                                            int mode, const float* x, int64_t ldx, const uint16_t* wo16,
                                            const float* ln_w, const float* ln_b, float ln_eps, const uint16_t* w1_16,
                                            const float* b1, const uint16_t* w2_16, const float* b2, float* out,
                                            int64_t ldo, int M, int D, int E, void* stream) {
    using namespace vasr;
    if (int rc = tail_args(yd, ldy, x, ldx, wo16, ln_w, ln_b, w1_16, b1, w2_16, b2, out, ldo, M, D, E,
                           "vasr_ssm_block_tail_gated_bf16"))
        return rc;
    VASR_CHECK_ARG(u && wz && ldu >= D && ldu % 4 == 0 && (reinterpret_cast<uintptr_t>(u) & 15) == 0 &&
                       (reinterpret_cast<uintptr_t>(wz) & 15) == 0,
                   "vasr_ssm_block_tail_gated_bf16: u (16-B aligned rows, ldu >= D, ldu %% 4 == 0) and wz needed");
    VASR_CHECK_ARG(mode == 0 || mode == 2, "vasr_ssm_block_tail_gated_bf16: mode must be 0 or 2 (the scan's gate)");
    if (M == 0) return VASR_OK;
    const TailParams p{yd, ldy, x, ldx, wo16, ln_w, ln_b, ln_eps, w1_16, b1, w2_16, b2, out, ldo, M};
    const GateParams gp{yd, ldy, u, ldu, wz};
    const dim3 grid((unsigned)((M + 31) / 32)), block(768);
    if (mode == 2) hipLaunchKernelGGL((ssm_tail_gated_kernel<2, 1>), grid, block, 0, as_stream(stream), p, gp);
    else hipLaunchKernelGGL((ssm_tail_gated_kernel<0, 1>), grid, block, 0, as_stream(stream), p, gp);
    return launch_status("vasr_ssm_block_tail_gated_bf16");
}
