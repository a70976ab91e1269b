// The head of an SSMBlock as ONE kernel (reference ssm.py:404-414 and SelectiveSSM.forward
// ssm.py:105-113):
//
//     u      = causal_dwconv_k4(LayerNorm_1(x))          (:407-414; conv pad 3, first L kept)
//     xz     = in_proj(u)            -> HBM [x_p | z]     (:105-106, no bias)
//     x_dt   = [x_proj; dt_proj](x_p) + [0; b_dt]         (:109-113)
//              softplus on the dt columns -> HBM [B | C | dt]
//
// for d_model 192, d_inner 384 and 2N + d_inner = 512 (N = 64: the local blocks).  The unfused
// form is three launches that write u (768 B per token) and re-read it, and re-read x_p
// (1536 B per token) for the second product.  Here one workgroup owns 32 token rows: LN1 of
// the rows and the 3 history rows of their causal window (recomputed, not re-read: rows of the
// previous utterance or before t = 0 are masked, as the conv's zero padding), the conv, then u
// as the A operand of in_proj and x_p (in_proj's first 384 columns, also written to HBM for the
// scan) as the A operand of the second product, both as bf16 planes in LDS.
//
// Arithmetic: LN1 + conv with the float operations of vasr_ln_dwconv_f32; the products are the
// split-bf16 fp32 GEMM (NP = 3) or the bf16 model's one-plane GEMM (NP = 1) on
// v_mfma_f32_16x16x32_bf16; bias + softplus as the x_dt GEMM epilogue (softplus20_fast).
// Weights stream global -> VGPRs from the 16x16x32 fragment layout, PD steps ahead: in_proj is
// 4 column quarters x 6 k-steps, the second product 3 column groups (192, 192, 128 columns) x
// 12 k-steps: 60 steps, one stream.
#include "ssm_fused.h"

namespace vasr {
namespace {

using namespace fused;

constexpr int HN = 2 * TE;         // in_proj width (768)
constexpr int HX = 512;            // [B | C | dt] width (2N + d_inner, N = 64)
constexpr int NS1 = 24;            // in_proj steps: 4 quarters x 6
constexpr int NSTEPS = NS1 + 36;   // + 3 groups x 12
constexpr int KC = 4;              // conv taps

template <int NP>
constexpr int hpd_of() { return NP == 3 ? 3 : 6; }

struct HeadParams {
    const float* x;
    int64_t ldx;
    const float* ln_w;
    const float* ln_b;
    float ln_eps;
    const float* conv_w;  // (192, 4)
    const float* conv_b;
    const uint16_t* win;  // in_proj (768 x 192) in the 16x16x32 fragment layout
    const uint16_t* wxd;  // [x_proj; dt_proj] (512 x 384)
    const float* bxd;     // (512) bias, zero on the B / C columns
    int n_sp;             // softplus from this column on (2N)
    float* xz;            // (M, 768)
    int64_t ldxz;
    float* xdt;           // (M, 512)
    int64_t ldxdt;
    int M, L;
};

template <int NP>
struct HeadCtx {
    static constexpr int PD = hpd_of<NP>();
    static constexpr int RING = PD + 1;
    const HeadParams& P;
    char* R;  // 384-wide planes: LN scratch, then x_p
    char* H;  // 192-wide planes: u
    int lane, wave, r, q, m0;
    floatx4 acc[2][3];
    bf16x8 w[RING][3][NP];
};

// column tiles of step S for this wave: 3 (in_proj quarters, the first two x_dt groups) or 2
// (the last x_dt group of 128 columns)
template <int S>
constexpr int tiles_of() { return (S >= NS1 && (S - NS1) / 12 == 2) ? 2 : 3; }

template <int S>
__device__ __forceinline__ int tile_of(int wave, int t) {
    if constexpr (S < NS1) return 12 * (S / 6) + 3 * wave + t;
    else if constexpr ((S - NS1) / 12 < 2) return 12 * ((S - NS1) / 12) + 3 * wave + t;
    else return 24 + 2 * wave + t;
}

template <int S, int NP>
__device__ __forceinline__ void hload_w(HeadCtx<NP>& c) {
    const uint16_t* W = S < NS1 ? c.P.win : c.P.wxd;
    constexpr int KS = S < NS1 ? TD / 32 : TE / 32;
    constexpr int ks = S < NS1 ? S % 6 : (S - NS1) % 12;
#pragma unroll
    for (int t = 0; t < tiles_of<S>(); ++t) {
        const int nt = tile_of<S>(c.wave, t);
#pragma unroll
        for (int pl = 0; pl < NP; ++pl)
            c.w[S % HeadCtx<NP>::RING][t][pl] =
                *reinterpret_cast<const bf16x8*>(W + ((int64_t)(nt * KS + ks) * NP + pl) * 512 + c.lane * 8);
    }
}

template <int S, int NP>
__device__ __forceinline__ void hload_first(HeadCtx<NP>& c) {
    hload_w<S, NP>(c);
    if constexpr (S + 1 < HeadCtx<NP>::PD) hload_first<S + 1, NP>(c);
}

template <int S, int NP>
__device__ __forceinline__ void head_step(HeadCtx<NP>& c) {
    constexpr int PD = HeadCtx<NP>::PD;
    if constexpr (S + PD < NSTEPS) hload_w<S + PD, NP>(c);
    __builtin_amdgcn_sched_barrier(0);  // keep the prefetch here (see ssm_tail.hip)
    constexpr int NT = tiles_of<S>();
    bf16x8 a[2][NP];
#pragma unroll
    for (int tm = 0; tm < 2; ++tm) {
        if constexpr (S < NS1) read_a<NP, TD>(c.H, 16 * tm + c.r, S % 6, c.q, a[tm]);
        else read_a<NP, TE>(c.R, 16 * tm + c.r, (S - NS1) % 12, c.q, a[tm]);
    }
#pragma unroll
    for (int tm = 0; tm < 2; ++tm)
#pragma unroll
        for (int t = 0; t < NT; ++t) c.acc[tm][t] = mac_tile<NP>(a[tm], c.w[S % HeadCtx<NP>::RING][t], c.acc[tm][t]);

    if constexpr (S < NS1 && S % 6 == 5) {
        // in_proj column quarter done: xz to HBM; x_p (quarters 0, 1) also as planes in R
        constexpr int qq = S / 6;
#pragma unroll
        for (int tm = 0; tm < 2; ++tm)
#pragma unroll
            for (int t = 0; t < 3; ++t) {
                const int col = 192 * qq + 16 * (3 * c.wave + t) + c.r;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int rl = 16 * tm + 4 * c.q + i;
                    const float v = c.acc[tm][t][i];
                    if (c.m0 + rl < c.P.M) c.P.xz[(int64_t)(c.m0 + rl) * c.P.ldxz + col] = v;
                    if constexpr (qq < 2) split_store<NP>(c.R, PLANE_E, poff<TE>(rl, col), v);
                }
                c.acc[tm][t] = floatx4{0.f, 0.f, 0.f, 0.f};
            }
        if constexpr (S == NS1 - 1) lds_barrier();  // x_p planes complete before the second product
    } else if constexpr (S >= NS1 && (S - NS1) % 12 == 11) {
        // [x_proj; dt_proj] column group done: + bias, softplus on the dt columns -> HBM
        constexpr int gg = (S - NS1) / 12;
#pragma unroll
        for (int tm = 0; tm < 2; ++tm)
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const int col = 16 * tile_of<S>(c.wave, t) + c.r;
                const float bv = c.P.bxd[col];
                const bool sp = col >= c.P.n_sp;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int rl = 16 * tm + 4 * c.q + i;
                    float v = c.acc[tm][t][i] + bv;
                    if (sp) v = softplus20_fast(v);
                    if (c.m0 + rl < c.P.M) c.P.xdt[(int64_t)(c.m0 + rl) * c.P.ldxdt + col] = v;
                }
                c.acc[tm][t] = floatx4{0.f, 0.f, 0.f, 0.f};
            }
        (void)gg;
    }
    if constexpr (S + 1 < NSTEPS) head_step<S + 1, NP>(c);
}

template <int NP>
__global__ __launch_bounds__(256, 1) void ssm_head_kernel(HeadParams P) {
    __shared__ __attribute__((aligned(16))) char R[NP * PLANE_E > (TBM + KC - 1) * TD * 4 ? NP * PLANE_E
                                                                                        : (TBM + KC - 1) * TD * 4];
    __shared__ __attribute__((aligned(16))) char H[NP * PLANE_D];
    HeadCtx<NP> c{P, R, H};
    c.lane = threadIdx.x & 63;
    c.wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    c.r = c.lane & 15;
    c.q = c.lane >> 4;
    c.m0 = blockIdx.x * TBM;
    hload_first<0, NP>(c);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int tm = 0; tm < 2; ++tm)
#pragma unroll
        for (int t = 0; t < 3; ++t) c.acc[tm][t] = floatx4{0.f, 0.f, 0.f, 0.f};

    // LN1 of rows m0 - 3 .. m0 + 31 into an fp32 scratch [35][192] in R, one wave per row,
    // vasr_ln_dwconv_f32's operations
    float* ln = reinterpret_cast<float*>(R);
    float lw[3], lb[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        lw[i] = P.ln_w[c.lane + 64 * i];
        lb[i] = P.ln_b[c.lane + 64 * i];
    }
    constexpr int NROWS = TBM + KC - 1;
    for (int j = c.wave; j < NROWS; j += TWAVES) {
        const int gm = min(max(c.m0 - (KC - 1) + j, 0), P.M - 1);
        float v[3];
        float sum = 0.f;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            v[i] = P.x[(int64_t)gm * P.ldx + c.lane + 64 * i];
            sum += v[i];
        }
        const float mean = wave_sum(sum) / (float)TD;
        float qs = 0.f;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const float d = v[i] - mean;
            qs += d * d;
        }
        const float rstd = 1.0f / sqrtf(wave_sum(qs) / (float)TD + P.ln_eps);
#pragma unroll
        for (int i = 0; i < 3; ++i) ln[j * TD + c.lane + 64 * i] = (v[i] - mean) * rstd * lw[i] + lb[i];
    }
    lds_barrier();
    // u = conv_b + sum_k w[k] LN[t - 3 + k] (rows of an earlier utterance / before t = 0 are the
    // conv's zero padding), 8 channels per thread-unit, split into H's planes
    for (int u = threadIdx.x; u < TBM * TD / 8; u += 256) {
        const int rl = u / (TD / 8), ch = u - rl * (TD / 8);
        const int gm = c.m0 + rl;
        const int t = gm % P.L;
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int col = 8 * ch + e;
            float acc = 0.f;
#pragma unroll
            for (int k = 0; k < KC; ++k) {
                const float lv = (t - (KC - 1) + k >= 0) ? ln[(rl + k) * TD + col] : 0.f;
                acc += lv * P.conv_w[col * KC + k];
            }
            o[e] = acc + P.conv_b[col];
        }
        split_store8<NP>(H, PLANE_D, rl * TD * 2 + ((ch ^ (rl & 7)) << 4), make_float4(o[0], o[1], o[2], o[3]),
                         make_float4(o[4], o[5], o[6], o[7]));
    }
    lds_barrier();  // u planes complete; the LN scratch in R is free for x_p
    head_step<0, NP>(c);
}

}  // namespace
}  // namespace vasr

VASR_API int vasr_ssm_block_head_f32(const float* x, int64_t ldx, const float* ln_w, const float* ln_b, float ln_eps,
                                     const float* conv_w, const float* conv_b, const uint16_t* win16,
                                     const uint16_t* wxd16, const float* bxd, int n_sp, float* xz, int64_t ldxz,
                                     float* xdt, int64_t ldxdt, int M, int L, int D, int Di, int Nx, int bf16,
                                     void* stream) {
    using namespace vasr;
    using namespace vasr::fused;
    VASR_CHECK_ARG(x && ln_w && ln_b && conv_w && conv_b && win16 && wxd16 && bxd && xz && xdt,
                   "vasr_ssm_block_head_f32: null pointer");
    VASR_CHECK_ARG(D == TD && Di == TE && Nx == HX && n_sp >= 0 && n_sp <= Nx,
                   "vasr_ssm_block_head_f32: built for d_model %d, d_inner %d, x_dt width %d (got %d, %d, %d)", TD, TE,
                   HX, D, Di, Nx);
    VASR_CHECK_ARG(M >= 0 && L > 0 && M % L == 0 && ldx >= D && ldxz >= 2 * Di && ldxdt >= Nx,
                   "vasr_ssm_block_head_f32: bad shape M=%d L=%d", M, L);
    VASR_CHECK_ARG(((reinterpret_cast<uintptr_t>(win16) | reinterpret_cast<uintptr_t>(wxd16)) & 15) == 0,
                   "vasr_ssm_block_head_f32: weight planes must be 16-byte aligned");
    if (M == 0) return VASR_OK;
    HeadParams p{x, ldx, ln_w, ln_b, ln_eps, conv_w, conv_b, win16, wxd16, bxd, n_sp, xz, ldxz, xdt, ldxdt, M, L};
    if (bf16)
        hipLaunchKernelGGL(ssm_head_kernel<1>, dim3((M + TBM - 1) / TBM), dim3(64 * TWAVES), 0, as_stream(stream), p);
    else
        hipLaunchKernelGGL(ssm_head_kernel<3>, dim3((M + TBM - 1) / TBM), dim3(64 * TWAVES), 0, as_stream(stream), p);
    return launch_status("vasr_ssm_block_head_f32");
}
