// Selective-SSM scan + D skip + SiLU gate (reference velocity_asr/ssm.py:119-129).
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
// Work decomposition (MI355X): one workgroup = (utterance b, DPB consecutive channels d).
// Within a wave, G = N/4 lanes share one channel and each lane owns 4 state indices n, so
// the y[t] = sum_n h C contraction is 4 FMAs + log2(G) DPP adds (quad_perm / row mirrors,
// no LDS).  Time is processed in 16-step chunks: the chunk's x, dt, z, B, C slices are
// staged to LDS (double-buffered with a register prefetch of the next chunk), the four
// in-chunk stack levels are compile-time registers (the push/merge pattern of step i is a
// constant), and the upper levels (chunk-sized blocks) are merged once per chunk.  The
// gated outputs of a chunk are written as coalesced row segments from an LDS tile.
#include "vasr_internal.h"

namespace vasr {
namespace {

constexpr int T = 16;    // time steps per chunk
constexpr int NPL = 4;   // state indices per lane

constexpr int ctz_c(int v) { return v & 1 ? 0 : 1 + ctz_c(v >> 1); }
constexpr int trailing_ones(int v) { return v & 1 ? 1 + trailing_ones(v >> 1) : 0; }
// Level of the stack entry right below a new block at level j after step i (count i+1),
// or -1 when the entry below is the upper (chunk-level) stack.
constexpr int below_level(int i, int j) {
    int rest = (i + 1) >> (j + 1);
    return rest == 0 || j + 1 >= 4 ? -1 : (j + 1 + ctz_c(rest) < 4 ? j + 1 + ctz_c(rest) : -1);
}

template <int CTRL>
__device__ __forceinline__ float dpp_mov(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}

// Sum over aligned groups of G lanes (G in {4, 8, 16}) with DPP; every lane gets the sum.
template <int G>
__device__ __forceinline__ float group_sum(float v) {
    v += dpp_mov<0xB1>(v);                          // quad_perm [1,0,3,2]
    v += dpp_mov<0x4E>(v);                          // quad_perm [2,3,0,1]
    if constexpr (G >= 8) v += dpp_mov<0x141>(v);   // row_half_mirror
    if constexpr (G >= 16) v += dpp_mov<0x140>(v);  // row_mirror
    return v;
}

template <int MAXUP>
struct TreeState {
    float la[4][NPL], lb[4][NPL], ca[4][NPL], cb[4][NPL];  // in-chunk levels 0..3
    float ula[MAXUP][NPL], ulb[MAXUP][NPL];                // chunk-level blocks
    float pa[NPL], pb[NPL];                                // prefix after the upper stack
};

struct StepIn {
    float x, dt;
    float Bn[NPL], Cn[NPL];
};

// One push of the streaming tree scan at in-chunk step I.  Returns the partial
// y contribution (sum over this lane's n of h[t] * C[t]).
template <int I, int MAXUP>
__device__ __forceinline__ float tree_step(TreeState<MAXUP>& s, const StepIn& in, const float (&A2)[NPL],
                                           float (&chunk_a)[NPL], float (&chunk_b)[NPL]) {
#pragma clang fp contract(off)
    float part = 0.f;
#pragma unroll
    for (int n = 0; n < NPL; ++n) {
        float hv;
        if constexpr (I == 0) hv = s.pb[n];
        else hv = s.cb[ctz_c(I)][n];
        part = __builtin_fmaf(hv, in.Cn[n], part);
    }
    constexpr int J = trailing_ones(I);
#pragma unroll
    for (int n = 0; n < NPL; ++n) {
        float cur_a = __builtin_amdgcn_exp2f(in.dt * A2[n]);
        const float dB = in.dt * in.Bn[n];
        float cur_b = in.x * dB;
#pragma unroll
        for (int k = 0; k < J; ++k) {  // up-sweep: (a_r, b_r) <- (a_r a_l, a_r b_l + b_r)
            cur_b = cur_a * s.lb[k][n] + cur_b;
            cur_a = cur_a * s.la[k][n];
        }
        if constexpr (J < 4) {
            s.la[J][n] = cur_a;
            s.lb[J][n] = cur_b;
            constexpr int BL = below_level(I, J);
            float Pa, Pb;
            if constexpr (BL >= 0) {
                Pa = s.ca[BL][n];
                Pb = s.cb[BL][n];
            } else {
                Pa = s.pa[n];
                Pb = s.pb[n];
            }
            const float c_a = Pa * cur_a;  // down-sweep: a_r <- a_p a_l ; b_r <- a_r b_l + b_p
            s.ca[J][n] = c_a;
            s.cb[J][n] = c_a * cur_b + Pb;
        } else {
            chunk_a[n] = cur_a;
            chunk_b[n] = cur_b;
        }
    }
    return part;
}

template <int MAXUP>
__device__ __forceinline__ void merge_upper(TreeState<MAXUP>& s, float (&chunk_a)[NPL], float (&chunk_b)[NPL],
                                            int cc) {
#pragma clang fp contract(off)
    const int j = __builtin_ctz(~cc);
#pragma unroll
    for (int n = 0; n < NPL; ++n) {
        float cur_a = chunk_a[n], cur_b = chunk_b[n];
#pragma unroll
        for (int u = 0; u < MAXUP; ++u) {
            if (u < j) {
                cur_b = cur_a * s.ulb[u][n] + cur_b;
                cur_a = cur_a * s.ula[u][n];
            }
        }
#pragma unroll
        for (int u = 0; u < MAXUP; ++u) {
            if (u == j) {
                s.ula[u][n] = cur_a;
                s.ulb[u][n] = cur_b;
            }
        }
        // Prefix after the upper stack, rebuilt bottom-up with the stream form's (1, 0) start:
        // identical float operations to carrying (ca, cb) per upper entry.
        const int cc1 = cc + 1;
        float pa = 1.0f, pb = 0.0f;
#pragma unroll
        for (int u = MAXUP - 1; u >= 0; --u) {
            if ((cc1 >> u) & 1) {
                pa = pa * s.ula[u][n];
                pb = pa * s.ulb[u][n] + pb;
            }
        }
        s.pa[n] = pa;
        s.pb[n] = pb;
    }
}

template <int I, int MAXUP, int G>
struct TreeChunk {
    __device__ __forceinline__ static void run(TreeState<MAXUP>& s, const float (&A2)[NPL], int nvalid,
                                               const float* xs, const float* dts, const float* bcs, float* yt,
                                               int dl, int g, int DPB, int N, float (&ca)[NPL], float (&cb)[NPL]) {
        if (I < nvalid) {
            StepIn in;
            in.x = xs[I * DPB + dl];
            in.dt = dts[I * DPB + dl];
            const float4 bv = *reinterpret_cast<const float4*>(bcs + I * 2 * N + g * NPL);
            const float4 cv = *reinterpret_cast<const float4*>(bcs + I * 2 * N + N + g * NPL);
            in.Bn[0] = bv.x; in.Bn[1] = bv.y; in.Bn[2] = bv.z; in.Bn[3] = bv.w;
            in.Cn[0] = cv.x; in.Cn[1] = cv.y; in.Cn[2] = cv.z; in.Cn[3] = cv.w;
            float part = tree_step<I, MAXUP>(s, in, A2, ca, cb);
            part = group_sum<G>(part);
            if (g == 0) yt[I * DPB + dl] = part;
            TreeChunk<I + 1, MAXUP, G>::run(s, A2, nvalid, xs, dts, bcs, yt, dl, g, DPB, N, ca, cb);
        }
    }
};
template <int MAXUP, int G>
struct TreeChunk<T, MAXUP, G> {
    __device__ __forceinline__ static void run(TreeState<MAXUP>&, const float (&)[NPL], int, const float*,
                                               const float*, const float*, float*, int, int, int, int,
                                               float (&)[NPL], float (&)[NPL]) {}
};

template <int N, int MODE, int MAXUP>
__global__ __launch_bounds__(256) void ssm_scan_kernel(const float* __restrict__ xz, int64_t ld_xz,
                                                       const float* __restrict__ dt, int64_t ld_dt,
                                                       const float* __restrict__ bc, int64_t ld_bc,
                                                       const float* __restrict__ A2g, const float* __restrict__ Dg,
                                                       float* __restrict__ out, int64_t ld_out, int L, int Di) {
#pragma clang fp contract(off)
    constexpr int G = N / NPL;       // lanes per channel
    constexpr int DPW = 64 / G;      // channels per wave
    constexpr int NW = 4;            // waves per block
    constexpr int DPB = NW * DPW;    // channels per block
    constexpr int MAXDPB = DPB;
    // LDS: two staging buffers {x, dt, z: T x DPB; bc: T x 2N} + y tile T x DPB
    constexpr int BUF = 3 * T * MAXDPB + T * 2 * N;
    __shared__ __attribute__((aligned(16))) float smem[2 * BUF + T * MAXDPB];
    float* ytile = smem + 2 * BUF;

    const int b = blockIdx.y;
    const int d0 = blockIdx.x * DPB;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int g = lane % G;
    const int dl = wave * DPW + lane / G;

    float A2[NPL];
#pragma unroll
    for (int j = 0; j < NPL; ++j) A2[j] = A2g[g * NPL + j];

    const int64_t row0 = (int64_t)b * L;
    constexpr int q_xzd = T * DPB / 4;      // float4 per x/z/dt slab
    constexpr int q_bc = T * 2 * N / 4;
    constexpr int q_total = 3 * q_xzd + q_bc;
    constexpr int nthreads = 64 * NW;
    constexpr int MAXQ = (q_total + nthreads - 1) / nthreads;
    float4 pre[MAXQ];

    auto load_chunk = [&](int t0) {
#pragma unroll
        for (int k = 0; k < MAXQ; ++k) {
            const int q = tid + k * nthreads;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (q < q_total) {
                if (q < 3 * q_xzd) {
                    const int arr = q / q_xzd, rem = q - arr * q_xzd;
                    const int t = rem / (DPB / 4), c = (rem - t * (DPB / 4)) * 4;
                    if (t0 + t < L) {
                        const int64_t row = row0 + t0 + t;
                        const float* src = arr == 0 ? xz + row * ld_xz + d0 + c
                                         : arr == 1 ? dt + row * ld_dt + d0 + c
                                                    : xz + row * ld_xz + Di + d0 + c;
                        v = *reinterpret_cast<const float4*>(src);
                    }
                } else {
                    const int rem = q - 3 * q_xzd;
                    const int t = rem / (2 * N / 4), c = (rem - t * (2 * N / 4)) * 4;
                    if (t0 + t < L) v = *reinterpret_cast<const float4*>(bc + (row0 + t0 + t) * ld_bc + c);
                }
            }
            pre[k] = v;
        }
    };
    auto store_chunk = [&](float* buf) {
#pragma unroll
        for (int k = 0; k < MAXQ; ++k) {
            const int q = tid + k * nthreads;
            if (q < q_total) {
                float* dst;
                if (q < 3 * q_xzd) {
                    const int arr = q / q_xzd, rem = q - arr * q_xzd;
                    const int t = rem / (DPB / 4), c = (rem - t * (DPB / 4)) * 4;
                    dst = buf + arr * T * MAXDPB + t * DPB + c;
                } else {
                    const int rem = q - 3 * q_xzd;
                    dst = buf + 3 * T * MAXDPB + rem * 4;
                }
                *reinterpret_cast<float4*>(dst) = pre[k];
            }
        }
    };

    const int nchunks = (L + T - 1) / T;
    load_chunk(0);
    store_chunk(smem);
    __syncthreads();

    TreeState<MAXUP> st;
    float h[NPL];
#pragma unroll
    for (int n = 0; n < NPL; ++n) {
        st.pa[n] = 1.0f;
        st.pb[n] = 0.0f;
        h[n] = 0.0f;
    }

    for (int c = 0; c < nchunks; ++c) {
        float* buf = smem + (c & 1) * BUF;
        const float* xs = buf;
        const float* dts = buf + T * MAXDPB;
        const float* zs = buf + 2 * T * MAXDPB;
        const float* bcs = buf + 3 * T * MAXDPB;
        const int t0 = c * T;
        const int nvalid = min(T, L - t0);
        if (c + 1 < nchunks) load_chunk(t0 + T);

        if constexpr (MODE == 0) {
            float cha[NPL], chb[NPL];
            TreeChunk<0, MAXUP, G>::run(st, A2, nvalid, xs, dts, bcs, ytile, dl, g, DPB, N, cha, chb);
            if (c + 1 < nchunks) merge_upper<MAXUP>(st, cha, chb, c);
        } else {
            for (int i = 0; i < nvalid; ++i) {
                const float xv = xs[i * DPB + dl];
                const float dv = dts[i * DPB + dl];
                const float4 bv = *reinterpret_cast<const float4*>(bcs + i * 2 * N + g * NPL);
                const float4 cv = *reinterpret_cast<const float4*>(bcs + i * 2 * N + N + g * NPL);
                const float Bn[4] = {bv.x, bv.y, bv.z, bv.w};
                const float Cn[4] = {cv.x, cv.y, cv.z, cv.w};
                float part = 0.f;
#pragma unroll
                for (int n = 0; n < NPL; ++n) {
                    const float dA = __builtin_amdgcn_exp2f(dv * A2[n]);
                    const float dB = dv * Bn[n];
                    h[n] = dA * h[n] + xv * dB;
                    part = __builtin_fmaf(h[n], Cn[n], part);
                }
                part = group_sum<G>(part);
                if (g == 0) ytile[i * DPB + dl] = part;
            }
        }
        __syncthreads();
        // gated output of this chunk: (y + x D) * silu(z), coalesced along d
        for (int idx = tid; idx < T * DPB; idx += nthreads) {
            const int t = idx / DPB, d = idx - t * DPB;
            if (t < nvalid) {
                const float xv = xs[t * DPB + d];
                const float zv = zs[t * DPB + d];
                const float y = ytile[t * DPB + d] + xv * Dg[d0 + d];
                const float silu = zv / (1.0f + expf(-zv));
                out[(row0 + t0 + t) * ld_out + d0 + d] = y * silu;
            }
        }
        if (c + 1 < nchunks) store_chunk(smem + ((c + 1) & 1) * BUF);
        __syncthreads();
    }
}

template <int N, int MODE>
int launch_n(const float* xz, int64_t ld_xz, const float* dt, int64_t ld_dt, const float* bc, int64_t ld_bc,
             const float* A2, const float* D, float* out, int64_t ld_out, int B, int L, int Di, hipStream_t s) {
    constexpr int G = N / NPL;
    constexpr int DPW = 64 / G;
    constexpr int nw = 4;
    if (Di % (nw * DPW) != 0) {
        set_error("vasr_ssm_scan_f32: Di=%d must be a multiple of %d for N=%d", Di, nw * DPW, N);
        return VASR_EUNSUPPORTED;
    }
    dim3 grid(Di / (nw * DPW), B);
    dim3 block(64 * nw);
    const int nchunks = (L + T - 1) / T;
    if (MODE == 1 || nchunks <= 32)
        hipLaunchKernelGGL((ssm_scan_kernel<N, MODE, 5>), grid, block, 0, s, xz, ld_xz, dt, ld_dt, bc, ld_bc, A2, D,
                           out, ld_out, L, Di);
    else if (nchunks <= 128)
        hipLaunchKernelGGL((ssm_scan_kernel<N, MODE, 7>), grid, block, 0, s, xz, ld_xz, dt, ld_dt, bc, ld_bc, A2, D,
                           out, ld_out, L, Di);
    else
        hipLaunchKernelGGL((ssm_scan_kernel<N, MODE, 9>), grid, block, 0, s, xz, ld_xz, dt, ld_dt, bc, ld_bc, A2, D,
                           out, ld_out, L, Di);
    return launch_status("vasr_ssm_scan_f32");
}

}  // namespace
}  // namespace vasr

VASR_API int vasr_ssm_scan_f32(const float* xz, int64_t ld_xz, const float* dt, int64_t ld_dt, const float* bc,
                               int64_t ld_bc, const float* A2, const float* D, float* out, int64_t ld_out, int B,
                               int L, int Di, int N, int mode, void* stream) {
    using namespace vasr;
    VASR_CHECK_ARG(xz && dt && bc && A2 && D && out, "vasr_ssm_scan_f32: null pointer");
    VASR_CHECK_ARG(mode == 0 || mode == 1, "vasr_ssm_scan_f32: mode must be 0 (tree) or 1 (recurrence)");
    VASR_CHECK_ARG(B >= 0 && L >= 0 && L <= 8192 && Di > 0, "vasr_ssm_scan_f32: bad shape B=%d L=%d Di=%d", B, L, Di);
    VASR_CHECK_ARG(ld_xz % 4 == 0 && ld_dt % 4 == 0 && ld_bc % 4 == 0 && Di % 4 == 0,
                   "vasr_ssm_scan_f32: leading dims and Di must be multiples of 4");
    VASR_CHECK_ARG(ld_xz >= 2 * Di && ld_dt >= Di && ld_bc >= 2 * N && ld_out >= Di,
                   "vasr_ssm_scan_f32: leading dims too small");
    VASR_CHECK_ARG(((reinterpret_cast<uintptr_t>(xz) | reinterpret_cast<uintptr_t>(dt) |
                     reinterpret_cast<uintptr_t>(bc)) & 15) == 0,
                   "vasr_ssm_scan_f32: inputs must be 16-byte aligned");
    if (B == 0 || L == 0) return VASR_OK;
    hipStream_t s = as_stream(stream);
    switch (N) {
        case 16: return mode == 0 ? launch_n<16, 0>(xz, ld_xz, dt, ld_dt, bc, ld_bc, A2, D, out, ld_out, B, L, Di, s)
                                  : launch_n<16, 1>(xz, ld_xz, dt, ld_dt, bc, ld_bc, A2, D, out, ld_out, B, L, Di, s);
        case 32: return mode == 0 ? launch_n<32, 0>(xz, ld_xz, dt, ld_dt, bc, ld_bc, A2, D, out, ld_out, B, L, Di, s)
                                  : launch_n<32, 1>(xz, ld_xz, dt, ld_dt, bc, ld_bc, A2, D, out, ld_out, B, L, Di, s);
        case 64: return mode == 0 ? launch_n<64, 0>(xz, ld_xz, dt, ld_dt, bc, ld_bc, A2, D, out, ld_out, B, L, Di, s)
                                  : launch_n<64, 1>(xz, ld_xz, dt, ld_dt, bc, ld_bc, A2, D, out, ld_out, B, L, Di, s);
        default: set_error("vasr_ssm_scan_f32: state dim N=%d not supported (16, 32, 64)", N); return VASR_EUNSUPPORTED;
    }
}
