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
// Work decomposition (MI355X): one workgroup = (utterance b, DPB consecutive channels d),
// 4 waves.  G = N/4 lanes share one channel and each lane owns 4 state indices n, held as
// two float2 pairs so the state algebra issues as packed v_pk_mul/v_pk_add_f32 (two lanes'
// worth of fp32 per instruction: the f32 vector peak).  Per time step each lane leaves its
// partial y = sum_n h C in an LDS tile; the chunk's gated outputs are reduced and written
// from LDS as coalesced row segments.  Time runs in 16-step chunks: x, dt, z, B, C slices
// are staged to LDS (double-buffered, register prefetch of the next chunk); the four
// in-chunk stack levels are compile-time registers (step i's push/merge pattern is a
// constant, full chunks carry no per-step guards); chunk-sized blocks form the upper stack,
// merged once per chunk.  Blocks are remapped so all channel blocks of one utterance share
// an XCD (its 4 MiB L2 then serves the B/C slices and the 64-B row segments they share).
#include "vasr_internal.h"

namespace vasr {
namespace {

typedef __attribute__((address_space(3))) void lds_void;

#ifndef VASR_SCAN_ABLATE
#define VASR_SCAN_ABLATE 0  // diagnostic builds only (tools/scan_ablate.sh): 1 no exp,
#endif                      // 4 no B/C LDS reads, 8 no chunk staging after the first,
                            // 16 no tree update, 32 no gated-output pass
#ifndef VASR_SCAN_WAVES
#define VASR_SCAN_WAVES 3   // waves per SIMD the register allocator targets
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

constexpr int T = 16;    // time steps per chunk
constexpr int TP = T + 1;  // padded row of the per-channel partial-sum tile
constexpr int NPL = 4;   // state indices per lane (2 packed pairs)
constexpr int NP = NPL / 2;
constexpr int NW = 4;    // waves per block

constexpr int ctz_c(int v) { return v & 1 ? 0 : 1 + ctz_c(v >> 1); }
constexpr int trailing_ones(int v) { return v & 1 ? 1 + trailing_ones(v >> 1) : 0; }
// Level of the stack entry right below a new block at level j after step i (count i+1),
// or -1 when the entry below is the upper (chunk-level) stack.
constexpr int below_level(int i, int j) {
    return ((i + 1) >> (j + 1)) == 0 ? -1
           : (j + 1 + ctz_c((i + 1) >> (j + 1)) < 4 ? j + 1 + ctz_c((i + 1) >> (j + 1)) : -1);
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

template <int CTRL, int S>
__device__ __forceinline__ void butterfly_level(float (&v)[8], bool sel) {
    if constexpr (S >= 2) {
#pragma unroll
        for (int j = 0; j < S / 2; ++j) {
            const float lo = v[j], hi = v[j + S / 2];
            const float keep = sel ? hi : lo;
            const float send = sel ? lo : hi;
            v[j] = keep + dpp_mov<CTRL>(send);
        }
    } else {
        v[0] = v[0] + dpp_mov<CTRL>(v[0]);
    }
}

template <int G>
__device__ __forceinline__ void reduce_half(float (&v)[8], int g) {
    if constexpr (G == 16) {
        butterfly_level<0x140, 8>(v, (g >> 3) & 1);  // row_mirror: lane ^ 15
        butterfly_level<0x141, 4>(v, (g >> 2) & 1);  // row_half_mirror: lane ^ 7
        butterfly_level<0x4E, 2>(v, (g >> 1) & 1);   // quad_perm [2,3,0,1]: lane ^ 2
        butterfly_level<0xB1, 1>(v, false);          // quad_perm [1,0,3,2]: lane ^ 1
    } else if constexpr (G == 8) {
        butterfly_level<0x141, 8>(v, (g >> 2) & 1);
        butterfly_level<0x4E, 4>(v, (g >> 1) & 1);
        butterfly_level<0xB1, 2>(v, g & 1);
    } else {
        static_assert(G == 4, "G in {4, 8, 16}");
        butterfly_level<0x4E, 8>(v, (g >> 1) & 1);
        butterfly_level<0xB1, 4>(v, g & 1);
    }
}

// Reduce the partial sums of steps [8*HALF, 8*HALF + 8) and store them to the channel's row
// of the partial-sum tile ([DPB][TP] floats).
template <int G, int HALF>
__device__ __forceinline__ void flush_half(float (&yv)[T], float* yp, int dl, int g) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = yv[HALF * 8 + j];
    reduce_half<G>(v, g);
#pragma unroll
    for (int j = 0; j < HalfReduce<G>::SF; ++j) yp[dl * TP + HALF * 8 + HalfReduce<G>::step(j, g)] = v[j];
}

template <int MAXUP>
struct TreeState {
    f2 la[4][NP], lb[4][NP], ca[4][NP], cb[4][NP];  // in-chunk levels 0..3
    f2 ula[MAXUP][NP], ulb[MAXUP][NP];              // chunk-level blocks
    f2 pa[NP], pb[NP];                              // prefix after the upper stack
};

struct Smem {
    const float* xs;
    const float* dts;
    const float* bcs;
    float* yp;  // per-channel partial sums y[t] = sum_n h C: [DPB][TP]
};

// Per-step operands of one lane, read from the staged chunk one step ahead of use.
struct StepIn {
    float x, dt;
    float4 bv, cv;
};

template <int I, int N, int DPB>
__device__ __forceinline__ StepIn load_step(const Smem& sm, int dl, int g) {
    StepIn in;
    in.x = sm.xs[I * DPB + dl];
    in.dt = sm.dts[I * DPB + dl];
    if constexpr (VASR_SCAN_ABLATE & 4) {
        in.bv = make_float4(in.x, in.dt, in.x, in.dt);
        in.cv = make_float4(in.dt, in.x, in.dt, in.x);
    } else {
        in.bv = *reinterpret_cast<const float4*>(sm.bcs + I * 2 * N + g * NPL);
        in.cv = *reinterpret_cast<const float4*>(sm.bcs + I * 2 * N + N + g * NPL);
    }
    return in;
}

__device__ __forceinline__ f2 exp2v(f2 v) {
    f2 r;
    r.x = __builtin_amdgcn_exp2f(v.x);
    r.y = __builtin_amdgcn_exp2f(v.y);
    return r;
}

// The state-independent part of a step: dA = exp2(dt A2), dBx = x (dt B), and C.
struct StepElem {
    f2 a[NP], b[NP];
    float4 cv;
};

__device__ __forceinline__ StepElem make_elem(const StepIn& in, const f2 (&A2)[NP]) {
#pragma clang fp contract(off)
    StepElem e;
    const f2 dt2 = {in.dt, in.dt};
    const f2 x2 = {in.x, in.x};
    const f2 Bn[NP] = {{in.bv.x, in.bv.y}, {in.bv.z, in.bv.w}};
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        e.a[p] = (VASR_SCAN_ABLATE & 1) ? dt2 * A2[p] : exp2v(dt2 * A2[p]);
        const f2 dB = dt2 * Bn[p];
        e.b[p] = x2 * dB;
    }
    e.cv = in.cv;
    return e;
}

// One push of the streaming tree scan at in-chunk step I; leaves this lane's partial y in yv[I].
template <int I, int MAXUP, int N, int DPB>
__device__ __forceinline__ void tree_step(TreeState<MAXUP>& s, const Smem& sm, const StepElem& el, int dl, int g,
                                          f2 (&chunk_a)[NP], f2 (&chunk_b)[NP], float (&yv)[T]) {
#pragma clang fp contract(off)
    constexpr int G = N / NPL;
    // y contribution of h[t] (the exclusive prefix = cb of the current top block)
    {
        f2 h0, h1;
        if constexpr (I == 0) {
            h0 = s.pb[0];
            h1 = s.pb[1];
        } else {
            h0 = s.cb[ctz_c(I)][0];
            h1 = s.cb[ctz_c(I)][1];
        }
        float y = h0.x * el.cv.x;
        y = __builtin_fmaf(h0.y, el.cv.y, y);
        y = __builtin_fmaf(h1.x, el.cv.z, y);
        yv[I] = __builtin_fmaf(h1.y, el.cv.w, y);
    }
    if constexpr (I == 7) flush_half<G, 0>(yv, sm.yp, dl, g);

    constexpr int J = trailing_ones(I);
    if constexpr (VASR_SCAN_ABLATE & 16) {
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            s.pb[p] = s.pb[p] + el.b[p];
            s.pa[p] = el.a[p];
        }
        if constexpr (I == T - 1) flush_half<G, 1>(yv, sm.yp, dl, g);
        return;
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        f2 cur_a = el.a[p];
        f2 cur_b = el.b[p];
#pragma unroll
        for (int k = 0; k < J; ++k) {  // up-sweep: (a_r, b_r) <- (a_r a_l, a_r b_l + b_r)
            cur_b = cur_a * s.lb[k][p] + cur_b;
            cur_a = cur_a * s.la[k][p];
        }
        if constexpr (J < 4) {
            s.la[J][p] = cur_a;
            s.lb[J][p] = cur_b;
            constexpr int BL = below_level(I, J);
            f2 Pa, Pb;
            if constexpr (BL >= 0) {
                Pa = s.ca[BL][p];
                Pb = s.cb[BL][p];
            } else {
                Pa = s.pa[p];
                Pb = s.pb[p];
            }
            const f2 c_a = Pa * cur_a;  // down-sweep: a_r <- a_p a_l ; b_r <- a_r b_l + b_p
            s.ca[J][p] = c_a;
            s.cb[J][p] = c_a * cur_b + Pb;
        } else {
            chunk_a[p] = cur_a;
            chunk_b[p] = cur_b;
        }
    }
    if constexpr (I == T - 1) flush_half<G, 1>(yv, sm.yp, dl, g);
}

// Merge the finished chunk block into the upper (chunk-level) stack when the chunk counter
// cc has J trailing ones (J = levels to merge, a wave-uniform value: one switch case runs),
// then rebuild the prefix after the upper stack bottom-up from the stream form's (1, 0)
// start: the same float operations as carrying (ca, cb) per upper entry.  The levels set in
// cc + 1 are J and those above J that were set in cc; the uniform per-level tests branch.
template <int J, int MAXUP>
__device__ __forceinline__ void merge_upper_j(TreeState<MAXUP>& s, const f2 (&chunk_a)[NP], const f2 (&chunk_b)[NP],
                                              int cc1) {
#pragma clang fp contract(off)
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        f2 cur_a = chunk_a[p], cur_b = chunk_b[p];
#pragma unroll
        for (int u = 0; u < J; ++u) {
            cur_b = cur_a * s.ulb[u][p] + cur_b;
            cur_a = cur_a * s.ula[u][p];
        }
        s.ula[J][p] = cur_a;
        s.ulb[J][p] = cur_b;
    }
    f2 pa[NP], pb[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        pa[p] = f2{1.0f, 1.0f};
        pb[p] = f2{0.0f, 0.0f};
    }
#pragma unroll
    for (int u = MAXUP - 1; u > J; --u) {
        if ((cc1 >> u) & 1) {
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                pa[p] = pa[p] * s.ula[u][p];
                pb[p] = pa[p] * s.ulb[u][p] + pb[p];
            }
        }
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        s.pa[p] = pa[p] * s.ula[J][p];
        s.pb[p] = s.pa[p] * s.ulb[J][p] + pb[p];
    }
}

template <int MAXUP>
__device__ __forceinline__ void merge_upper(TreeState<MAXUP>& s, const f2 (&chunk_a)[NP], const f2 (&chunk_b)[NP],
                                            int cc) {
    const int cc1 = cc + 1;
    switch (__builtin_ctz(~cc)) {
        case 0: merge_upper_j<0, MAXUP>(s, chunk_a, chunk_b, cc1); break;
        case 1: if constexpr (MAXUP > 1) merge_upper_j<1, MAXUP>(s, chunk_a, chunk_b, cc1); break;
        case 2: if constexpr (MAXUP > 2) merge_upper_j<2, MAXUP>(s, chunk_a, chunk_b, cc1); break;
        case 3: if constexpr (MAXUP > 3) merge_upper_j<3, MAXUP>(s, chunk_a, chunk_b, cc1); break;
        case 4: if constexpr (MAXUP > 4) merge_upper_j<4, MAXUP>(s, chunk_a, chunk_b, cc1); break;
        case 5: if constexpr (MAXUP > 5) merge_upper_j<5, MAXUP>(s, chunk_a, chunk_b, cc1); break;
        case 6: if constexpr (MAXUP > 6) merge_upper_j<6, MAXUP>(s, chunk_a, chunk_b, cc1); break;
        case 7: if constexpr (MAXUP > 7) merge_upper_j<7, MAXUP>(s, chunk_a, chunk_b, cc1); break;
        default: if constexpr (MAXUP > 8) merge_upper_j<8, MAXUP>(s, chunk_a, chunk_b, cc1); break;
    }
}

// Two-stage software pipeline over the chunk's 16 steps: operands of step I+2 are read from
// LDS and the state-independent part of step I+1 (exp2, dB, x*dB) is computed while step I's
// tree update runs, so the LDS and v_exp latencies overlap the dependent tree arithmetic.
template <int I, int MAXUP, int N, int DPB, bool FULL>
struct TreeChunk {
    __device__ __forceinline__ static void run(TreeState<MAXUP>& s, const Smem& sm, const StepIn& raw_next,
                                               const StepElem& el, const f2 (&A2)[NP], int dl, int g, int nvalid,
                                               f2 (&ca)[NP], f2 (&cb)[NP], float (&yv)[T]) {
        if (FULL || I < nvalid) {
            StepIn raw2;
            if constexpr (I + 2 < T) raw2 = load_step<I + 2, N, DPB>(sm, dl, g);
            StepElem el_next;
            if constexpr (I + 1 < T) el_next = make_elem(raw_next, A2);
            tree_step<I, MAXUP, N, DPB>(s, sm, el, dl, g, ca, cb, yv);
            TreeChunk<I + 1, MAXUP, N, DPB, FULL>::run(s, sm, raw2, el_next, A2, dl, g, nvalid, ca, cb, yv);
        } else if constexpr (!FULL) {
            // ragged last chunk: flush the partial sums of the steps that ran (the rest are 0)
            if (I < 8) flush_half<N / NPL, 0>(yv, sm.yp, dl, g);
            else flush_half<N / NPL, 1>(yv, sm.yp, dl, g);
        }
    }
};
template <int MAXUP, int N, int DPB, bool FULL>
struct TreeChunk<T, MAXUP, N, DPB, FULL> {
    __device__ __forceinline__ static void run(TreeState<MAXUP>&, const Smem&, const StepIn&, const StepElem&,
                                               const f2 (&)[NP], int, int, int, f2 (&)[NP], f2 (&)[NP], float (&)[T]) {}
};

template <int N, int MODE, int MAXUP>
__global__ __launch_bounds__(256, MAXUP <= 5 ? VASR_SCAN_WAVES : 2) void ssm_scan_kernel(const float* __restrict__ xz, int64_t ld_xz,
                                                       const float* __restrict__ dt, int64_t ld_dt,
                                                       const float* __restrict__ bc, int64_t ld_bc,
                                                       const float* __restrict__ A2g, const float* __restrict__ Dg,
                                                       float* __restrict__ out, int64_t ld_out, int B, int L,
                                                       int Di) {
#pragma clang fp contract(off)
    constexpr int G = N / NPL;       // lanes per channel
    constexpr int DPW = 64 / G;      // channels per wave
    constexpr int DPB = NW * DPW;    // channels per block
    // LDS: two staging buffers {x, dt, z: T x DPB; bc: T x 2N}, partial sums DPB x TP.  The
    // buffers are distinct objects and the chunk loop is unrolled by two, so the compiler can
    // tell that reads of one buffer do not alias the LDS-DMA into the other and does not drain
    // the prefetch (vmcnt(0)) before them.
    constexpr int BUF = 3 * T * DPB + T * 2 * N;
    __shared__ __attribute__((aligned(16))) float sbuf0[BUF];
    __shared__ __attribute__((aligned(16))) float sbuf1[BUF];
    __shared__ __attribute__((aligned(16))) float ypart[DPB * TP];

    // XCD-aware block mapping: blocks id, id+8, id+16, ... share an XCD; give each such
    // group consecutive (b, channel-block) work items so one utterance stays on one L2.
    const int nd = Di / DPB;
    const int nblk = B * nd;
    const int id = blockIdx.x;
    const int q8 = nblk / 8, r8 = nblk % 8, xg = id % 8;
    const int wid = (xg < r8 ? xg * (q8 + 1) : r8 * (q8 + 1) + (xg - r8) * q8) + id / 8;
    const int b = wid / nd;
    const int d0 = (wid - b * nd) * DPB;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int g = lane % G;
    const int dl = wave * DPW + lane / G;

    f2 A2[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) A2[p] = f2{A2g[g * NPL + 2 * p], A2g[g * NPL + 2 * p + 1]};

    const int64_t row0 = (int64_t)b * L;
    // Chunk staging by LDS-DMA (global_load_lds_dwordx4): each wave-instruction moves 1 KiB
    // into a lane-linear LDS range; slabs x | dt | z (T x DPB) and bc (T x 2N) are
    // contiguous, so instruction k of a chunk covers floats [256k, 256k + 256) of the buffer.
    constexpr int SLAB = T * DPB;
    constexpr int NINSTR = BUF / 256;
    static_assert(BUF % 256 == 0 && SLAB % 256 == 0, "staging buffer must be whole 1-KiB pieces");
    auto load_chunk = [&](int t0, float* buf) {
        for (int k = wave; k < NINSTR; k += NW) {
            const int off = k * 256 + lane * 4;  // float offset inside the buffer
            const float* src;
            if (off < 3 * SLAB) {
                const int arr = off / SLAB, rem = off - arr * SLAB;
                const int t = rem / DPB, c = rem - t * DPB;
                const int64_t row = row0 + min(t0 + t, L - 1);
                src = arr == 0 ? xz + row * ld_xz + d0 + c
                    : arr == 1 ? dt + row * ld_dt + d0 + c
                               : xz + row * ld_xz + Di + d0 + c;
            } else {
                const int rem = off - 3 * SLAB;
                const int t = rem / (2 * N), c = rem - t * (2 * N);
                src = bc + (row0 + min(t0 + t, L - 1)) * ld_bc + c;
            }
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src),
                                             (lds_void*)(buf + k * 256), 16, 0, 0);
        }
    };

    const int nchunks = (L + T - 1) / T;
    load_chunk(0, sbuf0);
    __syncthreads();
    const float Dd = Dg[d0 + tid % DPB];

    TreeState<MAXUP> st;
    f2 h[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        st.pa[p] = f2{1.0f, 1.0f};
        st.pb[p] = f2{0.0f, 0.0f};
        h[p] = f2{0.0f, 0.0f};
    }

    auto chunk = [&](int c, float* buf, float* nbuf) {
        Smem sm{buf, buf + T * DPB, buf + 3 * T * DPB, ypart};
        const float* zs = buf + 2 * T * DPB;
        const int t0 = c * T;
        const int nvalid = min(T, L - t0);
        if (c + 1 < nchunks && !((VASR_SCAN_ABLATE & 8) && c > 0)) load_chunk(t0 + T, nbuf);

        if constexpr (MODE == 0) {
            f2 cha[NP], chb[NP];
            float yv[T];
            const StepIn r0 = load_step<0, N, DPB>(sm, dl, g);
            const StepIn r1 = load_step<1, N, DPB>(sm, dl, g);
            const StepElem e0 = make_elem(r0, A2);
            if (nvalid == T) {
                TreeChunk<0, MAXUP, N, DPB, true>::run(st, sm, r1, e0, A2, dl, g, nvalid, cha, chb, yv);
            } else {
#pragma unroll
                for (int j = 0; j < T; ++j) yv[j] = 0.0f;
                TreeChunk<0, MAXUP, N, DPB, false>::run(st, sm, r1, e0, A2, dl, g, nvalid, cha, chb, yv);
            }
            if (c + 1 < nchunks) merge_upper<MAXUP>(st, cha, chb, c);
        } else {
            for (int i = 0; i < nvalid; ++i) {
                const float xv = sm.xs[i * DPB + dl];
                const float dv = sm.dts[i * DPB + dl];
                const float4 bv = *reinterpret_cast<const float4*>(sm.bcs + i * 2 * N + g * NPL);
                const float4 cv = *reinterpret_cast<const float4*>(sm.bcs + i * 2 * N + N + g * NPL);
                const f2 Bn[NP] = {{bv.x, bv.y}, {bv.z, bv.w}};
                const f2 Cn[NP] = {{cv.x, cv.y}, {cv.z, cv.w}};
                const f2 dv2 = {dv, dv}, xv2 = {xv, xv};
                f2 part = {0.f, 0.f};
#pragma unroll
                for (int p = 0; p < NP; ++p) {
                    const f2 dA = exp2v(dv2 * A2[p]);
                    const f2 dB = dv2 * Bn[p];
                    h[p] = dA * h[p] + xv2 * dB;
                    part = part + h[p] * Cn[p];
                }
                const float y = group_sum<G>(part.x + part.y);
                if (g == 0) ypart[dl * TP + i] = y;
            }
        }
        // partial sums visible to all waves; the LDS-DMA of chunk c+1 stays in flight
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) only
        __builtin_amdgcn_s_barrier();
        // gated output of this chunk: (sum_g partials + x D) * silu(z), coalesced along d
        for (int idx = tid; idx < T * DPB; idx += 64 * NW) {
            const int t = idx / DPB, d = idx - t * DPB;
            if (t < nvalid) {
                const float ysum = ypart[d * TP + t];
                if ((VASR_SCAN_ABLATE & 32) && ysum != 1.2345f) continue;
                const float xv = sm.xs[t * DPB + d];
                const float zv = zs[t * DPB + d];
                const float y = ysum + xv * Dd;
                const float silu = zv / (1.0f + expf(-zv));
                out[(row0 + t0 + t) * ld_out + d0 + d] = y * silu;
            }
        }
        __syncthreads();  // also drains this wave's LDS-DMA of chunk c+1 (vmcnt(0) before the barrier)
    };
    for (int c = 0; c < nchunks; c += 2) {
        chunk(c, sbuf0, sbuf1);
        if (c + 1 < nchunks) chunk(c + 1, sbuf1, sbuf0);
    }
}

template <int N, int MODE>
int launch_n(const float* xz, int64_t ld_xz, const float* dt, int64_t ld_dt, const float* bc, int64_t ld_bc,
             const float* A2, const float* D, float* out, int64_t ld_out, int B, int L, int Di, hipStream_t s) {
    constexpr int G = N / NPL;
    constexpr int DPB = NW * (64 / G);
    if (Di % DPB != 0) {
        set_error("vasr_ssm_scan_f32: Di=%d must be a multiple of %d for N=%d", Di, DPB, N);
        return VASR_EUNSUPPORTED;
    }
    dim3 grid(B * (Di / DPB));
    dim3 block(64 * NW);
    const int nchunks = (L + T - 1) / T;
    if (MODE == 1 || nchunks <= 32)
        hipLaunchKernelGGL((ssm_scan_kernel<N, MODE, 5>), grid, block, 0, s, xz, ld_xz, dt, ld_dt, bc, ld_bc, A2, D,
                           out, ld_out, B, L, Di);
    else if (nchunks <= 128)
        hipLaunchKernelGGL((ssm_scan_kernel<N, MODE, 7>), grid, block, 0, s, xz, ld_xz, dt, ld_dt, bc, ld_bc, A2, D,
                           out, ld_out, B, L, Di);
    else
        hipLaunchKernelGGL((ssm_scan_kernel<N, MODE, 9>), grid, block, 0, s, xz, ld_xz, dt, ld_dt, bc, ld_bc, A2, D,
                           out, ld_out, B, L, Di);
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
