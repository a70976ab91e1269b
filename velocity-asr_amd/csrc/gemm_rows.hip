// Split-bf16 fp32 GEMM for short K (K <= 16 * KS: the model's K = 192 projections), "A rows
// stationary": each wave loads its 32 rows of A once, splits them into the three bf16 planes
// (x = hi + mid + lo, gemm_split.h) and keeps all of them in VGPRs (12 k-steps x 3 planes x
// bf16x8 = 144 VGPRs at K = 192) for the whole kernel, then walks a run of 32-column W chunks:
// per chunk 12 k-steps x the same six v_mfma_f32_32x32x16_bf16 products in the same order as
// the LDS-ring tile kernel (gemm_x3.hip), so the results are bitwise those of that kernel.
//
// Why: at K = 192 the tile kernel spends a whole 128 x 128 tile's life in one short K loop and
// then stores 64 KB of C at the end, in phase with every other block (measured: MFMA phase
// 12.3 us and store phase 10.8 us per two tiles per CU, serialised).  Here a
// block owns 256 rows x a run of 32-column chunks, with two accumulator sets: chunk j's MFMAs
// issue while chunk j-1's epilogue stores (non-temporal) drain, and the W chunks (36 KiB each,
// in the fragment-native layout of vasr_split_weights_bf16x3, contiguous per chunk) stream
// through a three-slot LDS ring by LDS-DMA two chunks ahead (issued by four of the eight waves).
//
// Work decomposition: block = 8 waves (two per SIMD) x 32 rows = 256 rows, grid = row blocks x
// column groups (runs of chunks), at most one block per CU so the grid is one round; blocks id,
// id + 8, ... share an XCD and get consecutive (row block, column group) items, so the column
// groups of one row block read its A rows from one L2.  Epilogues: gemm_common.h's (unpaired
// ones), per 32 x 32 chunk.  Measured variants, all slower or equal: 4 waves per
// block, cached stores, store groups of 2-4 chunks written back to back (profiles/r03k), the
// chunk's DMA issued before the previous epilogue / no store waits in non-loader waves
// (profiles/r03r), and the epilogue interleaved into the next chunk's k-steps at 4 or 8 waves
// (37.0 / 37.6 vs 33.4 us, profiles/r03u).
#include <type_traits>

#include "gemm_common.h"
#include "gemm_split.h"

namespace vasr {
namespace {

using namespace gemm;

typedef __attribute__((address_space(3))) void lds_void;

// LDS-DMA of 16 B per lane into dst_base + 16 * lane (untracked by the compiler's waitcnt
// model, ordered by the kernel: counted vmcnt + barrier; the memory clobber keeps the
// epilogue's stores ahead of it in issue order)
__device__ __forceinline__ void glds16(const void* src, void* dst_base) {
    const unsigned lds = (unsigned)(uintptr_t)(lds_void*)dst_base;
    // M0 is compiler-reserved: saved and restored inside the statement, and the SALU write of M0
    // needs one wait state before the LDS-DMA reads it (s_nop 0)
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "s"(lds), "v"(src) : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

#ifndef VASR_ROWS_ABLATE
#define VASR_ROWS_ABLATE 0  // diagnostic builds only: 1 no MFMA, 2 no epilogue stores, 4 no LDS-DMA
#endif                      // after the first two chunks, 8 no per-chunk barrier
#ifndef VASR_ROWS_WAVES
#define VASR_ROWS_WAVES 8  // 256 A rows per block (r03k: 8 waves 37.8 us vs 4 waves 45.0 on the head GEMM)
#endif
#ifndef VASR_ROWS_DEPTH
#define VASR_ROWS_DEPTH 2  // W chunks in flight ahead of the one being multiplied (LDS slots = depth + 1)
#endif
#ifndef VASR_ROWS_STORE_AUX
#define VASR_ROWS_STORE_AUX 2  // cache-policy bits of the epilogue's buffer stores (2 = nt: C is not re-read from L2)
#endif
constexpr int RW = VASR_ROWS_WAVES;  // waves per block (4: one per SIMD)
constexpr int DEPTH = VASR_ROWS_DEPTH;
constexpr int NSLOT = DEPTH + 1;
#ifndef VASR_ROWS_STORE_WAIT
#define VASR_ROWS_STORE_WAIT 1  // 0: the store-only waves never wait for their older stores
#endif
#ifndef VASR_ROWS_MAX_GROUP
#define VASR_ROWS_MAX_GROUP 16
#endif
constexpr int MAX_GROUP = VASR_ROWS_MAX_GROUP;  // chunks per column group (LDS epilogue tables: MAX_GROUP x 32 columns)

// s_waitcnt vmcnt(n) for a runtime n in [0, 63] (the immediate has to be a constant)
__device__ __forceinline__ void wait_vmcnt_rt(int n) {
    switch (n) {
#define VASR_W(I) case I: wait_vmcnt<I>(); break;
#define VASR_W8(B) VASR_W(B) VASR_W(B + 1) VASR_W(B + 2) VASR_W(B + 3) VASR_W(B + 4) VASR_W(B + 5) VASR_W(B + 6) VASR_W(B + 7)
        VASR_W8(0) VASR_W8(8) VASR_W8(16) VASR_W8(24) VASR_W8(32) VASR_W8(40) VASR_W8(48) VASR_W8(56)
#undef VASR_W8
#undef VASR_W
        default: wait_vmcnt<0>();
    }
}

#ifdef VASR_ROWS_STAMPS
// Diagnostic builds only: per-wave sums of the cycles (s_memtime) spent in each phase of a chunk
// step, written once at the end of the kernel (no stores inside the loop), tools/diag/rows_stamps.py.
__device__ unsigned long long* g_rows_stamps;
#define VASR_STAMP(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#else
#define VASR_STAMP(v)
#endif

// Epilogue of one 32 x 32 chunk held as one MFMA accumulator (the tile kernel's epilogue_body
// arithmetic for TM = TN = 1), with the per-column bias / fake-quant parameters read from LDS
// and the results written by raw buffer stores: exactly NST store instructions per wave and
// chunk whatever the bounds (out-of-range lanes get an offset past the buffer's num_records,
// which the hardware drops), so the kernel's counted vmcnt waits stay exact.  No vector-memory
// loads besides the residual / positional operand, so the compiler's own vmcnt waits for those
// are the only ones that also cover the LDS-DMA ring in flight.
constexpr int NST = 16;  // store instructions per wave per chunk
constexpr int OOB = 0x7FFFFFFC;

template <int EPI>
__device__ __forceinline__ void rows_epilogue(const GemmParams& p, __amdgpu_buffer_rsrc_t cbuf, int m0, int n0,
                                              const floatx16& acc, int r, int h, const float* __restrict__ bias_s,
                                              const float4* __restrict__ qp_s, int cfirst) {
    const int col = n0 + r;
    const bool col_ok = col < p.N;
    const int lc = col - cfirst;  // column in the group's LDS tables
    const float bv = p.bias ? bias_s[lc] : 0.0f;
    float4 qc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (p.qp) qc = qp_s[lc];
    if constexpr (EPI == VASR_EPI_ARGMAX) {
        const int slot = n0 / 32;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int row = m0 + (i & 3) + 8 * (i >> 2) + 4 * h;
            float v = acc[i];
            if (p.bias) v = v + bv;
            if (p.qp) v = fake_quant(v, qc);
            const unsigned u = __float_as_uint(v);
            const unsigned ord = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
            const unsigned long long k0 = col_ok ? ((unsigned long long)ord << 32) | (0xFFFFFFFFu - (unsigned)col) : 0ull;
            const unsigned long long key = gemm::max_u64_over_32_lanes(k0);  // lanes r = 16..31 hold it
            const int off = (r == 31 && row < p.M) ? (row * (int)p.ldc + slot) * 8 : OOB;
            typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
            const u32x2 kv = {(unsigned)key, (unsigned)(key >> 32)};
            if (!(VASR_ROWS_ABLATE & 2)) __builtin_amdgcn_raw_buffer_store_b64(kv, cbuf, off, 0, VASR_ROWS_STORE_AUX);
        }
        return;
    }
    // SP: 0 no softplus, 1 every column of the chunk, 2 per column (the chunk straddles n_out)
    auto body = [&](auto SPc) {
        constexpr int SP = decltype(SPc)::value;
        const bool sp = SP == 1 || (SP == 2 && col >= p.n_out);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int row = m0 + (i & 3) + 8 * (i >> 2) + 4 * h;
            const bool ok = col_ok && row < p.M;
            float v = acc[i];
            if (p.bias) v = v + bv;
            if (p.qp) v = fake_quant(v, qc);
            if constexpr (EPI == VASR_EPI_GELU) {
                v = gelu_fast(v);
            } else if constexpr (EPI == VASR_EPI_SOFTPLUS_FROM) {
                if constexpr (SP == 1) v = softplus20_fast(v);
                else if constexpr (SP == 2) v = sp ? softplus20_fast(v) : v;
            } else if constexpr (EPI == VASR_EPI_RESIDUAL) {
                v = v + p.aux[(int64_t)min(row, p.M - 1) * p.ld_aux + min(col, p.N - 1)];
            } else if constexpr (EPI == VASR_EPI_GELU_PE) {
                v = gelu_fast(v) + p.aux[(int64_t)min(row, p.M - 1) * p.ld_aux + min(col, p.N - 1)];
            }
            if (!(VASR_ROWS_ABLATE & 2))
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), cbuf, ok ? (row * (int)p.ldc + col) * 4 : OOB,
                                                      0, VASR_ROWS_STORE_AUX);
        }
    };
    // n0 is wave-uniform: whole chunks branch (a per-lane select ran softplus's exp / log on
    // every chunk and discarded it: 33.4 vs 39 us for the composed head GEMM, profiles/r03t)
    if constexpr (EPI == VASR_EPI_SOFTPLUS_FROM) {
        if (n0 >= p.n_out) body(std::integral_constant<int, 1>());
        else if (n0 + 32 <= p.n_out) body(std::integral_constant<int, 0>());
        else body(std::integral_constant<int, 2>());
    } else {
        body(std::integral_constant<int, 0>());
    }
}

template <int KS, int EPI>
__global__ __launch_bounds__(64 * RW, 1) void gemm_rows_kernel(GemmParams p, int n_groups, int chunks_per_group) {
    constexpr int CHUNK = KS * 3 * 1024;       // one 32-column W chunk: [KS][3 planes][64 lanes][16 B]
    constexpr int DW = 4;                      // loader waves (the first four) issue the chunk's DMA
    constexpr int NDMA = 3 * KS / DW;          // LDS-DMA instructions per loader wave per chunk
    static_assert((3 * KS) % DW == 0 && RW % DW == 0, "whole DMA pieces per loader wave");
    __shared__ __attribute__((aligned(16))) char wb0[CHUNK];
    __shared__ __attribute__((aligned(16))) char wb1[CHUNK];
    __shared__ __attribute__((aligned(16))) char wb2[CHUNK];
    __shared__ __attribute__((aligned(16))) char wb3[NSLOT > 3 ? CHUNK : 16];
    __shared__ float bias_s[MAX_GROUP * 32];
    __shared__ float4 qp_s[MAX_GROUP * 32];

    const int nblk = (int)gridDim.x;
    const int id = blockIdx.x;
    const int q8 = nblk / 8, r8 = nblk % 8, xg = id % 8;
    const int w = (xg < r8 ? xg * (q8 + 1) : r8 * (q8 + 1) + (xg - r8) * q8) + id / 8;
    const int rb = w / n_groups, ng = w - rb * n_groups;
    const int NT = (p.N + 31) / 32;
    const int c0 = ng * chunks_per_group;
    const int nc = min(chunks_per_group, NT - c0);
    if (nc <= 0) return;  // block-uniform

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int wave_u = __builtin_amdgcn_readfirstlane(wave);
    const int m0 = rb * 32 * RW + wave * 32;  // this wave's rows
    const int cfirst = c0 * 32;

    // A rows (lane (r, h): row r, k = 16 ks + 8 h + 0..7; columns past K read as 0 from a
    // clamped address, no branches) and the group's epilogue tables
    const float* __restrict__ arow = p.A + (int64_t)min(m0 + r, p.M - 1) * p.lda;
    float4 xa[KS][2];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int k = 16 * ks + 8 * h + 4 * u;
            const float4 v = *reinterpret_cast<const float4*>(arow + min(k, p.K - 4));
            xa[ks][u] = k < p.K ? v : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    for (int i = tid; i < nc * 32; i += 64 * RW) {
        const int col = min(cfirst + i, p.N - 1);
        if (p.bias) bias_s[i] = p.bias[col];
        if (p.qp) qp_s[i] = p.qp[col];
    }
    bf16x8 a[KS][3];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) split8(xa[ks][0], xa[ks][1], a[ks][0], a[ks][1], a[ks][2]);

    const char* __restrict__ Wx = reinterpret_cast<const char*>(p.Wx);
    auto slot = [&](int i) -> char* { return i == 0 ? wb0 : i == 1 ? wb1 : i == 2 ? wb2 : wb3; };
    const bool loader = wave_u < DW;
    auto issue = [&](int j) {
        if (!loader) return;
        const char* src = Wx + (int64_t)(c0 + j) * CHUNK + lane * 16;
        char* dst = slot(j % NSLOT);
#pragma unroll
        for (int i = 0; i < NDMA; ++i) {
            const int piece = i * DW + wave_u;
            glds16(src + piece * 1024, dst + piece * 1024);
        }
    };
    for (int j = 0; j < DEPTH && j < nc; ++j) issue(j);

    // C as a raw buffer over its valid bytes (the host checks they fit 31 bits)
    const int c_bytes = (EPI == VASR_EPI_ARGMAX ? 8 : 4) * ((p.M - 1) * (int)p.ldc + (EPI == VASR_EPI_ARGMAX ? NT : p.N));
    const __amdgpu_buffer_rsrc_t cbuf = __builtin_amdgcn_make_buffer_rsrc(p.C, 0, c_bytes, 0x00020000);
    // two accumulator sets: chunk j's MFMAs into set j & 1 while chunk j - 1's epilogue stores
    // (set (j - 1) & 1) drain
    floatx16 acc[2];
#ifdef VASR_ROWS_STAMPS
    unsigned long long st_wait = 0, st_bar = 0, st_epi = 0, st_dma = 0, st_mfma = 0;
    VASR_STAMP(st_begin);
#endif
    // chunk j into set S: wait for its DMA (counted: younger DMAs and stores stay in flight),
    // publish it block-wide (the barrier also certifies every wave is done with the slot
    // DMA(j + DEPTH) refills), chunk j - 1's epilogue, prefetch chunk j + DEPTH, chunk j's MFMAs
    auto step = [&](auto Sc, int j) {
        constexpr int S = decltype(Sc)::value;
        // A loader wave waits for everything it issued: its DMA(j) has epilogue stores issued
        // after it (step j - 1 stores chunk j - 2), and vmcnt counts loads and stores together
        // with a store able to complete before an older load, so a count that includes those
        // stores does not prove DMA(j) landed (the scan's fix of the same mistake:
        // scan_body.inc, profiles/r04b/).  (Counting only the younger DMA loads -- safe if loads
        // retire in order among themselves -- measured no faster, 69.5 vs 68.7-70.5 us at
        // M = 16032, profiles/r04v/, so the plain form stays.)  The other waves issue stores only
        // (one event type: in order): they keep the stores of steps j - DEPTH + 1 .. j - 1 in
        // flight and bound the older ones.
        int n_vm = 0;
        if (!loader && !(VASR_ROWS_ABLATE & 2)) n_vm = VASR_ROWS_STORE_WAIT ? NST * max(0, j - max(j - DEPTH + 1, 1)) : 63;
        VASR_STAMP(t0);
        wait_vmcnt_rt(min(n_vm, 63));
        VASR_STAMP(t1);
        if (!(VASR_ROWS_ABLATE & 8)) __builtin_amdgcn_s_barrier();
        VASR_STAMP(t2);
        const char* wb = slot((VASR_ROWS_ABLATE & 4) ? min(j, DEPTH - 1) : j % NSLOT) + lane * 16;
        // W fragments of k-step 0 first, so the chunk's first MFMA does not wait behind the epilogue
        bf16x8 wf[2][3];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) wf[0][pl] = *reinterpret_cast<const bf16x8*>(wb + pl * 1024);
        if (j >= 1) rows_epilogue<EPI>(p, cbuf, m0, (c0 + j - 1) * 32, acc[S ^ 1], r, h, bias_s, qp_s, cfirst);
        VASR_STAMP(t3);
        if (j + DEPTH < nc && !(VASR_ROWS_ABLATE & 4)) issue(j + DEPTH);
        VASR_STAMP(t4);
        floatx16 c;
#pragma unroll
        for (int i = 0; i < 16; ++i) c[i] = 0.f;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const int cur = ks & 1;
            if (ks + 1 < KS) {  // next k-step's fragments one step ahead of their MFMAs
#pragma unroll
                for (int pl = 0; pl < 3; ++pl)
                    wf[cur ^ 1][pl] = *reinterpret_cast<const bf16x8*>(wb + ((ks + 1) * 3 + pl) * 1024);
            }
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (VASR_ROWS_ABLATE & 1) {
                c[0] += (float)a[ks][0][0] * (float)wf[cur][0][0] + (float)a[ks][2][1] * (float)wf[cur][2][1];
                continue;
            }
            // small terms first, then the leading hi*hi term (gemm_x3.hip's order)
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ks][2], wf[cur][0], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ks][0], wf[cur][2], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ks][1], wf[cur][1], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ks][1], wf[cur][0], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ks][0], wf[cur][1], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ks][0], wf[cur][0], c, 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
        acc[S] = c;
#ifdef VASR_ROWS_STAMPS
        VASR_STAMP(t5);
        st_wait += t1 - t0;
        st_bar += t2 - t1;
        st_epi += t3 - t2;
        st_dma += t4 - t3;
        st_mfma += t5 - t4;
#endif
    };
    for (int j = 0; j < nc; j += 2) {
        step(std::integral_constant<int, 0>(), j);
        if (j + 1 < nc) step(std::integral_constant<int, 1>(), j + 1);
    }
    const int jl = nc - 1;  // the last chunk's epilogue
    rows_epilogue<EPI>(p, cbuf, m0, (c0 + jl) * 32, (jl & 1) ? acc[1] : acc[0], r, h, bias_s, qp_s, cfirst);
#ifdef VASR_ROWS_STAMPS
    __builtin_amdgcn_s_waitcnt(0);
    VASR_STAMP(st_end);
    if (lane == 0 && g_rows_stamps) {
        unsigned long long* o = g_rows_stamps + ((int64_t)blockIdx.x * RW + wave) * 8;
        o[0] = st_wait; o[1] = st_bar; o[2] = st_epi; o[3] = st_dma; o[4] = st_mfma; o[5] = st_end - st_begin;
        o[6] = (unsigned long long)nc; o[7] = loader ? 1 : 0;
    }
#endif
}

template <int KS>
int launch_rows(const GemmParams& p, int epi, hipStream_t s) {
    const int NT = (p.N + 31) / 32;
    const int row_blocks = (p.M + 32 * RW - 1) / (32 * RW);
    // column groups: at most one block per CU (LDS: NSLOT x 36 KiB per block), so a grid of more
    // than kCUs blocks runs in rounds, and a partial round costs as much as a full one.  The
    // groups minimise rounds x (chunks per block + 1), the 1 standing for a block's A prologue
    // (its 256 rows loaded and split): M = 16032 keeps 4 groups of 10 chunks (252 blocks, one
    // round); the 30-s clips' M = 48096 takes 4 groups in 3 rounds (30 chunk-steps per CU) instead
    // of 3 groups of 16 (the MAX_GROUP cap) in 3 rounds (48), M = 24048 5 groups of 8 in 2 rounds
    // (16) instead of 3 of 16 in 2 (32).
    int groups = 1, per = min(NT, MAX_GROUP), best = -1;
    for (int g = 1; g <= NT; ++g) {
        const int pg = (NT + g - 1) / g;
        if (pg > MAX_GROUP) continue;
        const int gg = (NT + pg - 1) / pg;
        const int cost = ((row_blocks * gg + kCUs - 1) / kCUs) * (pg + 1);
        if (best < 0 || cost < best) {
            best = cost;
            groups = gg;
            per = pg;
        }
    }
    const dim3 grid(row_blocks * groups), block(64 * RW);
#define VASR_R(E) hipLaunchKernelGGL((gemm_rows_kernel<KS, E>), grid, block, 0, s, p, groups, per)
    switch (epi) {
        case VASR_EPI_NONE: VASR_R(VASR_EPI_NONE); break;
        case VASR_EPI_GELU: VASR_R(VASR_EPI_GELU); break;
        case VASR_EPI_SOFTPLUS_FROM: VASR_R(VASR_EPI_SOFTPLUS_FROM); break;
        case VASR_EPI_RESIDUAL: VASR_R(VASR_EPI_RESIDUAL); break;
        case VASR_EPI_GELU_PE: VASR_R(VASR_EPI_GELU_PE); break;
        case VASR_EPI_ARGMAX: VASR_R(VASR_EPI_ARGMAX); break;
        default: set_error("vasr_linear_x3_f32: rows engine: epilogue %d not supported", epi); return VASR_EINVAL;
    }
#undef VASR_R
    return launch_status("vasr_linear_x3_f32");
}

}  // namespace

// The rows engine serves batch-1 launches with K <= 192 and unpaired epilogues (the model's
// projection GEMMs at K = 192, the CTC head); returns false when the tile kernel should run.
bool try_rows_x3(const GemmParams& p, int batch, int epi, hipStream_t s, int* rc) {
    if (batch != 1 || p.Kp > 192 || p.M <= 0 || epi == VASR_EPI_PAIR_POWER || epi == VASR_EPI_PAIR_FUSION) return false;
    if (p.Kp != 128 && p.Kp != 192) return false;  // the W chunk stride is Kp / 16 k-steps
    // raw-buffer C addressing: the valid bytes must fit the 31-bit offsets
    if ((int64_t)p.M * p.ldc * (epi == VASR_EPI_ARGMAX ? 8 : 4) >= ((int64_t)1 << 31) - 64) return false;
    const int engine = option(VASR_OPT_GEMM_ENGINE);  // 0 auto, 1 tiles, 2 rows
    if (engine == 1) return false;
    // auto: the rows engine where it measured faster (profiles/r03l: K = 192, N >= 512 -- the
    // composed head GEMM 35.8 vs 45.6 us, in_proj 21.1 vs 22.8; at N = 384 / 192 a block's short
    // chunk run does not amortise its A load; one utterance, M = 501: 13.2 vs 8.4 us in the
    // graph, profiles/r03m -- two 256-row blocks per column group); the argmax head keeps the tiles (its per-chunk
    // 32-lane reductions), and so do the residual / GELU+PE epilogues (they spill at 8 waves)
    if (engine == 0 && (p.Kp != 192 || p.N < 512 || p.M < 4096 ||
                        !(epi == VASR_EPI_NONE || epi == VASR_EPI_GELU || epi == VASR_EPI_SOFTPLUS_FROM)))
        return false;
    *rc = p.Kp == 128 ? launch_rows<8>(p, epi, s) : launch_rows<12>(p, epi, s);
    return true;
}

}  // namespace vasr

#ifdef VASR_ROWS_STAMPS
VASR_API int vasr_diag_rows_stamps(void* buf) {  // diagnostic builds only
    return hipMemcpyToSymbol(HIP_SYMBOL(vasr::g_rows_stamps), &buf, sizeof(buf)) == hipSuccess ? VASR_OK : VASR_EINVAL;
}
#endif
