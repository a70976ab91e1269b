// CTC greedy decode on device (reference velocity_asr/decode.py:27-125).
//  argmax   : one wave per frame row over V logits, ties -> lowest index (torch.argmax).
//  collapse : per utterance, keep each maximal run of one non-blank token once
//             (collapse=1; decode.py:56-67) or every non-blank frame (collapse=0), and
//             optionally the run's [start, end) frames (with_timestamps, decode.py:89-123).
#include "vasr_internal.h"

namespace vasr {
namespace {

__global__ __launch_bounds__(256) void argmax_kernel(const float* __restrict__ x, int64_t ld, int rows, int V,
                                                     int32_t* __restrict__ out) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const int lane = threadIdx.x & 63;
    const float* xr = x + (int64_t)row * ld;
    float best = -INFINITY;
    int bi = V;  // sentinel larger than any index
    for (int j = lane; j < V; j += 64) {
        const float v = xr[j];
        // NaN propagates as the max (torch semantics); first index wins ties
        if (v > best || (v != v && best == best)) {
            best = v;
            bi = j;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float ov = __shfl_xor(best, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        const bool o_nan = ov != ov, b_nan = best != best;
        bool take;
        if (o_nan || b_nan) take = o_nan && (!b_nan || oi < bi);
        else take = ov > best || (ov == best && oi < bi);
        if (take) {
            best = ov;
            bi = oi;
        }
    }
    if (lane == 0) out[row] = bi < V ? bi : 0;
}

// One wave per utterance, 64 frames per iteration.  A frame t is kept iff it is not blank
// and (collapse == 0 or t == 0 or pred[t-1] != pred[t]) -- equivalent to the reference's
// prev-token loop, since prev is None after a blank and equals pred[t-1] otherwise.  Kept
// frames are compacted with a ballot + popcount prefix.  A kept token's end frame is the
// next run start (the first frame whose value differs), matching decode.py:89-123.
// p: the utterance's frame predictions (global memory or LDS); its first L frames collapse
// (outputs at row stride ldL).
__device__ __forceinline__ void collapse_wave(const int32_t* p, int L, int ldL, int b, int blank, int collapse,
                                              int32_t* __restrict__ toks, int32_t* __restrict__ lens,
                                              int32_t* __restrict__ st, int32_t* __restrict__ en) {
    const int lane = threadIdx.x & 63;
    int32_t* o = toks + (int64_t)b * ldL;
    int base = 0;  // tokens kept before this window
    for (int t0 = 0; t0 < L; t0 += 64) {
        const int t = t0 + lane;
        const bool in = t < L;
        const int tok = in ? p[t] : blank;
        const int prv = (in && t > 0) ? p[t - 1] : -1;
        const bool keep = in && tok != blank && (!collapse || t == 0 || prv != tok);
        const unsigned long long kmask = __ballot(keep);
        const int before = __popcll(kmask & ((1ull << lane) - 1ull));
        if (keep) {
            o[base + before] = tok;
            if (st) st[(int64_t)b * ldL + base + before] = t;
        }
        if (st) {
            // a run starting at t closes the previous run; if that run was a kept token, it is
            // the last token kept before t
            const bool run_start = in && t > 0 && prv != tok && prv != blank;
            if (run_start) en[(int64_t)b * ldL + base + before - 1] = t;
        }
        base += __popcll(kmask);
    }
    if (lane == 0) {
        lens[b] = base;
        if (st && L > 0 && p[L - 1] != blank && base > 0) en[(int64_t)b * ldL + base - 1] = L;
    }
}

// Rows utterance b collapses: frames[b] clamped to [0, L] (a value past L would read predictions
// this launch did not write and write tokens past the utterance's row), or all L.
__device__ __forceinline__ int frames_of(const int32_t* frames, int b, int ldL) {
    return frames ? min(max(frames[b], 0), ldL) : ldL;
}

// frames (optional): utterance b collapses its own first frames[b] rows (row stride stays L).
__global__ __launch_bounds__(64) void collapse_kernel(const int32_t* __restrict__ pred, int ldL, int blank, int collapse,
                                                      int32_t* __restrict__ toks, int32_t* __restrict__ lens,
                                                      int32_t* __restrict__ st, int32_t* __restrict__ en,
                                                      const int32_t* __restrict__ frames) {
    const int b = blockIdx.x;
    collapse_wave(pred + (int64_t)b * ldL, frames_of(frames, b, ldL), ldL, b, blank, collapse, toks, lens, st, en);
}

// Argmax keys -> tokens -> collapse in one launch, one workgroup per utterance: its 256 threads
// reduce a row each (the row's slot keys, as argmax_keys_kernel) into an LDS copy of the
// utterance's predictions, then wave 0 collapses them (collapse_wave).  Saves the collapse's
// launch and its read-back of the predictions (one utterance: ~4.5 us of ~0.58 ms).
constexpr int kCollapseKeysMaxL = 8192;
__global__ __launch_bounds__(256) void collapse_keys_kernel(const unsigned long long* __restrict__ keys, int64_t ld,
                                                            int slots, int ldL, const int32_t* __restrict__ frames,
                                                            int blank, int collapse, int32_t* __restrict__ pred,
                                                            int32_t* __restrict__ toks, int32_t* __restrict__ lens,
                                                            int32_t* __restrict__ st, int32_t* __restrict__ en) {
    __shared__ int32_t sp[kCollapseKeysMaxL];
    const int b = blockIdx.x;
    for (int t = threadIdx.x; t < ldL; t += 256) {
        const unsigned long long* kr = keys + ((int64_t)b * ldL + t) * ld;
        unsigned long long k = 0ull;
#pragma unroll 8
        for (int s = 0; s < slots; ++s) {
            const unsigned long long v = kr[s];
            k = v > k ? v : k;
        }
        const int32_t tok = (int32_t)(0xFFFFFFFFu - (unsigned)(k & 0xFFFFFFFFull));
        sp[t] = tok;
        if (pred) pred[(int64_t)b * ldL + t] = tok;
    }
    __syncthreads();
    if (threadIdx.x < 64) collapse_wave(sp, frames_of(frames, b, ldL), ldL, b, blank, collapse, toks, lens, st, en);
}

// One wave per two rows: lane l reads slot l % 32 of row 2w + l / 32 (coalesced), then a
// 32-lane max by shuffles.
__global__ __launch_bounds__(256) void argmax_keys_kernel(const unsigned long long* __restrict__ keys, int64_t ld,
                                                          int slots, int rows, int32_t* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int row = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 + (lane >> 5);
    const int sl = lane & 31;
    unsigned long long k = 0ull;
    if (row < rows)
        for (int s = sl; s < slots; s += 32) {
            const unsigned long long v = keys[(int64_t)row * ld + s];
            k = v > k ? v : k;
        }
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) {
        const unsigned long long v = __shfl_xor(k, o, 64);
        k = v > k ? v : k;
    }
    if (row < rows && sl == 0) out[row] = (int32_t)(0xFFFFFFFFu - (unsigned)(k & 0xFFFFFFFFull));
}

}  // namespace
}  // namespace vasr

VASR_API int vasr_argmax_f32(const float* logits, int64_t ld, int rows, int V, int32_t* out, void* stream) {
    using namespace vasr;
    VASR_CHECK_ARG(logits && out, "vasr_argmax_f32: null pointer");
    VASR_CHECK_ARG(rows >= 0 && V >= 1 && ld >= V, "vasr_argmax_f32: bad shape");
    if (rows == 0) return VASR_OK;
    hipLaunchKernelGGL(argmax_kernel, dim3((rows + 3) / 4), dim3(256), 0, as_stream(stream), logits, ld, rows, V, out);
    return launch_status("vasr_argmax_f32");
}

static int ctc_collapse(const int32_t* pred, int B, int L, const int32_t* frames, int blank, int collapse,
                        int32_t* out_tokens, int32_t* out_len, int32_t* out_start, int32_t* out_end, void* stream,
                        const char* who) {
    using namespace vasr;
    VASR_CHECK_ARG(pred && out_tokens && out_len, "%s: null pointer", who);
    VASR_CHECK_ARG((out_start == nullptr) == (out_end == nullptr), "%s: start/end must both be set", who);
    VASR_CHECK_ARG(out_start == nullptr || collapse, "%s: timestamps need collapse=1", who);
    VASR_CHECK_ARG(B >= 0 && L >= 0, "%s: bad shape", who);
    if (B == 0) return VASR_OK;
    hipLaunchKernelGGL(collapse_kernel, dim3(B), dim3(64), 0, as_stream(stream), pred, L, blank, collapse, out_tokens,
                       out_len, out_start, out_end, frames);
    return launch_status(who);
}

VASR_API int vasr_ctc_collapse(const int32_t* pred, int B, int L, int blank, int collapse, int32_t* out_tokens,
                               int32_t* out_len, int32_t* out_start, int32_t* out_end, void* stream) {
    return ctc_collapse(pred, B, L, nullptr, blank, collapse, out_tokens, out_len, out_start, out_end, stream,
                        "vasr_ctc_collapse");
}

// frames (device): frames[b] rows of utterance b, clamped to [0, L] (row stride of pred and outputs stays L).
VASR_API int vasr_ctc_collapse_var(const int32_t* pred, int B, int L, const int32_t* frames, int blank, int collapse,
                                   int32_t* out_tokens, int32_t* out_len, int32_t* out_start, int32_t* out_end,
                                   void* stream) {
    VASR_CHECK_ARG(frames, "vasr_ctc_collapse_var: null frames");
    return ctc_collapse(pred, B, L, frames, blank, collapse, out_tokens, out_len, out_start, out_end, stream,
                        "vasr_ctc_collapse_var");
}

VASR_API int vasr_ctc_collapse_keys(const uint64_t* keys, int64_t ld, int slots, int B, int L, const int32_t* frames,
                                    int blank, int collapse, int32_t* pred, int32_t* out_tokens, int32_t* out_len,
                                    int32_t* out_start, int32_t* out_end, void* stream) {
    using namespace vasr;
    VASR_CHECK_ARG(keys && out_tokens && out_len && slots >= 1 && ld >= slots, "vasr_ctc_collapse_keys: bad arguments");
    VASR_CHECK_ARG((out_start == nullptr) == (out_end == nullptr), "vasr_ctc_collapse_keys: start/end must both be set");
    VASR_CHECK_ARG(out_start == nullptr || collapse, "vasr_ctc_collapse_keys: timestamps need collapse=1");
    VASR_CHECK_ARG(B >= 0 && L >= 0 && L <= kCollapseKeysMaxL, "vasr_ctc_collapse_keys: bad shape B=%d L=%d (L <= %d)", B,
                   L, kCollapseKeysMaxL);
    if (B == 0) return VASR_OK;
    hipLaunchKernelGGL(collapse_keys_kernel, dim3(B), dim3(256), 0, as_stream(stream),
                       reinterpret_cast<const unsigned long long*>(keys), ld, slots, L, frames, blank, collapse, pred,
                       out_tokens, out_len, out_start, out_end);
    return launch_status("vasr_ctc_collapse_keys");
}

VASR_API int vasr_argmax_keys(const uint64_t* keys, int64_t ld, int slots, int rows, int32_t* out, void* stream) {
    using namespace vasr;
    VASR_CHECK_ARG(keys && out && rows >= 0 && slots >= 1 && ld >= slots, "vasr_argmax_keys: bad arguments");
    if (rows == 0) return VASR_OK;
    hipLaunchKernelGGL(argmax_keys_kernel, dim3((rows + 7) / 8), dim3(256), 0, as_stream(stream),
                       reinterpret_cast<const unsigned long long*>(keys), ld, slots, rows, out);
    return launch_status("vasr_argmax_keys");
}
