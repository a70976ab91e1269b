// CTC prefix beam search on the device (reference velocity_asr/decode.py:128-217).
//
// One workgroup per utterance walks the frames.  The reference keys its beams by the
// collapsed prefix tuple; here each prefix is a node of a per-utterance trie (parent node,
// appended token) held in caller-owned workspace, so key equality is node equality: an
// extension prefix_i + (tok) equals a live beam j's prefix exactly when j's node has parent
// node_i and token tok.  Per frame:
//   1. log_softmax of the logit row (max, sum of exp, log) in fp32 into LDS;
//   2. for every live beam j, the merged record of its own key: its blank extension, its
//      repeat of the last token, and the extension of the beam whose node is j's parent --
//      max score, the first candidate in the reference's insertion order winning ties
//      (strict `<` update), and the key's insertion position = its first candidate's;
//   3. the W best candidates in the order of the reference's stable sort: score descending,
//      insertion position ascending, found as W successive block-wide maxima below the
//      previous winner (candidates = live keys + new extensions (i, tok), tok not blank, not
//      i's last token, not an existing node);
//   4. new extensions get fresh trie nodes.
// Scores are float64 sums of float32 log-probabilities, as the reference's Python floats.
#include "vasr_internal.h"

namespace vasr {
namespace {

constexpr int kBeamThreads = 256;
constexpr int kMaxBeam = 32;

struct Cand {
    double s;
    long long idx;  // insertion position; -1 = none
};

__device__ __forceinline__ bool better(const Cand& a, const Cand& b) {  // a before b in the sorted order
    if (a.idx < 0) return false;
    if (b.idx < 0) return true;
    return a.s > b.s || (a.s == b.s && a.idx < b.idx);
}

__device__ Cand block_best(Cand c, Cand* red) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        Cand d;
        d.s = __shfl_xor(c.s, o, 64);
        d.idx = __shfl_xor(c.idx, o, 64);
        if (better(d, c)) c = d;
    }
    if ((tid & 63) == 0) red[tid >> 6] = c;
    __syncthreads();
    Cand best = red[0];
    for (int w = 1; w < kBeamThreads / 64; ++w)
        if (better(red[w], best)) best = red[w];
    __syncthreads();
    return best;
}

__device__ float block_reduce_f(float v, float* red, bool is_max) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float u = __shfl_xor(v, o, 64);
        v = is_max ? fmaxf(v, u) : v + u;
    }
    if ((tid & 63) == 0) red[tid >> 6] = v;
    __syncthreads();
    float r = red[0];
    for (int w = 1; w < kBeamThreads / 64; ++w) r = is_max ? fmaxf(r, red[w]) : r + red[w];
    __syncthreads();
    return r;
}

__global__ __launch_bounds__(kBeamThreads) void ctc_beam_kernel(const float* __restrict__ logits, int64_t ld_row,
                                                               int64_t ld_utt, int L, int V, int W, int blank,
                                                               int32_t* __restrict__ trie, int64_t trie_stride,
                                                               int32_t* __restrict__ out_tokens,
                                                               int32_t* __restrict__ out_len, double* __restrict__ out_score,
                                                               int32_t* __restrict__ out_nbeams) {
    extern __shared__ __attribute__((aligned(16))) float lp[];  // V log-probabilities
    __shared__ double sc[kMaxBeam], msc[kMaxBeam];
    __shared__ long long midx[kMaxBeam];
    __shared__ int last[kMaxBeam], node[kMaxBeam], pnode[kMaxBeam], ptok[kMaxBeam], mlast[kMaxBeam];
    __shared__ int src_of[kMaxBeam];  // beam i whose extension reaches beam j's node, or -1
    __shared__ Cand red[kBeamThreads / 64];
    __shared__ float fred[kBeamThreads / 64];
    __shared__ Cand win[kMaxBeam];
    __shared__ int nb_s, nodes_s;

    const int b = blockIdx.x, tid = threadIdx.x;
    const float* lg = logits + (int64_t)b * ld_utt;
    int32_t* par = trie + (int64_t)b * trie_stride;           // parent node
    int32_t* tk = par + trie_stride / 2;                     // appended token
    const long long VP = (long long)V + 1;
    if (tid == 0) {
        sc[0] = 0.0;
        last[0] = -1;  // None
        node[0] = 0;
        pnode[0] = -1;
        ptok[0] = -1;
        par[0] = -1;
        tk[0] = -1;
        nb_s = 1;
        nodes_s = 1;
    }
    __syncthreads();

    for (int t = 0; t < L; ++t) {
        // 1. log_softmax of row t
        const float* row = lg + (int64_t)t * ld_row;
        float mx = -INFINITY;
        for (int v = tid; v < V; v += kBeamThreads) {
            const float x = row[v];
            lp[v] = x;
            mx = fmaxf(mx, x);
        }
        mx = block_reduce_f(mx, fred, true);
        float se = 0.f;
        for (int v = tid; v < V; v += kBeamThreads) se += expf(lp[v] - mx);
        se = block_reduce_f(se, fred, false);
        const float lse = logf(se);
        for (int v = tid; v < V; v += kBeamThreads) lp[v] = (lp[v] - mx) - lse;
        const int nb = nb_s;
        // 2. merged record of every live key
        if (tid < nb) {
            const int j = tid;
            int src = -1;
            for (int i = 0; i < nb; ++i)
                if (node[i] == pnode[j] && ptok[j] != last[i]) src = i;
            src_of[j] = src;
        }
        __syncthreads();
        if (tid < nb) {
            const int j = tid;
            // candidates in insertion order: (src, ptok) if src < j, (j, blank), (j, last), (src, ptok) if src > j
            Cand best{0.0, -1};
            int bl = -1;
            long long first = -1;
            auto offer = [&](double s, long long idx, int lt) {
                if (first < 0 || idx < first) first = idx;
                if (best.idx < 0 || s > best.s || (s == best.s && idx < best.idx)) {
                    best.s = s;
                    best.idx = idx;
                    bl = lt;
                }
            };
            const int src = src_of[j];
            offer(sc[j] + (double)lp[blank], (long long)j * VP, blank);
            if (last[j] >= 0 && last[j] != blank) offer(sc[j] + (double)lp[last[j]], (long long)j * VP + last[j] + 1, last[j]);
            if (src >= 0) offer(sc[src] + (double)lp[ptok[j]], (long long)src * VP + ptok[j] + 1, ptok[j]);
            msc[j] = best.s;
            midx[j] = first;
            mlast[j] = bl;
        }
        __syncthreads();
        // 3. W best candidates, each the maximum strictly below the previous winner
        const int ncand = nb * V;
        Cand prev{INFINITY, -2};
        int nw = 0;
        for (int r = 0; r < W; ++r) {
            Cand mine{0.0, -1};
            for (int c = tid; c < ncand; c += kBeamThreads) {
                const int i = c / V, tok = c - i * V;
                Cand k;
                if (tok == blank) {
                    k.s = msc[i];
                    k.idx = midx[i];
                } else {
                    if (tok == last[i]) continue;
                    bool existing = false;
                    for (int j = 0; j < nb; ++j)
                        if (src_of[j] == i && ptok[j] == tok) existing = true;
                    if (existing) continue;
                    k.s = sc[i] + (double)lp[tok];
                    k.idx = (long long)i * VP + tok + 1;
                }
                // below the previous winner in the sorted order
                if (prev.idx != -2 && !(prev.s > k.s || (prev.s == k.s && prev.idx < k.idx))) continue;
                if (better(k, mine)) mine = k;
            }
            const Cand w = block_best(mine, red);
            if (w.idx < 0) break;
            if (tid == 0) win[r] = w;
            prev = w;
            ++nw;
        }
        __syncthreads();
        // 4. new beam set, in winner order
        if (tid == 0) {
            double nsc[kMaxBeam];
            int nlast[kMaxBeam], nnode[kMaxBeam], npn[kMaxBeam], npt[kMaxBeam];
            int nodes = nodes_s;
            for (int r = 0; r < nw; ++r) {
                const long long idx = win[r].idx;
                const int i = (int)(idx / VP);
                const int pos = (int)(idx - (long long)i * VP);  // 0 = blank, tok + 1 otherwise
                int key_beam = -1;
                for (int j = 0; j < nb; ++j)
                    if (midx[j] == idx) key_beam = j;
                if (key_beam >= 0) {
                    const int j = key_beam;
                    nsc[r] = msc[j];
                    nlast[r] = mlast[j];
                    nnode[r] = node[j];
                    npn[r] = pnode[j];
                    npt[r] = ptok[j];
                } else {
                    const int tok = pos - 1;
                    nsc[r] = win[r].s;
                    nlast[r] = tok;
                    nnode[r] = nodes;
                    npn[r] = node[i];
                    npt[r] = tok;
                    par[nodes] = node[i];
                    tk[nodes] = tok;
                    ++nodes;
                }
            }
            for (int r = 0; r < nw; ++r) {
                sc[r] = nsc[r];
                last[r] = nlast[r];
                node[r] = nnode[r];
                pnode[r] = npn[r];
                ptok[r] = npt[r];
            }
            nb_s = nw;
            nodes_s = nodes;
        }
        __syncthreads();
    }
    // results: beams are already in the reference's final sorted order
    const int nb = nb_s;
    if (tid < nb) {
        int len = 0;
        for (int n = node[tid]; n > 0; n = par[n]) ++len;
        int32_t* o = out_tokens + ((int64_t)b * W + tid) * L;
        int k = len;
        for (int n = node[tid]; n > 0; n = par[n]) o[--k] = tk[n];
        out_len[(int64_t)b * W + tid] = len;
        out_score[(int64_t)b * W + tid] = sc[tid];
    }
    if (tid == 0) out_nbeams[b] = nb;
}

}  // namespace
}  // namespace vasr

VASR_API int64_t vasr_ctc_beam_workspace_elems(int L, int W) { return 2 * ((int64_t)L * W + 1); }

VASR_API int vasr_ctc_beam_search(const float* logits, int64_t ld_row, int64_t ld_utt, int B, int L, int V, int W,
                                  int blank, int32_t* trie, int32_t* out_tokens, int32_t* out_len, double* out_score,
                                  int32_t* out_nbeams, void* stream) {
    using namespace vasr;
    VASR_CHECK_ARG((logits || L == 0) && trie && out_tokens && out_len && out_score && out_nbeams,
                   "vasr_ctc_beam_search: null pointer");
    VASR_CHECK_ARG(B >= 0 && L >= 0 && V >= 1 && V <= 16384 && W >= 1 && W <= kMaxBeam && blank >= 0 && blank < V,
                   "vasr_ctc_beam_search: bad shape B=%d L=%d V=%d W=%d blank=%d", B, L, V, W, blank);
    if (B == 0) return VASR_OK;
    hipLaunchKernelGGL(ctc_beam_kernel, dim3(B), dim3(kBeamThreads), V * sizeof(float), as_stream(stream), logits,
                       ld_row, ld_utt, L, V, W, blank, trie, vasr_ctc_beam_workspace_elems(L, W), out_tokens, out_len,
                       out_score, out_nbeams);
    return launch_status("vasr_ctc_beam_search");
}
