/*
 * vasr.h — C ABI of libvasr_hip.so, the MI355X (gfx950) kernels behind the
 * VELOCITY-ASR inference path.
 *
 * The reference (shaderko/velocity-asr) has no native layer at all: its hot path is
 * implicit ATen ops under Python modules.  Each entry point below replaces one of
 * those op groups; the reference file:line it stands in for is cited per function.
 * The one native-operator contract the reference itself defines is
 * `selective_scan_fn(u, delta, A, B, C, D, z, ...)` (velocity_asr/ssm.py:20-26,
 * call site ssm.py:326-332); vasr_ssm_scan_f32 is its replacement and also covers
 * the reference's default pure-PyTorch tree scan (ssm.py:173-295).
 *
 * Conventions (all functions):
 *   - All pointers are DEVICE pointers owned by the caller; the library never
 *     allocates or frees on these paths (graph-capturable).
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream).  Work is
 *     enqueued, never synchronised.
 *   - Matrices are row-major float32; `ld*` are row strides in ELEMENTS, `stride_*`
 *     are batch strides in elements.
 *   - Return 0 on success, a negative VASR_E* code for invalid arguments, or a
 *     positive hipError_t if a launch failed.  vasr_last_error() returns a
 *     thread-local description of the last failure.  No C++ exception crosses
 *     this boundary.
 *   - Functions are stateless and re-entrant.
 */
#ifndef VASR_H_
#define VASR_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VASR_ABI_VERSION 19

#define VASR_OK 0
#define VASR_EINVAL (-1)
#define VASR_EUNSUPPORTED (-2)

/* ABI version (== VASR_ABI_VERSION) and last-error text. */
int vasr_version(void);
const char* vasr_last_error(void);

/* Tuning options of the launchers (process-wide; not numerics: every setting computes the same
 * results).  Defaults are read once from the environment variable named per key; 0 = automatic.
 * vasr_set_option returns the previous value (value < 0 only queries), VASR_EINVAL otherwise. */
enum vasr_option {
    VASR_OPT_SCAN_LANES = 0, /* state indices per lane of vasr_ssm_scan_f32: 0, 2, 4 (VASR_SCAN_NPL)       */
    VASR_OPT_SCAN_CHUNK = 1, /* time steps per staged chunk of the streaming scan: 0, 16, 32 (VASR_SCAN_T) */
    VASR_OPT_TAIL_ROWS = 2,  /* token rows per fused-SSMBlock-tail workgroup: 0, 16, 32 (VASR_TAIL_ROWS)   */
    VASR_OPT_GEMM_ENGINE = 3, /* split-bf16 GEMM main loop: 0 auto, 1 LDS-ring tiles, 2 A-rows-stationary
                                 (K = 128 / 192, batch 1, unpaired epilogues) (VASR_GEMM_ENGINE)         */
    VASR_OPT_TAIL_WAVES = 4,  /* waves per fused-SSMBlock-tail workgroup: 0, 4, 6, 12 (VASR_TAIL_WAVES)    */
    VASR_OPT_SCAN_SPLIT = 5,  /* form of vasr_ssm_scan_chunked_f32: 0 auto, 1 three launches, 2 one launch
                                 (time split inside the workgroup) (VASR_SCAN_SPLIT)                     */
    VASR_OPT_DW_ROWS = 6      /* output rows per vasr_ln_dwconv_f32 workgroup: 0 auto, 4, 8, 16 (VASR_DW_ROWS) */
};
int vasr_set_option(int key, int value);

/* Diagnostics (no reference counterpart; bench.py's machine-state record).  A `blocks`-workgroup
 * launch of 256 threads, each running a dependent VALU chain of `iters` steps; per workgroup b:
 * out[3b] = the XCD (XCC_ID hardware register) it ran on, out[3b + 1] / out[3b + 2] = the shader
 * clock (s_memtime) / 100-MHz constant (s_memrealtime) ticks its wave 0 spent in the chain.  The
 * clock is out[3b+1] / out[3b+2] * 100 MHz; out[3b] == b % 8 checks the round-robin XCD dispatch
 * the kernels' XCD-aware block maps assume.  out: device, 3 * blocks int64. */
int vasr_probe_clock(int64_t* out, int blocks, int iters, void* stream);

/* ------------------------------------------------------------------ GEMM
 * C[b] = epilogue(A[b] (M x K) * W^T (K x N) + bias), W row-major [N][K] as in
 * nn.Linear, fp32 in / fp32 out (vasr_linear_x3_f32), or bf16 weights (vasr_linear_bf16).
 * Replaces every nn.Linear / Conv1d-as-GEMM on the path: in_proj, x_proj+dt_proj
 * (ssm.py:72-79, :105-113), out_proj (:90, :130), FFN (:394-400), temporal conv
 * (model.py:156-162), pool_proj (attention.py:35, :76), q/k/v/out (:107-110),
 * gated fusion (:183-218), CTC head (model.py:218-227), and the STFT as a
 * windowed-DFT GEMM (audio.py:104-115).
 */
enum vasr_epilogue {
    VASR_EPI_NONE = 0,          /* C = acc + bias                                      */
    VASR_EPI_GELU = 1,          /* C = gelu_erf(acc + bias)                            */
    VASR_EPI_SOFTPLUS_FROM = 2, /* C = acc + bias; softplus on columns >= n_out        */
    VASR_EPI_RESIDUAL = 3,      /* C = (acc + bias) + aux[b][row][col]                 */
    VASR_EPI_GELU_PE = 4,       /* C = gelu_erf(acc + bias) + aux[row][col] (pos. enc.) */
    VASR_EPI_PAIR_POWER = 5,    /* W rows paired in 32s (re|im): C[row][k] = re^2+im^2 */
    VASR_EPI_PAIR_FUSION = 6,   /* W rows paired (gate|global): gated fusion, see doc  */
    VASR_EPI_ARGMAX = 7         /* row argmax of acc + bias (after qparams), no logits write:
                                   C is (rows, ldc) uint64 partial keys, one per 32 columns
                                   (ldc >= ceil(N/32)), every slot written; decode with
                                   vasr_argmax_keys (ties -> first index, decode.py:46) */
};

typedef struct vasr_gemm_args {
    const float* A;
    int64_t lda, stride_a;
    const float* W;
    int64_t ldw;
    const float* bias;      /* [N] or NULL */
    float* C;
    int64_t ldc, stride_c;
    int32_t batch, M, N, K; /* M rows per batch */
    int32_t epilogue;       /* enum vasr_epilogue */
    const float* aux;       /* residual / positional table / paired partial product */
    int64_t ld_aux, stride_aux;
    const float* aux2;      /* PAIR_FUSION: local_proj bias [n_out] */
    int32_t n_out;          /* PAIR_*: output columns; SOFTPLUS_FROM: first softplus column */
    const float* qparams;   /* NULL, or per-column activation fake-quant {scale, zero_point,
                               qmin, qmax} (4 floats per column) applied to acc + bias before
                               the epilogue's function (QuantizedLinear / QuantizedConv1d
                               activation_quantizer, quantize.py:177-191, :252-266).
                               PAIR_FUSION: N entries in the paired column layout (gate |
                               global_proj) followed by n_out entries for local_proj.
                               A column whose scale is 0 is not quantized.  Not allowed
                               with PAIR_POWER. */
} vasr_gemm_args;

/* The fp32 GEMM (fp32 results to within accumulation order) on the bf16 matrix cores: fp32
 * operands are split exactly into three bf16 terms (x = hi + mid + lo, all 24 significant
 * bits) and the six products larger than 2^-25 |a||b| are accumulated in fp32 on
 * v_mfma_f32_32x32x16_bf16 — 2.67x the f32-input MFMA rate.  `w_split` holds W pre-split by
 * vasr_split_weights_bf16x3 (args->W is not read).
 */
int vasr_linear_x3_f32(const vasr_gemm_args* args, const uint16_t* w_split, void* stream);

/* Split W (N x K fp32, row stride ldw) into bf16 terms (hi, mid, lo) in the fragment-native
 * layout out[NT][KS][3][64][8] (NT = ceil(N/32), KS = Kp/16, Kp = K rounded up to 32):
 * element (n, k) of plane p is out[n/32][k/16][p][32*((k%16)/8) + n%32][k%8]; padding is
 * zero.  vasr_split_weights_elems(N, K) = 3 * 32*NT * Kp. */
int vasr_split_weights_bf16x3(const float* W, int64_t ldw, int N, int K, uint16_t* out, void* stream);
int64_t vasr_split_weights_elems(int N, int K);

/* The GEMM of a bf16 model (BASELINE config C3, `model.to(torch.bfloat16)`): W is bf16,
 * packed once by vasr_pack_weights_bf16 into the same fragment-native layout with one plane
 * (out[NT][KS][64][8], vasr_pack_weights_bf16_elems(N, K) = 32*NT * Kp elements); A stays
 * fp32 in HBM and is rounded to bf16 (round-to-nearest-even) as it enters the MFMA
 * (v_mfma_f32_32x32x16_bf16), accumulation and epilogues in fp32 — the reference's bf16
 * Linear (ssm.py, attention.py, model.py nn.Linear under bf16 parameters) with fp32
 * accumulation.  Same args and epilogues as vasr_linear_x3_f32. */
int vasr_linear_bf16(const vasr_gemm_args* args, const uint16_t* w_packed, void* stream);
int vasr_pack_weights_bf16(const uint16_t* W, int64_t ldw, int N, int K, uint16_t* out, void* stream);
int64_t vasr_pack_weights_bf16_elems(int N, int K);

/* ------------------------------------------------------------------ norms / conv
 * nn.LayerNorm over the last dim (C <= 1024), biased variance.  y may alias x.
 * Replaces every LayerNorm on the path (26 per forward).
 */
int vasr_layer_norm_f32(const float* x, int64_t ldx, const float* w, const float* b,
                        float* y, int64_t ldy, int rows, int C, float eps, void* stream);

/* Two LayerNorms in a row, one launch: y1 = LN(x; w1, b1, eps1), y2 = LN(y1; w2, b2, eps2), each
 * bitwise what vasr_layer_norm_f32 gives (y2 from y1's registers, not re-read).  Replaces the
 * local stack's final norm (LocalSSMProcessor.norm, reference ssm.py:504) followed by the
 * global context's query norm (HierarchicalGlobalContext.norm2, attention.py:307), which the
 * reference runs as two nn.LayerNorm calls.  y1 != y2; C <= 1024. */
int vasr_layer_norm_pair_f32(const float* x, int64_t ldx, const float* w1, const float* b1, float eps1,
                             float* y1, int64_t ldy1, const float* w2, const float* b2, float eps2,
                             float* y2, int64_t ldy2, int rows, int C, void* stream);

/* out[b][l][c] = x[b][l][c] + table[l][c] for x (B, L, C) contiguous (standalone
 * PositionalEncoding2D.forward, model.py:106-127; the model fuses it into the conv GEMM). */
int vasr_add_table_f32(const float* x, const float* table, float* out, int B, int L, int C,
                       void* stream);

/* SSMBlock pre-norm + causal depthwise conv (ssm.py:409-414, :377-383):
 * y[b,t,c] = bias[c] + sum_j conv_w[c][j] * LN(x)[b, t-(Kc-1)+j, c]  (zero for t<0).
 * x, y: (B, L, C) contiguous; conv_w: (C, Kc) contiguous; Kc <= 8.
 */
int vasr_ln_dwconv_f32(const float* x, const float* ln_w, const float* ln_b,
                       const float* conv_w, const float* conv_b, float* y,
                       int B, int L, int C, int Kc, float eps, void* stream);

/* vasr_ln_dwconv_f32 on LN0(x) without the LN0 launch: xo = LN0(x; pre_w, pre_b, pre_eps) (the
 * temporal binding's LayerNorm, reference model.py:200, applied to its conv + GELU + PE rows) is
 * formed in registers, stored once (the first SSM block's residual input) and fed to norm1 + the
 * causal conv: xo and y bitwise vasr_layer_norm_f32 followed by vasr_ln_dwconv_f32.  C = 192,
 * Kc = 4 (the model's); x, xo, y distinct. */
int vasr_ln_dwconv_prenorm_f32(const float* x, const float* pre_w, const float* pre_b, float pre_eps, float* xo,
                               const float* ln_w, const float* ln_b, const float* conv_w, const float* conv_b,
                               float* y, int B, int L, int C, int Kc, float eps, void* stream);

/* ------------------------------------------------------------------ selective scan
 * SelectiveSSM scan + D skip + SiLU gate (ssm.py:119-129):
 *   dA = exp(dt*A), dBx = x*(dt*B)
 *   mode 0 (scan_mode="parallel", the reference default): the reference's exclusive,
 *          mis-combined Blelloch tree prefix h (ssm.py:216-295), streamed in its exact
 *          float-operation order with an O(log L) block stack per state lane;
 *   mode 1 (scan_mode="sequential"): the true recurrence h_t = dA_t h_{t-1} + dBx_t
 *          (ssm.py:134-171);
 *   mode 2: the tree of mode 0 with each a*b + c as one fused multiply-add and
 *          dBx = (x*dt)*B (one rounding fewer per op; the model's default for
 *          scan_mode="parallel", VASR_SCAN_FMA=0 selects mode 0);
 *   out[b,t,d] = (sum_n h[b,t,d,n] C[b,t,n] + x[b,t,d] D[d]) * silu(z[b,t,d]).
 * x = xz[:, :, 0:Di], z = xz[:, :, Di:2Di]; B = bc[:, :, 0:N], C = bc[:, :, N:2N].
 * A2 = A * log2(e) (A = -exp(A_log), shared across Di).  N in {16, 32, 64, 128}: any other
 * state dim N' < 128 runs as the next size up with B and C zero-padded (columns N'..N-1 of each
 * half of bc) and A2 padded with 0 -- the padded states then stay exactly 0 and add nothing to
 * y, so the outputs are those of N' states (velocity_asr.ssm pads the projection weights with
 * zero rows, so the GEMM writes that layout).  Di a multiple of 4 * 64 * NPL / N channels per
 * workgroup (16 at N = 64, 8 at N = 128; host checks); L <= 8192.
 */
int vasr_ssm_scan_f32(const float* xz, int64_t ld_xz, const float* dt, int64_t ld_dt,
                      const float* bc, int64_t ld_bc, const float* A2, const float* D,
                      float* out, int64_t ld_out, int B, int L, int Di, int N, int mode,
                      void* stream);

/* The ungated form of the tree modes (0, 2) for the z-in-tail SSMBlock (ABI 15):
 *   out[b,t,d] = sum_n h[b,t,d,n] C[b,t,n] + x[b,t,d] D[d]
 * with x = x[:, :, 0:Di] (row stride ld_x >= Di; no z is read) and the other operands as
 * vasr_ssm_scan_f32; the same kernels and lane layout, so out * silu(z) (gate.h) is bitwise
 * vasr_ssm_scan_f32's output.  vasr_ssm_block_tail_gated_f32 applies the gate. */
int vasr_ssm_scan_ungated_f32(const float* x, int64_t ld_x, const float* dt, int64_t ld_dt,
                              const float* bc, int64_t ld_bc, const float* A2, const float* D,
                              float* out, int64_t ld_out, int B, int L, int Di, int N, int mode,
                              void* stream);

/* Chunk-parallel form of modes 0 and 2 for small launches (one utterance at a time, as
 * scripts/transcribe.py:69-78 and evaluate.py:91-98 run the model): time is cut at the
 * streaming kernel's 16-step chunks; pass 1 forms each chunk's up-sweep composite, pass 2
 * the composites of aligned blocks of 2^k chunks (the entries of the streaming kernel's
 * chunk-level stack), pass 3 folds each chunk's prefix from them and runs the chunk's tree
 * with the y reduction and gate.  Launches whose workgroups fit the CUs once (N <= 64, B * Di * N
 * / 128 <= 256; VASR_OPT_SCAN_SPLIT) run the same passes in ONE launch instead: a workgroup
 * owns one wave's channels and its waves split time into ranges of aligned 8-step chunk blocks
 * (2 state indices per lane; the workspace is then unused).  Same float operations as
 * vasr_ssm_scan_f32 with the same lane layout: bitwise equal outputs.
 * workspace: >= vasr_ssm_scan_workspace_floats(B, L, Di, N) floats, 16-byte aligned. */
int vasr_ssm_scan_chunked_f32(const float* xz, int64_t ld_xz, const float* dt, int64_t ld_dt,
                              const float* bc, int64_t ld_bc, const float* A2, const float* D,
                              float* out, int64_t ld_out, int B, int L, int Di, int N, int mode,
                              float* workspace, int64_t workspace_floats, void* stream);
int64_t vasr_ssm_scan_workspace_floats(int B, int L, int Di, int N);
/* 1 when vasr_ssm_scan_chunked_f32 runs this shape as the one-launch time-split form under the
 * current options (VASR_OPT_SCAN_SPLIT / VASR_OPT_SCAN_LANES), else 0: the launcher's own rule,
 * for hosts that choose between the streaming and chunked entry points (ABI 15). */
int vasr_ssm_scan_split_selected(int B, int L, int Di, int N);

/* ------------------------------------------------------------------ SSMBlock tail, fused
 * The tail of SSMBlock._forward_impl (ssm.py:415-425) in one launch for d_model D = 192 and
 * FFN width / d_inner E = 384:
 *   x1 = g @ Wo^T + x;  h = LayerNorm(x1; ln_w, ln_b, ln_eps);  f = gelu(h @ W1^T + b1);
 *   out = f @ W2^T + b2 + x1
 * with g (M, E) the gated scan output (row stride ldg), x (M, D) the block input, Wo = out_proj
 * (D x E, ssm.py:90), W1 = ffn.0 (E x D), W2 = ffn.3 (D x E) (ssm.py:394-400), each given as
 * vasr_split_weights16_bf16x3 planes.  x1 and f never leave the chip.  fp32-accurate (split
 * bf16 products, as vasr_linear_x3_f32). */
int vasr_ssm_block_tail_f32(const float* g, int64_t ldg, const float* x, int64_t ldx, const uint16_t* wo16,
                            const float* ln_w, const float* ln_b, float ln_eps, const uint16_t* w1_16,
                            const float* b1, const uint16_t* w2_16, const float* b2, float* out, int64_t ldo,
                            int M, int D, int E, void* stream);
/* The tail of the z-in-tail block (ABI 15): z = u @ W_z^T (W_z = in_proj rows Di..2Di-1 as
 * vasr_split_weights_bf16x3 planes; u (M, D) the in_proj input, row stride ldu) with the split
 * GEMM's exact product, g = yd * silu(z) with the gate of scan mode `mode` (0 or 2; yd = the
 * vasr_ssm_scan_ungated_f32 output, row stride ldy), then the tail above on g.  Bitwise the
 * output of vasr_ssm_scan_f32 + vasr_ssm_block_tail_f32 on the full projection; the projection
 * GEMM no longer writes z (E floats per token).  32-row workgroups of 12 waves. */
int vasr_ssm_block_tail_gated_f32(const float* yd, int64_t ldy, const float* u, int64_t ldu, const uint16_t* wz,
                                  int mode, const float* x, int64_t ldx, const uint16_t* wo16,
                                  const float* ln_w, const float* ln_b, float ln_eps, const uint16_t* w1_16,
                                  const float* b1, const uint16_t* w2_16, const float* b2, float* out, int64_t ldo,
                                  int M, int D, int E, void* stream);
/* The same tail for the bf16 model (C3): weights as one bf16 plane (vasr_pack_weights16_bf16 of
 * the bf16 parameters), activations rounded to bf16 at the MFMA input, fp32 accumulation and
 * fp32 LayerNorm / bias / GELU / residual -- the arithmetic of vasr_linear_bf16. */
int vasr_ssm_block_tail_bf16(const float* g, int64_t ldg, const float* x, int64_t ldx, const uint16_t* wo16,
                             const float* ln_w, const float* ln_b, float ln_eps, const uint16_t* w1_16,
                             const float* b1, const uint16_t* w2_16, const float* b2, float* out, int64_t ldo,
                             int M, int D, int E, void* stream);
/* The z-in-tail tail for the bf16 model (ABI 16): z = u @ W_z^T with W_z as one
 * vasr_pack_weights_bf16 plane (the bf16 in_proj rows Di..2Di-1) and u rounded to bf16 at the MFMA
 * input -- vasr_linear_bf16's exact product --, g = yd * silu(z) rounded to bf16 as the tail
 * above stages it, then that tail (Wo, W1, W2 as vasr_pack_weights16_bf16 planes).  Bitwise the
 * output of vasr_ssm_scan_f32 + vasr_ssm_block_tail_bf16 on vasr_linear_bf16's [x | z]. */
int vasr_ssm_block_tail_gated_bf16(const float* yd, int64_t ldy, const float* u, int64_t ldu, const uint16_t* wz,
                                   int mode, const float* x, int64_t ldx, const uint16_t* wo16,
                                   const float* ln_w, const float* ln_b, float ln_eps, const uint16_t* w1_16,
                                   const float* b1, const uint16_t* w2_16, const float* b2, float* out, int64_t ldo,
                                   int M, int D, int E, void* stream);
int vasr_pack_weights16_bf16(const uint16_t* W, int64_t ldw, int N, int K, uint16_t* out, void* stream);
int64_t vasr_pack_weights16_bf16_elems(int N, int K);
/* Split-bf16 planes of a (N, K) fp32 weight in the fragment layout of v_mfma_f32_16x16x32_bf16
 * ([ceil(N/16)][ceil(K/32)][3][64][8] bf16), vasr_split_weights16_elems(N, K) uint16 elements. */
int vasr_split_weights16_bf16x3(const float* W, int64_t ldw, int N, int K, uint16_t* out, void* stream);
int64_t vasr_split_weights16_elems(int N, int K);

/* ------------------------------------------------------------------ audio I/O (host)
 * load_audio (audio.py:22-62) without torchaudio.  Host functions on host memory (the only
 * entry points here that are not device work): they produce the waveform the front end reads.
 * vasr_flac_decode: a FLAC stream (torchaudio.load's FLAC path, audio.py:47) -> channel-major
 *   (channels, samples) float32 scaled by 2^(bits-1); out = NULL queries the sizes.  Frame
 *   CRCs are checked; errors return VASR_EINVAL with vasr_last_error().
 * vasr_resample_f32: torchaudio.transforms.Resample(orig, new) defaults (sinc_interp_hann,
 *   lowpass_filter_width 6, rolloff 0.99; audio.py:54-56), vasr_resample_length() outputs. */
int vasr_flac_decode(const uint8_t* data, int64_t n, float* out, int64_t out_cap, int* channels,
                     int* sample_rate, int* bits, int64_t* samples);
int64_t vasr_resample_length(int64_t n, int orig_sr, int new_sr);
int vasr_resample_f32(const float* x, int channels, int64_t n, int64_t ld_x, int orig_sr, int new_sr,
                      float* y, int64_t ld_y);

/* ------------------------------------------------------------------ mel front end
 * compute_mel_spectrogram (audio.py:65-143) is three launches:
 *  1. vasr_reflect_pad_f32: xp[b][0:S+2*pad] = reflect-padded audio (audio.py:100-101),
 *     rows of stride ld_out (>= S + 2*pad + n_fft); the tail is zero-filled.
 *  2. vasr_linear_x3_f32 with VASR_EPI_PAIR_POWER on rows of stride `hop` of xp against the
 *     Hann-windowed DFT matrix -> power[b][f][k] = |X_k|^2 (audio.py:104-115).
 *  3. vasr_mel_log_norm_f32: mel = fb @ power (audio.py:126), log(mel + 1e-10) (:129),
 *     per-(b, mel bin) (x - mean)/(std_unbiased + 1e-10) over frames (:132-135), written
 *     to out[b][frame_off + f][m] with batch stride out_stride.  The other frames of each
 *     utterance's padded slab of out_stride / n_mels frames are written as 0: the zero-framed
 *     (B, F + 2, n_mels) layout the stride-2 temporal conv GEMM reads as plain strided rows
 *     (model.py:156-162, padding 1), with no separate padding pass.  fb is passed in CSR form
 *     (rows = mel bins).
 */
int vasr_reflect_pad_f32(const float* audio, int64_t ld_audio, float* xp, int64_t ld_out,
                         int B, int S, int pad, void* stream);
int vasr_mel_log_norm_f32(const float* power, int64_t ld_power, int64_t stride_power,
                          const int32_t* fb_rowptr, const int32_t* fb_col, const float* fb_val,
                          float* out, int64_t out_stride, int frame_off, int B, int F, int n_mels,
                          int normalize, float* workspace, void* stream);
/* Utterances of different lengths in one zero-padded batch (the _var entry points below and
 * vasr_stft_power_400_var_f32, vasr_adaptive_pool_var_f32, vasr_pooled_attention_var_f32,
 * vasr_ctc_collapse_var): a device int32 array gives each utterance's own size, and every
 * value an utterance keeps is the one it gets alone (the reference runs one file at a time,
 * scripts/evaluate.py:91-98).  Here frames[b] <= F is utterance b's frame count: its
 * statistics cover its own frames only and its later frames are written as 0.  Needs
 * ld_power <= 256 and n_mels <= 85 (the chunked pass). */
int vasr_mel_log_norm_var_f32(const float* power, int64_t ld_power, int64_t stride_power,
                              const int32_t* fb_rowptr, const int32_t* fb_col, const float* fb_val,
                              float* out, int64_t out_stride, int frame_off, int B, int F, int n_mels,
                              int normalize, const int32_t* frames, float* workspace, void* stream);
/* workspace size of vasr_mel_log_norm_f32 in floats (log-mel rows + per-chunk fp64 partials) */
int64_t vasr_mel_workspace_floats(int B, int F, int n_mels);

/* Steps 1 + 2 in one launch for n_fft = 400, hop = 160 (the reference defaults, audio.py:15-18):
 * power[b][f][k] = |X_k|^2, k = 0..200, frame f of the reflect-padded audio (pad 200, computed
 * on the fly, no padded copy) times window[0:400], by a 400-point real FFT in LDS (200-point
 * complex FFT as 8 x 5 x 5 + real unpack).  F = S / 160 + 1 frames; power rows of stride ldp
 * (>= 201), batch stride stride_power (>= F * ldp).  Needs S > 200 (torch's reflect-pad rule). */
int vasr_stft_power_400_f32(const float* audio, int64_t ld_audio, int B, int S, const float* window,
                            float* power, int64_t ldp, int64_t stride_power, void* stream);
/* samples[b] (device, 200 < samples[b] <= S): utterance b's length inside the zero-padded
 * (B, S) batch; its reflect padding is taken at its own end, so its first samples[b]/160 + 1
 * frames equal those of the utterance alone (later frames: ignored by the _var mel pass). */
int vasr_stft_power_400_var_f32(const float* audio, int64_t ld_audio, int B, int S, const int32_t* samples,
                                const float* window, float* power, int64_t ldp, int64_t stride_power,
                                void* stream);
/* Write (B, F, C) rows into a zero-padded frame layout: out[b][off + f][c] = x[b][f][c]
 * and zero for the other out_frames - F frames (batch stride out_frames * C).  Feeds mel
 * to the stride-2 temporal conv, whose im2col rows are then plain strided rows (the public
 * model(mel) path; the device pipeline has vasr_mel_log_norm_f32 write the padded layout). */
int vasr_pad_frames_f32(const float* x, float* out, int out_frames, int off,
                        int B, int F, int C, void* stream);

/* ------------------------------------------------------------------ global context
 * F.adaptive_avg_pool1d over time (attention.py:71-73): bin i = [floor(iL/K), ceil((i+1)L/K)).
 * x: (B, L, C), out: (B, K, C).
 */
int vasr_adaptive_pool_f32(const float* x, float* out, int B, int L, int C, int K, void* stream);
/* Per utterance (device): its first lens[b] rows pooled into ks[b] bins (1 <= ks[b] <= lens[b]
 * <= L, ks[b] <= K), bins past ks[b] written as 0; x and out keep the strides L and K. */
int vasr_adaptive_pool_var_f32(const float* x, float* out, int B, int L, int C, int K, const int32_t* lens,
                               const int32_t* ks, void* stream);

/* LayerNorm(x; w, b, eps) of every row, then vasr_adaptive_pool_f32 (lens / ks null) or
 * vasr_adaptive_pool_var_f32 (both given) of the normalised rows, in one launch without the
 * normalised rows in memory: bitwise vasr_layer_norm_f32 followed by the pooling.  Replaces the
 * global SSM stack's final norm (reference ssm.py:555) followed by the second pooling level's
 * average pool (attention.py:303, AdaptivePool.forward :69-73).  C <= 1024. */
int vasr_ln_adaptive_pool_f32(const float* x, const float* w, const float* b, float eps, float* out, int B, int L,
                              int C, int K, const int32_t* lens, const int32_t* ks, void* stream);

/* Pooled multi-head cross attention core (attention.py:143-160), no mask:
 * out[b,t,h*hd:(h+1)*hd] = softmax(q_bth . k_bh^T / sqrt(hd)) v_bh over the Kp pooled keys.
 * q: (B, L, A) with row stride ld_q; kv: (B, Kp, 2A) [k | v]; out: (B, L, A) contiguous.
 * Kp <= 64, hd <= 64.
 */
int vasr_pooled_attention_f32(const float* q, int64_t ld_q, const float* kv, float* out,
                              int B, int L, int Kp, int heads, int head_dim, void* stream);
/* kps[b] (device, 1 <= kps[b] <= Kp): utterance b attends over its own first kps[b] keys. */
int vasr_pooled_attention_var_f32(const float* q, int64_t ld_q, const float* kv, float* out,
                                  int B, int L, int Kp, int heads, int head_dim, const int32_t* kps,
                                  void* stream);

/* ------------------------------------------------------------------ INT8 fake quantisation (C5)
 * FakeQuantize.forward in eval with calibrated buffers (quantize.py:79-97, :118-133):
 *   q = clamp(round_half_even(x / scale + zp), qmin, qmax); x_dq = (q - zp) * scale;
 *   y = x + (x_dq - x)
 * every operation IEEE-rounded in that order (bit-identical to torch's CPU evaluation).
 * x, y: (rows, cols) with row strides ldx, ldy (y may alias x).  scale / zero_point are
 * device arrays of `rows` entries if per_row != 0 (per-output-channel weights,
 * channel_dim 0) or of one entry (per-tensor).
 */
int vasr_fakequant_f32(const float* x, int64_t ldx, float* y, int64_t ldy, int rows, int cols,
                       const float* scale, const float* zero_point, int per_row, float qmin,
                       float qmax, void* stream);

/* Per-row min and max of x (rows, cols), NaN-propagating like torch.amin / amax: the
 * statistics FakeQuantize._update_scale_zp observes (quantize.py:99-116).  A per-tensor
 * range is two calls (rows of x, then the row results as one row). */
int vasr_minmax_f32(const float* x, int64_t ldx, int rows, int cols, float* out_min,
                    float* out_max, void* stream);

/* ------------------------------------------------------------------ CTC decode
 * argmax over V per row, ties -> first index (decode.py:46).
 */
int vasr_argmax_f32(const float* logits, int64_t ld, int rows, int V, int32_t* out, void* stream);

/* Partial keys of a VASR_EPI_ARGMAX GEMM ((rows, ld), `slots` = ceil(N/32) used) -> int32
 * argmax indices.  Keys are order-preserving (float bits, ~column) pairs, so the largest is
 * the largest logit with the smallest index.  The fused CTC head (model.py:223-227 +
 * decode.py:46) never writes the (rows, V) logits. */
int vasr_argmax_keys(const uint64_t* keys, int64_t ld, int slots, int rows, int32_t* out, void* stream);

/* CTC prefix beam search (decode.py:128-217, lm_scorer = None), one workgroup per utterance.
 * logits: (B, L, V) with row stride ld_row and utterance stride ld_utt; W <= 32 beams.
 * Outputs per utterance b, beam r < out_nbeams[b] (sorted as the reference returns them):
 * out_tokens[(b*W + r)*L + 0 .. out_len[b*W + r]), out_score[b*W + r] (float64 sum of the
 * float32 log-softmax values, as the reference's Python floats).  trie: caller workspace of
 * B * vasr_ctc_beam_workspace_elems(L, W) int32. */
int vasr_ctc_beam_search(const float* logits, int64_t ld_row, int64_t ld_utt, int B, int L, int V,
                         int W, int blank, int32_t* trie, int32_t* out_tokens, int32_t* out_len,
                         double* out_score, int32_t* out_nbeams, void* stream);
int64_t vasr_ctc_beam_workspace_elems(int L, int W);

/* Greedy CTC collapse per utterance (decode.py:51-69, :89-123): drop blank (and reset
 * prev), skip repeats of prev if collapse != 0.  out_tokens (B, L) holds each
 * utterance's kept tokens left-aligned, out_len (B) their counts.  If out_start /
 * out_end are non-NULL they receive the (start_frame, end_frame) of each kept token
 * with the semantics of ctc_greedy_decode_with_timestamps (collapse must be 1).
 */
int vasr_ctc_collapse(const int32_t* pred, int B, int L, int blank, int collapse,
                      int32_t* out_tokens, int32_t* out_len, int32_t* out_start,
                      int32_t* out_end, void* stream);
/* frames[b] (device): utterance b collapses its own first frames[b] rows; values outside [0, L]
 * are clamped to it (no row past L is read or written). */
int vasr_ctc_collapse_var(const int32_t* pred, int B, int L, const int32_t* frames, int blank, int collapse,
                          int32_t* out_tokens, int32_t* out_len, int32_t* out_start, int32_t* out_end,
                          void* stream);
/* Greedy decode straight from a VASR_EPI_ARGMAX GEMM's keys (B * L rows, `slots` used, row
 * stride ld): vasr_argmax_keys then vasr_ctc_collapse[_var] in ONE launch, one workgroup per
 * utterance (the predictions stay in LDS; the fused CTC head + decode.py:46-69 of the
 * reference's greedy path).  frames: NULL or device int32[B] as in vasr_ctc_collapse_var;
 * pred: NULL or device int32[B * L] to also receive the per-frame argmax.  L <= 8192. */
int vasr_ctc_collapse_keys(const uint64_t* keys, int64_t ld, int slots, int B, int L, const int32_t* frames,
                           int blank, int collapse, int32_t* pred, int32_t* out_tokens, int32_t* out_len,
                           int32_t* out_start, int32_t* out_end, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* VASR_H_ */
