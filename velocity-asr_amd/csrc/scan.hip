// C ABI of the selective scan (include/vasr.h): argument checks, lane-layout choice and
// dispatch to the per-state-dim launchers (scan_n<N>.hip; kernels in scan_kernels.h).
#include "scan_kernels.h"

namespace vasr {
namespace {
// Lane layout of the streaming kernel (see vasr_ssm_scan_f32): 2 state indices per lane below 512
// waves at 4 per lane, unless vasr_set_option(VASR_OPT_SCAN_LANES, 2|4) forces one.  Shared by the
// gated and ungated entry points: the layouts differ in the order of the y = sum_n h C sums.
bool streaming_two(int B, int Di, int N) {
    const int npl_env = option(VASR_OPT_SCAN_LANES);  // vasr_set_option / env VASR_SCAN_NPL
    const long waves4 = (long)B * Di * N / 256;
    return npl_env == 2 || (npl_env != 4 && waves4 < 512);
}
}  // namespace
}  // namespace vasr

VASR_API int vasr_ssm_scan_f32(const float* xz, int64_t ld_xz, const float* dt, int64_t ld_dt, const float* bc,
                               int64_t ld_bc, const float* A2, const float* D, float* out, int64_t ld_out, int B,
                               int L, int Di, int N, int mode, void* stream) {
    using namespace vasr;
    VASR_CHECK_ARG(xz && dt && bc && A2 && D && out, "vasr_ssm_scan_f32: null pointer");
    VASR_CHECK_ARG(mode >= 0 && mode <= 2,
                   "vasr_ssm_scan_f32: mode must be 0 (tree), 1 (recurrence) or 2 (tree, fused multiply-adds)");
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
    // Lane layout (B * Di * N / 256 waves at 4 state indices per lane).  A lone wave issues a
    // VALU instruction every ~8.5 cycles; two or more per SIMD reach the SIMD's rate.  2 per lane
    // (twice the waves, ~25 % more VALU per element) is faster ALONE below 2 waves per SIMD: the
    // bench's 16-clip launch 76 vs 81 us, 79 vs 86 us in the graph (32 clips: 134 vs 114 us).
    // But its extra VALU issue slows the other utterance group's concurrent GEMMs: end to end
    // C2 +1.3 %, C3 (bf16) -2.6 %, C4 (30 s) -8.5 % (profiles/r02_npl/).  So 2 per lane is kept
    // for launches under half a wave per SIMD (B <= 4 at Di 384, N 64: 62 vs 69 us), where the
    // shorter serial chain per wave wins.  vasr_set_option(VASR_OPT_SCAN_LANES, 2|4) (env VASR_SCAN_NPL) forces one.
    const bool two = streaming_two(B, Di, N);
#define VASR_SCAN_N(NN) scan_streaming_n##NN(two, mode, xz, ld_xz, dt, ld_dt, bc, ld_bc, A2, D, out, ld_out, B, L, Di, s)
    switch (N) {
        case 16: return VASR_SCAN_N(16);
        case 32: return VASR_SCAN_N(32);
        case 64: return VASR_SCAN_N(64);
        case 128: return VASR_SCAN_N(128);  // 4 state indices per lane only
        default:
            set_error("vasr_ssm_scan_f32: state dim N=%d not supported (16, 32, 64, 128; zero-pad B, C and A2 to the "
                      "next one: padded states stay 0 and add nothing to y)", N);
            return VASR_EUNSUPPORTED;
    }
#undef VASR_SCAN_N
}

VASR_API int vasr_ssm_scan_ungated_f32(const float* x, int64_t ld_x, const float* dt, int64_t ld_dt, const float* bc,
                                       int64_t ld_bc, const float* A2, const float* D, float* out, int64_t ld_out, int B,
                                       int L, int Di, int N, int mode, void* stream) {
    using namespace vasr;
    VASR_CHECK_ARG(x && dt && bc && A2 && D && out, "vasr_ssm_scan_ungated_f32: null pointer");
    VASR_CHECK_ARG(mode == 0 || mode == 2, "vasr_ssm_scan_ungated_f32: mode must be 0 or 2 (tree modes)");
    VASR_CHECK_ARG(B >= 0 && L >= 0 && L <= 8192 && Di > 0, "vasr_ssm_scan_ungated_f32: bad shape B=%d L=%d Di=%d", B,
                   L, Di);
    VASR_CHECK_ARG(ld_x % 4 == 0 && ld_dt % 4 == 0 && ld_bc % 4 == 0 && Di % 4 == 0,
                   "vasr_ssm_scan_ungated_f32: leading dims and Di must be multiples of 4");
    VASR_CHECK_ARG(ld_x >= Di && ld_dt >= Di && ld_bc >= 2 * N && ld_out >= Di,
                   "vasr_ssm_scan_ungated_f32: leading dims too small");
    VASR_CHECK_ARG(((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(dt) |
                     reinterpret_cast<uintptr_t>(bc)) & 15) == 0,
                   "vasr_ssm_scan_ungated_f32: inputs must be 16-byte aligned");
    if (B == 0 || L == 0) return VASR_OK;
    hipStream_t s = as_stream(stream);
    const bool two = streaming_two(B, Di, N);
#define VASR_SCAN_U(NN) scan_ungated_n##NN(two, mode, x, ld_x, dt, ld_dt, bc, ld_bc, A2, D, out, ld_out, B, L, Di, s)
    switch (N) {
        case 16: return VASR_SCAN_U(16);
        case 32: return VASR_SCAN_U(32);
        case 64: return VASR_SCAN_U(64);
        case 128: return VASR_SCAN_U(128);
        default:
            set_error("vasr_ssm_scan_ungated_f32: state dim N=%d not supported (16, 32, 64, 128)", N);
            return VASR_EUNSUPPORTED;
    }
#undef VASR_SCAN_U
}

VASR_API int64_t vasr_ssm_scan_workspace_floats(int B, int L, int Di, int N) {
    if (B <= 0 || L <= 0 || Di <= 0 || N <= 0) return 0;
    return 4 * (int64_t)B * ((L + 15) / 16) * Di * N;  // two arrays of [B][2 * nchunks][Di][N]
}

VASR_API int vasr_ssm_scan_split_selected(int B, int L, int Di, int N) {
    using namespace vasr;
    const int split_opt = option(VASR_OPT_SCAN_SPLIT);
    const bool split_ok = N <= 64 && N > 0 && option(VASR_OPT_SCAN_LANES) != 4;
    return split_ok && (split_opt == 2 || (split_opt == 0 && (int64_t)B * Di * N / 128 <= 256 && L <= 512)) ? 1 : 0;
}

VASR_API int vasr_ssm_scan_chunked_f32(const float* xz, int64_t ld_xz, const float* dt, int64_t ld_dt,
                                       const float* bc, int64_t ld_bc, const float* A2, const float* D, float* out,
                                       int64_t ld_out, int B, int L, int Di, int N, int mode, float* workspace,
                                       int64_t workspace_floats, void* stream) {
    using namespace vasr;
    VASR_CHECK_ARG(xz && dt && bc && A2 && D && out, "vasr_ssm_scan_chunked_f32: null pointer");
    VASR_CHECK_ARG(mode == 0 || mode == 2, "vasr_ssm_scan_chunked_f32: mode must be 0 or 2 (tree modes)");
    VASR_CHECK_ARG(B >= 0 && L >= 0 && L <= 8192 && Di > 0, "vasr_ssm_scan_chunked_f32: bad shape B=%d L=%d Di=%d", B,
                   L, Di);
    VASR_CHECK_ARG(ld_xz % 4 == 0 && ld_dt % 4 == 0 && ld_bc % 4 == 0 && Di % 4 == 0,
                   "vasr_ssm_scan_chunked_f32: leading dims and Di must be multiples of 4");
    VASR_CHECK_ARG(ld_xz >= 2 * Di && ld_dt >= Di && ld_bc >= 2 * N && ld_out >= Di,
                   "vasr_ssm_scan_chunked_f32: leading dims too small");
    VASR_CHECK_ARG(((reinterpret_cast<uintptr_t>(xz) | reinterpret_cast<uintptr_t>(dt) |
                     reinterpret_cast<uintptr_t>(bc) | reinterpret_cast<uintptr_t>(workspace)) & 15) == 0,
                   "vasr_ssm_scan_chunked_f32: inputs and workspace must be 16-byte aligned");
    if (B == 0 || L == 0) return VASR_OK;
    const int64_t need = vasr_ssm_scan_workspace_floats(B, L, Di, N);
    VASR_CHECK_ARG(workspace != nullptr && workspace_floats >= need,
                   "vasr_ssm_scan_chunked_f32: workspace of %lld floats, %lld needed", (long long)workspace_floats,
                   (long long)need);
    VASR_CHECK_ARG(((int64_t)Di * N / 2) % 16 == 0 && (L + 15) / 16 - 1 <= 511,
                   "vasr_ssm_scan_chunked_f32: needs Di * N / 2 divisible by 16 and L <= 8192");
    float* ws_a = workspace;
    float* ws_b = workspace + need / 2;
    hipStream_t s = as_stream(stream);
    // Form: one launch (time split inside a workgroup of one wave's channels, 2 state indices per
    // lane, N <= 64) while its B * Di / DPW workgroups fit the CUs once (~157 KiB of LDS each) and
    // L <= 512, else the three launches below.  The one launch is VALU-bound on B * Di * N / 128
    // CUs (192 at the model's B = 1): 16.2-16.8 vs 18 us for the three launches at L = 501, but
    // slower from L ~ 1000 (one-utterance 30 s: 0.806 vs 0.777 ms; profiles/r05ap).
    // vasr_set_option(VASR_OPT_SCAN_SPLIT, 1|2) (env VASR_SCAN_SPLIT) forces them (three | one).
    // A forced 4-states-per-lane layout takes the three launches.
    if (vasr_ssm_scan_split_selected(B, L, Di, N)) {
        switch (N) {
            case 16: return scan_split_n16(mode, xz, ld_xz, dt, ld_dt, bc, ld_bc, A2, D, out, ld_out, B, L, Di, s);
            case 32: return scan_split_n32(mode, xz, ld_xz, dt, ld_dt, bc, ld_bc, A2, D, out, ld_out, B, L, Di, s);
            case 64: return scan_split_n64(mode, xz, ld_xz, dt, ld_dt, bc, ld_bc, A2, D, out, ld_out, B, L, Di, s);
            default: break;  // other N: the three launches report it
        }
    }
    // lane layout: 4 state indices per lane (the chunk-parallel grid has waves enough; 2 per lane
    // measured slower: 40.0 vs 35.9 us at B = 1, L = 501 and 43.4 vs 37.7 at L = 1501);
    // VASR_OPT_SCAN_LANES = 2 forces the other (outputs are bitwise those of the streaming kernel with
    // the same layout; the layouts differ in the order of the y = sum_n h C partial sums)
    const bool two = option(VASR_OPT_SCAN_LANES) == 2;
#define VASR_SCAN_C(NN) \
    scan_chunked_n##NN(two, mode, xz, ld_xz, dt, ld_dt, bc, ld_bc, A2, D, out, ld_out, B, L, Di, ws_a, ws_b, s)
    switch (N) {
        case 16: return VASR_SCAN_C(16);
        case 32: return VASR_SCAN_C(32);
        case 64: return VASR_SCAN_C(64);
        case 128: return VASR_SCAN_C(128);
        default:
            set_error("vasr_ssm_scan_chunked_f32: state dim N=%d not supported (16, 32, 64, 128)", N);
            return VASR_EUNSUPPORTED;
    }
#undef VASR_SCAN_C
}
