// Selective-scan launchers for state dim N = 64 (kernels: scan_kernels.h).
#include "scan_kernels.h"

namespace vasr {
namespace {
constexpr int N = 64;

template <int M, bool GATE = true>
int streaming(bool two, const float* xz, int64_t ld_xz, const float* dt, int64_t ld_dt, const float* bc, int64_t ld_bc,
              const float* A2, const float* D, float* out, int64_t ld_out, int B, int L, int Di, hipStream_t s) {
    return two ? npl2::launch_n<N, M, GATE>(xz, ld_xz, dt, ld_dt, bc, ld_bc, A2, D, out, ld_out, B, L, Di, s)
                   : npl4::launch_n<N, M, GATE>(xz, ld_xz, dt, ld_dt, bc, ld_bc, A2, D, out, ld_out, B, L, Di, s);
}

template <int M>
int chunked(bool two, const float* xz, int64_t ld_xz, const float* dt, int64_t ld_dt, const float* bc, int64_t ld_bc,
            const float* A2, const float* D, float* out, int64_t ld_out, int B, int L, int Di, float* ws_a, float* ws_b,
            hipStream_t s) {
    return two ? npl2::launch_chunked_n<N, M>(xz, ld_xz, dt, ld_dt, bc, ld_bc, A2, D, out, ld_out, B, L, Di, ws_a, ws_b, s)
                   : npl4::launch_chunked_n<N, M>(xz, ld_xz, dt, ld_dt, bc, ld_bc, A2, D, out, ld_out, B, L, Di, ws_a, ws_b, s);
}
}  // namespace

int scan_streaming_n64(bool two, int mode, const float* xz, int64_t ld_xz, const float* dt, int64_t ld_dt,
                        const float* bc, int64_t ld_bc, const float* A2, const float* D, float* out, int64_t ld_out,
                        int B, int L, int Di, hipStream_t s) {
    return mode == 0   ? streaming<0>(two, xz, ld_xz, dt, ld_dt, bc, ld_bc, A2, D, out, ld_out, B, L, Di, s)
           : mode == 2 ? streaming<2>(two, xz, ld_xz, dt, ld_dt, bc, ld_bc, A2, D, out, ld_out, B, L, Di, s)
                       : streaming<1>(two, xz, ld_xz, dt, ld_dt, bc, ld_bc, A2, D, out, ld_out, B, L, Di, s);
}

// the ungated form (tree modes): out = y + x D, z not read (the z-in-tail block)
int scan_ungated_n64(bool two, int mode, const float* x, int64_t ld_x, const float* dt, int64_t ld_dt, const float* bc,
                      int64_t ld_bc, const float* A2, const float* D, float* out, int64_t ld_out, int B, int L, int Di,
                      hipStream_t s) {
    return mode == 0 ? streaming<0, false>(two, x, ld_x, dt, ld_dt, bc, ld_bc, A2, D, out, ld_out, B, L, Di, s)
                     : streaming<2, false>(two, x, ld_x, dt, ld_dt, bc, ld_bc, A2, D, out, ld_out, B, L, Di, s);
}

int scan_chunked_n64(bool two, int mode, const float* xz, int64_t ld_xz, const float* dt, int64_t ld_dt,
                      const float* bc, int64_t ld_bc, const float* A2, const float* D, float* out, int64_t ld_out,
                      int B, int L, int Di, float* ws_a, float* ws_b, hipStream_t s) {
    return mode == 0 ? chunked<0>(two, xz, ld_xz, dt, ld_dt, bc, ld_bc, A2, D, out, ld_out, B, L, Di, ws_a, ws_b, s)
                     : chunked<2>(two, xz, ld_xz, dt, ld_dt, bc, ld_bc, A2, D, out, ld_out, B, L, Di, ws_a, ws_b, s);
}

int scan_split_n64(int mode, const float* xz, int64_t ld_xz, const float* dt, int64_t ld_dt, const float* bc,
                    int64_t ld_bc, const float* A2, const float* D, float* out, int64_t ld_out, int B, int L, int Di,
                    hipStream_t s) {
    return mode == 0 ? npl2::launch_split_n<N, 0>(xz, ld_xz, dt, ld_dt, bc, ld_bc, A2, D, out, ld_out, B, L, Di, s)
                     : npl2::launch_split_n<N, 2>(xz, ld_xz, dt, ld_dt, bc, ld_bc, A2, D, out, ld_out, B, L, Di, s);
}
}  // namespace vasr

#ifdef VASR_SCAN_STAMPS
VASR_API int vasr_diag_scan_stamps(void* buf) {  // diagnostic builds only (N = 64 kernels)
    return hipMemcpyToSymbol(HIP_SYMBOL(vasr::g_scan_stamps), &buf, sizeof(buf)) == hipSuccess ? VASR_OK : VASR_EINVAL;
}
#endif
