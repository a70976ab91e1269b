// Pieces of the fused SSMBlock tail kernel (ssm_tail.hip: out_proj -> LN2 -> FFN): A operands
// as bf16 planes in LDS (split once per block), weights streamed global -> VGPRs in the
// v_mfma_f32_16x16x32_bf16 fragment layout.
#pragma once

#include "gemm_split.h"

namespace vasr {
namespace fused {

using gemm::bf16x8;
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int TD = 192;          // d_model
constexpr int TE = 384;          // FFN width = d_inner

// byte offset of bf16 element (r, col) in one plane: 8-element (16-B) chunks, chunk c of row r
// at c ^ (r & 15) (384-wide) or c ^ (r & 7) (192-wide): conflict-free ds_read_b128 fragment
// reads (16 rows x two chunk columns per lane group)
template <int WIDTH>
__device__ __forceinline__ int poff(int r, int col) {
    constexpr int SW = WIDTH == TE ? 15 : 7;
    return r * WIDTH * 2 + ((((col >> 3) ^ (r & SW))) << 4) + ((col & 7) << 1);
}

// v as NP bf16 planes: the exact three-way split, or (NP = 1, the bf16 model) v rounded to
// bf16 as vasr_linear_bf16 rounds its A operand
template <int NP>
__device__ __forceinline__ void split_store(char* plane0, int plane_bytes, int off, float v) {
    if constexpr (NP == 3) {
        __bf16 a, b, cc;
        gemm::split1(v, a, b, cc);
        *reinterpret_cast<__bf16*>(plane0 + off) = a;
        *reinterpret_cast<__bf16*>(plane0 + plane_bytes + off) = b;
        *reinterpret_cast<__bf16*>(plane0 + 2 * plane_bytes + off) = cc;
    } else {
        *reinterpret_cast<__bf16*>(plane0 + off) = (__bf16)v;
    }
}

// eight consecutive values of one row as NP planes (one 16-B chunk each)
template <int NP>
__device__ __forceinline__ void split_store8(char* plane0, int plane_bytes, int off, const float4& v0,
                                             const float4& v1) {
    if constexpr (NP == 3) {
        bf16x8 hi, mid, lo;
        gemm::split8(v0, v1, hi, mid, lo);
        *reinterpret_cast<bf16x8*>(plane0 + off) = hi;
        *reinterpret_cast<bf16x8*>(plane0 + plane_bytes + off) = mid;
        *reinterpret_cast<bf16x8*>(plane0 + 2 * plane_bytes + off) = lo;
    } else {
        const bf16x8 v = {(__bf16)v0.x, (__bf16)v0.y, (__bf16)v0.z, (__bf16)v0.w,
                          (__bf16)v1.x, (__bf16)v1.y, (__bf16)v1.z, (__bf16)v1.w};
        *reinterpret_cast<bf16x8*>(plane0 + off) = v;
    }
}

__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes done (prefetch stays in flight)
    __builtin_amdgcn_s_barrier();
}

// acc += A (NP planes) x W (NP planes) for one 16 x 16 tile, K = 32: the split-bf16 products,
// small terms first, then the leading hi * hi (the order of gemm_x3.hip)
template <int NP>
__device__ __forceinline__ floatx4 mac_tile(const bf16x8 (&a)[NP], const bf16x8 (&w)[NP], floatx4 v) {
    if constexpr (NP == 3) {
        v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], w[0], v, 0, 0, 0);
        v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], w[2], v, 0, 0, 0);
        v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], w[1], v, 0, 0, 0);
        v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], w[0], v, 0, 0, 0);
        v = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], w[1], v, 0, 0, 0);
    }
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], w[0], v, 0, 0, 0);
}

// the A fragment of one 16-row tile for a 32-k step: NP chunks of the plane image at `base`
// (planes of ROWS rows)
template <int NP, int WIDTH, int ROWS>
__device__ __forceinline__ void read_a(const char* base, int row, int ks, int q, bf16x8 (&a)[NP]) {
    constexpr int SW = WIDTH == TE ? 15 : 7;
    constexpr int PB = ROWS * WIDTH * 2;
#pragma unroll
    for (int pl = 0; pl < NP; ++pl)
        a[pl] = *reinterpret_cast<const bf16x8*>(base + pl * PB + row * WIDTH * 2 + (((4 * ks + q) ^ (row & SW)) << 4));
}

}  // namespace fused
}  // namespace vasr
