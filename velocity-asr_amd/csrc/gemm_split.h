// Exact fp32 -> 3 x bf16 operand splitting shared by the split-bf16 GEMM main loops
// (gemm_x3.hip: LDS-ring tiles; gemm_panel.hip: LDS-resident weight panels).
#pragma once

#include "vasr_internal.h"

namespace vasr {
namespace gemm {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// x = hi + mid + lo, each a bf16 (RNE); the residuals are exact in fp32.
__device__ __forceinline__ void split1(float v, __bf16& hi, __bf16& mid, __bf16& lo) {
    hi = (__bf16)v;
    const float r1 = v - (float)hi;
    mid = (__bf16)r1;
    lo = (__bf16)(r1 - (float)mid);
}

__device__ __forceinline__ void split8(const float4& x0, const float4& x1, bf16x8& hi, bf16x8& mid, bf16x8& lo) {
    const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        __bf16 a, b, c;
        split1(v[j], a, b, c);
        hi[j] = a;
        mid[j] = b;
        lo[j] = c;
    }
}

}  // namespace gemm
}  // namespace vasr
