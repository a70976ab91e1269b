// The SiLU gate of SelectiveSSM (reference ssm.py:129, y * F.silu(z)) as every kernel that applies
// it evaluates it: the scan kernels' gated outputs and the z-in-tail block's fused tail
// (ssm_tail.hip) share this definition, so the two forms of a block give bitwise the same g.
#pragma once

#include "vasr_internal.h"

namespace vasr {

constexpr float kLog2e = 1.4426950408889634f;

// mode 2 (the default tree with fused multiply-adds): exp2 and reciprocal on the hardware units (a
// few ULP, like the scan's dA); other modes: the IEEE form.  Contraction off: z / (1 + e^-z).
template <int MODE>
__device__ __forceinline__ float silu_of(float z) {
#pragma clang fp contract(off)
    if constexpr (MODE == 2) return z * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(z * -kLog2e));
    else return z / (1.0f + expf(-z));
}

}  // namespace vasr
