// Correctly rounded fp32 sqrt, reciprocal and normalize from the hardware approximations.
//
// GLM's normalize is v * (1 / sqrt(dot(v, v))) with IEEE fp32 sqrt and division (the
// reference's PyGLM numerics). The compiler's IEEE sequences handle
// every input class (subnormal scaling, division scale/fixup); for arguments in
// [2^-100, 2^100] the same results come from:
//  - sqrt: v_sqrt_f32 (<= 1 ulp) and the fma test of its two neighbours (the fix-up LLVM
//    uses after its own subnormal scaling);
//  - reciprocal: v_rcp_f32 (<= 1 ulp) and one fma Newton step, r + r (1 - s r); 1 - s r is
//    exact in the fma, and the result is checked against IEEE division for every fp32
//    significand over a range of binades on the MI355X (tests/test_gpu_fastmath.py).
// normalize() takes this path when every lane's dot lies in the range (wave-uniform
// branch) and the IEEE sequence otherwise, so results are identical for all inputs.
#pragma once

namespace rtx {
namespace fm {
constexpr float kLo = 0x1p-100f, kHi = 0x1p100f;
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ float sqrt_rn(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __int_as_float(__float_as_int(s) - 1);
    const float sp = __int_as_float(__float_as_int(s) + 1);
    const float rm = __builtin_fmaf(-sm, s, x);
    const float rp = __builtin_fmaf(-sp, s, x);
    float r = rm <= 0.0f ? sm : s;
    return rp > 0.0f ? sp : r;
}
__device__ __forceinline__ float rcp_rn(float s) {
    const float r = __builtin_amdgcn_rcpf(s);
    const float e = __builtin_fmaf(-s, r, 1.0f);
    return __builtin_fmaf(r, e, r);
}
#else
// host builds (the tests-only host emulation): IEEE operations
__host__ __device__ inline float sqrt_rn(float x) { return __builtin_sqrtf(x); }
__host__ __device__ inline float rcp_rn(float s) { return 1.0f / s; }
#endif
}  // namespace fm
}  // namespace rtx
