// Tests only: every fp32 significand of selected binades through the product's fast
// correctly rounded sqrt / reciprocal (csrc/rtx_fastmath.h) vs IEEE sqrtf and 1.0f / x;
// and the shading's `x ** hardness` (csrc/rtx_trace.h spec_pow) on given inputs.
#include <hip/hip_runtime.h>
#include <cstdint>
#include "../../python-raytracer_amd/csrc/rtx_trace.h"

__global__ void k_check(int e, unsigned long long* bad) {
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;  // 24 bits: two binades
    if (m >= (1u << 24)) return;
    // x = 2^e * [1, 4): significand m & (2^23-1), extra exponent bit m >> 23
    const uint32_t bits = ((uint32_t)(127 + e + (m >> 23)) << 23) | (m & 0x7fffffu);
    const float x = __uint_as_float(bits);
    const float s_ref = sqrtf(x), s_fast = rtx::fm::sqrt_rn(x);
    const float r_ref = 1.0f / x, r_fast = rtx::fm::rcp_rn(x);
    if (__float_as_uint(s_ref) != __float_as_uint(s_fast)) atomicAdd(bad, 1ull);
    if (__float_as_uint(r_ref) != __float_as_uint(r_fast)) atomicAdd(bad + 1, 1ull);
    // harness self-check: the raw hardware approximations do differ somewhere
    if (__float_as_uint(r_ref) != __float_as_uint(__builtin_amdgcn_rcpf(x))) atomicAdd(bad + 2, 1ull);
}

extern "C" int rtx_mathcheck(int e, unsigned long long* out3) {
    unsigned long long* d = nullptr;
    if (hipMalloc(&d, 24) != hipSuccess) return -1;
    if (hipMemset(d, 0, 24) != hipSuccess) return -1;
    hipLaunchKernelGGL(k_check, dim3((1u << 24) / 256), dim3(256), 0, 0, e, d);
    if (hipMemcpy(out3, d, 24, hipMemcpyDeviceToHost) != hipSuccess) return -2;
    return hipFree(d) == hipSuccess ? 0 : -3;
}

// (float)spec_pow(x, hardness) as regular_lighting evaluates it (integer hardness; the
// scene-uniform loop length is the exponent's bit count, as rtx_scene_create sets it).
__global__ void k_spec_pow(const float* x, int64_t n, int hard, int bits, float* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    rtx::DMat m{};
    m.hard_is_int = 1;
    m.hard_int = hard;
    m.hardness = hard;
    out[i] = (float)rtx::spec_pow((double)x[i], m, bits);
}

// x: n host floats; out: n host floats. Hardness in [0, 4096] (rtx_scene_create's range).
extern "C" int rtx_powcheck(const float* x, int64_t n, int hard, float* out) {
    if (n <= 0 || hard < 0 || hard > 4096) return -4;
    int bits = 0;
    while (hard >> bits) ++bits;
    float *dx = nullptr, *dy = nullptr;
    if (hipMalloc(&dx, n * 4) != hipSuccess || hipMalloc(&dy, n * 4) != hipSuccess) return -1;
    if (hipMemcpy(dx, x, n * 4, hipMemcpyHostToDevice) != hipSuccess) return -2;
    hipLaunchKernelGGL(k_spec_pow, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, dx, n, hard, bits, dy);
    if (hipMemcpy(out, dy, n * 4, hipMemcpyDeviceToHost) != hipSuccess) return -2;
    return (hipFree(dx) == hipSuccess && hipFree(dy) == hipSuccess) ? 0 : -3;
}
