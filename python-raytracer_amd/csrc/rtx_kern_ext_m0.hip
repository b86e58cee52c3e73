// Hierarchy/texture render kernels with MESH = false (tile and sample-parallel mappings):
// a translation unit of their own so they compile in parallel with the rest of librtx.so.
#include <hip/hip_runtime.h>

#define RTX_EXT_TU 1
#include "rtx_kernels.h"
#include "rtx_split.h"
#include "rtx_launch.h"

namespace rtx {

hipError_t launch_render_ext_m0(int sel, const RenderLaunch& r, const Launch& L) {
    constexpr int B = kBlock<true>;
#define RTX_EXT_LAUNCH(S, C, J)                                                                          \
    if (r.spp)                                                                                           \
        hipLaunchKernelGGL((k_render_spp<false, S, true, C, J>), dim3(r.nblocks, r.nframes), dim3(B), r.lds_bytes,  \
                           r.stream, r.kp, L);                                                           \
    else                                                                                                 \
        hipLaunchKernelGGL((k_render<false, S, true, C, J>), dim3(r.nblocks, r.nframes), dim3(B), r.lds_bytes,      \
                           r.stream, r.kp, L)
#define RTX_EXT_CASE(n) \
    case n: RTX_EXT_LAUNCH(((n) & 8) != 0, ((n) & 2) != 0, ((n) & 1) != 0); break
    switch (sel & 11) {
        RTX_EXT_CASE(0); RTX_EXT_CASE(1); RTX_EXT_CASE(2); RTX_EXT_CASE(3);
        RTX_EXT_CASE(8); RTX_EXT_CASE(9); RTX_EXT_CASE(10); RTX_EXT_CASE(11);
    }
#undef RTX_EXT_CASE
#undef RTX_EXT_LAUNCH
    return hipGetLastError();
}

hipError_t launch_split_m0(int sel, int pass, const RenderLaunch& r, const Launch& L, const SplitBuf& sb) {
    constexpr int B = kBlock<true>;
    const bool sec = (sel & 8) != 0, cnt = (sel & 2) != 0, jit = (sel & 1) != 0;
    const dim3 g(r.nblocks), b(B);
    if (pass == 0) {
#define RTX_SPLIT_A(S, C, J) hipLaunchKernelGGL((k_split_trace<false, S, C, J>), g, b, r.lds_bytes, r.stream, r.kp, L, sb)
        if (sec) { if (cnt) { if (jit) RTX_SPLIT_A(true, true, true); else RTX_SPLIT_A(true, true, false); }
                   else { if (jit) RTX_SPLIT_A(true, false, true); else RTX_SPLIT_A(true, false, false); } }
        else { if (cnt) { if (jit) RTX_SPLIT_A(false, true, true); else RTX_SPLIT_A(false, true, false); }
               else { if (jit) RTX_SPLIT_A(false, false, true); else RTX_SPLIT_A(false, false, false); } }
#undef RTX_SPLIT_A
    } else if (pass == 1) {
        if (cnt) hipLaunchKernelGGL((k_split_shadow<false, true>), g, b, r.lds_bytes, r.stream, r.kp, L, sb);
        else hipLaunchKernelGGL((k_split_shadow<false, false>), g, b, r.lds_bytes, r.stream, r.kp, L, sb);
    } else {
        if (sec) hipLaunchKernelGGL((k_split_shade<false, true>), g, b, 0, r.stream, r.kp, L, sb);
        else hipLaunchKernelGGL((k_split_shade<false, false>), g, b, 0, r.stream, r.kp, L, sb);
    }
    return hipGetLastError();
}

}  // namespace rtx
