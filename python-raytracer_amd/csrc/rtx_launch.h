// rtx_launch.h — launchers of the precompiled hierarchy/texture (X) render kernels, which
// live in their own translation units (rtx_kern_ext_m0.hip / _m1.hip, by MESH) so the
// library's largest kernels compile in parallel.
#pragma once

#include <hip/hip_runtime.h>

namespace rtx {
struct KParams;
struct Launch;

struct RenderLaunch {
    const KParams* kp;
    unsigned nblocks;
    unsigned nframes;  // gridDim.y: frames of a batched launch (rtx_render_frames)
    size_t lds_bytes;  // dynamic LDS (hierarchy stacks)
    hipStream_t stream;
    bool spp;          // sample-parallel mapping (render_body_spp)
};

// sel: (SEC ? 8 : 0) | (COUNT ? 2 : 0) | (JITTER ? 1 : 0); returns hipGetLastError().
hipError_t launch_render_ext_m0(int sel, const RenderLaunch& r, const Launch& L);
hipError_t launch_render_ext_m1(int sel, const RenderLaunch& r, const Launch& L);

// The split passes of rtx_split.h (pass 0 trace, 1 shadow, 2 shade) with r.nblocks blocks.
struct SplitBuf;
hipError_t launch_split_m0(int sel, int pass, const RenderLaunch& r, const Launch& L, const SplitBuf& sb);
hipError_t launch_split_m1(int sel, int pass, const RenderLaunch& r, const Launch& L, const SplitBuf& sb);
}  // namespace rtx
