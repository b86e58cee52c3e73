// rtx_wavefront.hip — EXPERIMENT (not part of librtx.so): the SoA wavefront form of the
// render path, to measure against the megakernel (SURVEY §7 "benchmark both"). Built
// with the library's own sources (it includes rtx_api.hip, so it also exports the
// rtx_* entry points) by tools/wavefront/build.sh into _abl/librtx_wf.so.
//
// One frame = 1 + L + 1 launches over SoA buffers in HBM, 1-spp flat scenes only:
//   k_wf_gen      camera rays of every pixel (8x8 tiles per wave, as the megakernel),
//   k_wf_trace    per level: closest hit, shading + shadow rays, and for mirror /
//                 refractive hits the frame (lighting, material) and the next ray, which
//                 is queued (wave-aggregated atomics) for the next level,
//   k_wf_combine  the bottom-up clamp of each pixel's frames (scene.py:104-116), the
//                 sample mean and the framebuffer store.
// The per-ray functions are rtx_trace.h's, in the same order, so the frame is
// bit-identical to rtx_render's (tools/wavefront/bench_wf.py checks it).
#include "../../python-raytracer_amd/csrc/rtx_api.hip"

namespace wf {
using namespace rtx;

struct Bufs {
    float* o;            // [3][cap] ray origins
    float* d;            // [3][cap] directions
    uint8_t* in_shape;   // [cap]
    int32_t* q[2];       // ping-pong queues of pixel indices
    int32_t* counts;     // [kMaxDepth + 1] queue lengths per level
    float* frames;       // [kMaxDepth][4][cap] lighting RGB + material
    int32_t* nfr;        // [cap]
    float* tail;         // [3][cap]
    int64_t cap;
};

__global__ __launch_bounds__(256) void k_wf_gen(const KParams* __restrict__ Pp, Bufs B, int32_t tiles_x, int64_t nq) {
    const KParams& P = *Pp;
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t == 0) B.counts[0] = (int32_t)nq;
    if (t >= nq) return;
    const int32_t tile = (int32_t)(t >> 6), lane = (int32_t)(t & 63);
    const int32_t r = (tile / tiles_x) * 8 + (lane >> 3), c = (tile % tiles_x) * 8 + (lane & 7);
    if (r >= P.height || c >= P.ncols) { B.q[0][t] = -1; return; }
    const int64_t p = (int64_t)r * P.ncols + c;
    const int j = P.height - 1 - r;
    const f3 focal = pixel_focal(P, c, j);
    const f3 ddir = normalize(sub(focal, ld3(P.dof_o)));  // scene.py:58
    const f3 o = sample_origin<false>(P, c, j, 0, 0);
    const int64_t n = B.cap;
    B.o[p] = o.x; B.o[n + p] = o.y; B.o[2 * n + p] = o.z;
    B.d[p] = ddir.x; B.d[n + p] = ddir.y; B.d[2 * n + p] = ddir.z;
    B.in_shape[p] = 0;
    B.nfr[p] = 0;
    B.tail[p] = B.tail[n + p] = B.tail[2 * n + p] = 0.0f;
    B.q[0][t] = (int32_t)p;
}

template <bool MESH, bool SEC>
__global__ __launch_bounds__(256) void k_wf_trace(const KParams* __restrict__ Pp, Bufs B, int level) {
    const SceneView& S = Pp->S;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= B.counts[level]) return;
    const int32_t p = B.q[level & 1][i];
    if (p < 0) return;
    const int64_t n = B.cap;
    f3 o = mk(B.o[p], B.o[n + p], B.o[2 * n + p]);
    f3 d = mk(B.d[p], B.d[n + p], B.d[2 * n + p]);
    const bool in_shape = B.in_shape[p] != 0;
    const float time = Pp->times[0];
    Tally tl{};
    const HStack hs{nullptr, 1};
    HHit hh;
    // level 0 runs in the generator's tile order: the wave's tile has one primary bin
    int32_t bin = -1;
    if (level == 0) {
        const int32_t r = p / Pp->ncols, c = p % Pp->ncols;
        bin = primary_bin(S, r & ~7, c & ~7);
    }
    const Hit h = closest_hit<MESH, false, false>(S, o, d, time, tl, hs, hh, bin);
    if (h.obj == -1) return;  // miss -> black
    const Surface sf = resolve_hit<MESH, false>(S, h, hh, o, d, time);
    const DMat m = RTX_MAT(S, sf.mat);
    f3 nrm = sf.normal;
    bool chain = false, tir = false;
    f3 next_o = o, next_d = d;
    if (SEC && m.type == MAT_MIRROR) {
        const f3 rdir = reflect(d, nrm);
        next_o = add(sf.position, scale(rdir, 0.01f));
        next_d = rdir;
        chain = true;
    } else if (SEC && m.type == MAT_REFRACTIVE) {
        const float eta = in_shape ? m.eta_in : m.eta_out;
        if (in_shape) nrm = neg(nrm);
        const f3 rdir = refract(d, nrm, eta);
        tir = is_zero(rdir);
        next_o = add(sf.position, scale(rdir, 0.0001f));
        next_d = rdir;
        chain = true;
    }
    const f3 diffuse = ld3(m.diffuse);
    const f3 L = regular_lighting<MESH, false, false>(S, d, sf.position, nrm, m, diffuse, time, tl, hs);
    if (!SEC || !chain) {
        const f3 t = clamp01(L);
        B.tail[p] = t.x; B.tail[n + p] = t.y; B.tail[2 * n + p] = t.z;
        return;
    }
    float* fr = B.frames + (int64_t)level * 4 * n;
    fr[p] = L.x; fr[n + p] = L.y; fr[2 * n + p] = L.z; fr[3 * n + p] = __builtin_bit_cast(float, sf.mat);
    B.nfr[p] = level + 1;
    if (tir || level + 1 >= kMaxDepth) return;
    B.o[p] = next_o.x; B.o[n + p] = next_o.y; B.o[2 * n + p] = next_o.z;
    B.d[p] = next_d.x; B.d[n + p] = next_d.y; B.d[2 * n + p] = next_d.z;
    B.in_shape[p] = (m.type == MAT_REFRACTIVE ? !in_shape : false) ? 1 : 0;
    // wave-aggregated enqueue
    const uint64_t m64 = __ballot(1);
    const int lanes_before = __popcll(m64 & ((1ull << __lane_id()) - 1ull));
    int32_t base = 0;
    if (lanes_before == 0) base = atomicAdd(&B.counts[level + 1], (int32_t)__popcll(m64));
    base = __shfl(base, __builtin_ctzll(m64));
    B.q[(level + 1) & 1][base + lanes_before] = p;
}

__global__ __launch_bounds__(256) void k_wf_combine(const KParams* __restrict__ Pp, Bufs B, float* __restrict__ fb) {
    const KParams& P = *Pp;
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t npix = (int64_t)P.height * P.ncols;
    if (p >= npix) return;
    const int64_t n = B.cap;
    f3 tail = mk(B.tail[p], B.tail[n + p], B.tail[2 * n + p]);
    for (int k = B.nfr[p] - 1; k >= 0; --k) {
        const float* fr = B.frames + (int64_t)k * 4 * n;
        const f3 L = mk(fr[p], fr[n + p], fr[2 * n + p]);
        const DMat m = RTX_MAT(P.S, __builtin_bit_cast(int32_t, fr[3 * n + p]));
        tail = clamp01(add(scale(L, m.tint), scale(tail, m.omt)));
    }
    f3 colour = add(mk(0.0f, 0.0f, 0.0f), tail);
    colour = mk(sample_mean(P, colour.x), sample_mean(P, colour.y), sample_mean(P, colour.z));
    fb[3 * p] = colour.x; fb[3 * p + 1] = colour.y; fb[3 * p + 2] = colour.z;
}

Bufs g_bufs{};

}  // namespace wf

extern "C" int rtx_wf_render(rtx_scene* s, float* fb_dev, void* stream) {
    using namespace wf;
    if (!s || !s->cam_set) return fail(RTX_ERR_STATE, "rtx_wf_render: no scene/camera");
    const KParams& k = s->kp;
    if (s->has_ext || k.n_dof != 1 || k.n_aa != 1 || k.n_times != 1 || k.jitter != RTX_JITTER_OFF || k.col0 != 0)
        return fail(RTX_ERR_INVALID, "rtx_wf_render: 1-spp flat full frames only");
    const int32_t tiles_x = (k.ncols + 7) / 8, tiles_y = (k.height + 7) / 8;
    const int64_t nq = (int64_t)tiles_x * tiles_y * 64;
    const int64_t cap = std::max(nq, (int64_t)k.ncols * k.height);
    Bufs& B = g_bufs;
    if (B.cap < cap) {
        for (void* p : {(void*)B.o, (void*)B.d, (void*)B.in_shape, (void*)B.q[0], (void*)B.q[1], (void*)B.counts,
                        (void*)B.frames, (void*)B.nfr, (void*)B.tail})
            (void)hipFree(p);
        RTX_HIP(hipMalloc((void**)&B.o, 12 * cap));
        RTX_HIP(hipMalloc((void**)&B.d, 12 * cap));
        RTX_HIP(hipMalloc((void**)&B.in_shape, cap));
        RTX_HIP(hipMalloc((void**)&B.q[0], 4 * cap));
        RTX_HIP(hipMalloc((void**)&B.q[1], 4 * cap));
        RTX_HIP(hipMalloc((void**)&B.counts, 4 * (kMaxDepth + 1)));
        RTX_HIP(hipMalloc((void**)&B.frames, (size_t)16 * kMaxDepth * cap));
        RTX_HIP(hipMalloc((void**)&B.nfr, 4 * cap));
        RTX_HIP(hipMalloc((void**)&B.tail, 12 * cap));
        B.cap = cap;
    }
    hipStream_t st = (hipStream_t)stream;
    RTX_HIP(hipMemsetAsync(B.counts, 0, 4 * (kMaxDepth + 1), st));
    const unsigned gq = (unsigned)((nq + 255) / 256);
    hipLaunchKernelGGL(k_wf_gen, dim3(gq), dim3(256), 0, st, s->d_kp, B, tiles_x, nq);
    const int levels = s->has_secondary ? kMaxDepth : 1;
    for (int level = 0; level < levels; ++level) {
        // every level's queue is at most nq long; threads past the level's count exit
        if (s->has_mesh) {
            if (s->has_secondary) hipLaunchKernelGGL((k_wf_trace<true, true>), dim3(gq), dim3(256), 0, st, s->d_kp, B, level);
            else hipLaunchKernelGGL((k_wf_trace<true, false>), dim3(gq), dim3(256), 0, st, s->d_kp, B, level);
        } else {
            if (s->has_secondary) hipLaunchKernelGGL((k_wf_trace<false, true>), dim3(gq), dim3(256), 0, st, s->d_kp, B, level);
            else hipLaunchKernelGGL((k_wf_trace<false, false>), dim3(gq), dim3(256), 0, st, s->d_kp, B, level);
        }
    }
    const int64_t npix = (int64_t)k.ncols * k.height;
    hipLaunchKernelGGL(k_wf_combine, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, st, s->d_kp, B, fb_dev);
    RTX_HIP(hipGetLastError());
    return RTX_OK;
}
