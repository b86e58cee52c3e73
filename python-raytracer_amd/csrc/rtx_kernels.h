// rtx_kernels.h — device side of the render path: per-frame parameters, the per-pixel
// sample loops (scene.py:47-79) and the kernels of librtx.so. Compiled into librtx.so
// (rtx_api.hip) and, for scene-specialized kernels, at run time by hiprtc (rtx_jit.cpp),
// which only needs render_body.
#pragma once

#include "rtx_trace.h"
#if defined(__HIPCC_RTC__)
#include "rtx.h"  // handed to hiprtc by name
#else
#include "../../include/rtx.h"
#endif

namespace rtx {

struct KParams {
    SceneView S;
    // camera tables (device)
    cptr<float> xs;
    cptr<float> ys;
    cptr<float> dof_o;   // [n_dof][3]
    cptr<float> aa_o;    // [n_dof][n_aa][3]
    cptr<float> times;   // [n_times] fp32
    cptr<float> noise;   // replay jitter
    float pos[4], u[4], v[4], dw[4];
    float focal, divisor, jscale, inv_divisor;
    int32_t div_pow2, pad0, pad1, pad2;
    int32_t width, height, col0, ncols;
    int32_t n_dof, n_aa, n_times, jitter;
    uint32_t seed_lo, seed_hi;
    // tools/wave_timeline.py only (kernels built with RTX_WAVE_LOG): per wave, its start
    // and end (s_memrealtime, 100 MHz) and hardware ids, 4 x uint64 per wave of the launch
    unsigned long long* wave_log;
    // measured tile schedule (RTX_TILE_SCHED kernels, rtx_api.hip tile_schedule): the
    // dispatch order of a whole frame's 8x8 tiles (wave w renders tile tile_perm[w]) and,
    // while it is measured, each tile's wave duration (s_memrealtime ticks); tile_n entries
    cptr<int32_t> tile_perm;
    unsigned int* tile_time;
    int32_t tile_n;
    // RTX_PRIM_ORIGIN kernels (one sample, no jitter, static scene: every primary ray starts
    // at aa_o[0]): its origin-only plane and sphere terms, computed by rtx_camera_set with
    // closest_hit's fp32 operations (po_valid: computed)
    int32_t po_valid;
    float po_pnum[4];
    float po_soc[16][3];
    float po_sq[16];
};

template <bool COUNT>
__device__ __forceinline__ void flush_tally(const Tally& tl, unsigned long long* counters, bool active) {
    if (!COUNT || counters == nullptr) return;
    uint32_t vals[RTX_COUNTERS] = {};
#pragma unroll
    for (int k = 0; k < kMaxDepth; ++k) vals[k] = active ? tl.cast[k] : 0u;
    vals[RTX_CNT_SHADOW] = active ? tl.shadow : 0u;
    vals[RTX_CNT_SHADE] = active ? tl.shade : 0u;
    vals[RTX_CNT_TRI] = active ? tl.tri : 0u;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < RTX_COUNTERS; ++k) {
        unsigned long long s = vals[k];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
        if (lane == 0 && s) atomicAdd(&counters[k], s);
    }
}

// Sample counts per pixel; the scene-specialized kernels pin them (with the camera's
// values) so the sample loops of the 1-spp configs disappear.
#ifdef RTX_FIXED_SAMPLES
#define RTX_NDOF(P) RTX_FIXED_NDOF
#define RTX_NAA(P) RTX_FIXED_NAA
#define RTX_NTIMES(P) RTX_FIXED_NTIMES
#else
#define RTX_NDOF(P) (P).n_dof
#define RTX_NAA(P) (P).n_aa
#define RTX_NTIMES(P) (P).n_times
#endif

// scene.py:54-55: base_ray_direction and focal_point of pixel (column cc, reference row j).
RTX_HD f3 pixel_focal(const KParams& P, int32_t cc, int j) {
    const float fx = P.xs[cc];
    const float fy = P.ys[j];
    // base_ray_direction = normalize(x * u + y * v - d * w)  (scene.py:54)
    const f3 bdir = normalize(sub(add(scale(ld3(P.u), fx), scale(ld3(P.v), fy)), ld3(P.dw)));
    return add(ld3(P.pos), scale(bdir, P.focal));  // scene.py:55
}

#ifdef RTX_FIXED_JMODE  // scene-specialized kernels pin the jitter mode
#define RTX_JMODE(P) RTX_FIXED_JMODE
#else
#define RTX_JMODE(P) (P).jitter
#endif

// Production jitter (RTX_JITTER_PHILOX): sample s = kd * n_aa + ka of pixel (column
// col0 + cc, reference row j) takes half s & 1 of one Philox4x32-10 block with counter
// (col0 + cc, j, s >> 1, 0) and the scene's seed: 128 bits -> 6 uniforms of 21 bits,
// three per sample (half 0: the top 21 bits of words 0-2; half 1: their low 11 bits
// joined with 10-bit pieces of word 3). Consecutive samples share a block, so a pixel's
// samples cost half a Philox evaluation each (the render loops keep the block).
RTX_HD void jitter_block(const KParams& P, int32_t cc, int j, int pair, uint32_t w[4]) {
    w[0] = (uint32_t)(P.col0 + cc);
    w[1] = (uint32_t)j;
    w[2] = (uint32_t)pair;
    w[3] = 0u;
    philox4x32(w, P.seed_lo, P.seed_hi);
}
RTX_HD f3 jitter_rnd(const uint32_t w[4], int half) {
    const uint32_t a = half ? ((w[0] & 0x7FFu) | ((w[3] & 0x3FFu) << 11)) : w[0] >> 11;
    const uint32_t b = half ? ((w[1] & 0x7FFu) | (((w[3] >> 10) & 0x3FFu) << 11)) : w[1] >> 11;
    const uint32_t c = half ? ((w[2] & 0x7FFu) | (((w[3] >> 20) & 0x3FFu) << 11)) : w[2] >> 11;
    return mk((float)a * 0x1p-21f, (float)b * 0x1p-21f, (float)c * 0x1p-21f);
}

// scene.py:60-65: the origin of AA sample ka of DOF sample kd, jittered (JIT). jr: this
// sample's Philox uniforms when the caller has them (render_pixel keeps the odd sample's
// from the pair's block), else they are computed here.
template <bool JIT>
RTX_HD f3 sample_origin(const KParams& P, int32_t cc, int j, int kd, int ka, const f3* jr = nullptr) {
    f3 o = ld3(P.aa_o + 3 * (kd * RTX_NAA(P) + ka));
    if (JIT) {  // scene.py:63-65
        f3 rnd;
        if (RTX_JMODE(P) == RTX_JITTER_REPLAY) {
            const int64_t idx = (((int64_t)cc * P.height + j) * RTX_NDOF(P) + kd) * RTX_NAA(P) + ka;
            rnd = ld3(P.noise + 3 * idx);
        } else if (RTX_PROBE(15)) {  // cost probe only: no RNG
            rnd = mk(0.25f + 0.001f * (float)ka, 0.5f, 0.75f + 0.001f * (float)kd);
        } else if (jr != nullptr) {
            rnd = *jr;
        } else {
            const int s = kd * RTX_NAA(P) + ka;
            uint32_t w[4];
            jitter_block(P, cc, j, s >> 1, w);
            rnd = jitter_rnd(w, s & 1);
        }
        o = add(o, scale(normalize(rnd), P.jscale));
    }
    return o;
}

// colour / (samples * dof_samples * len(motion_times)) (scene.py:73); for a power of two
// the exact reciprocal multiply gives the identical correctly rounded result.
RTX_HD float sample_mean(const KParams& P, float c) {
#ifdef RTX_FIXED_DIVPOW2
    return RTX_FIXED_DIVPOW2 ? c * P.inv_divisor : c / P.divisor;
#else
    return P.div_pow2 ? c * P.inv_divisor : c / P.divisor;
#endif
}

// The framebuffer store. fp32 RGB (rtx_render), or -- scene-specialized kernels built
// with RTX_OUT8=1 for rtx_render_rgb8 -- main.py:33's (v * 255).astype(uint8) of the same
// fp32 value, written as bytes (the PNG's layout: 4x fewer bytes to store and to gather).
#ifndef RTX_OUT8
#define RTX_OUT8 0
#endif
RTX_HD void put_channel(float* fb, int64_t i, float v) {
    if (RTX_OUT8)
        reinterpret_cast<uint8_t*>(fb)[i] = (uint8_t)(int)((double)v * 255.0);
    else
        fb[i] = v;
}

// Multi-sample kernels re-read the scene records in every sample instead of keeping
// them live across the sample loops: the compiler otherwise hoists every record load and
// its loop-invariant VALU conversions (fp64 box bounds, padded culling boxes) out of the
// loops, where they occupy SGPRs and VGPRs for the kernel's whole life and spill (the
// DepthOfField kernel: 54 SGPRs into VGPR lanes and 176 B/lane of scratch, written once
// per pixel = 1.46 GB per 4K frame). Re-reads are scalar-cache hits, once per sample.
#ifndef RTX_RELOAD_RECORDS
#if defined(RTX_FIXED_SAMPLES)
#define RTX_RELOAD_RECORDS (RTX_FIXED_NDOF * RTX_FIXED_NAA * RTX_FIXED_NTIMES > 1)
#else
#define RTX_RELOAD_RECORDS 1
#endif
#endif
// A wave-uniform pointer the compiler cannot prove loop-invariant (its halves pass through
// readfirstlane, a no-op on a uniform value, and an empty asm that "redefines" them).
template <class T>
__device__ __forceinline__ cptr<T> opaque_uniform(cptr<T> p) {
    const uint64_t v = (uint64_t)p;
    uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    asm volatile("" : "+s"(lo), "+s"(hi));
    return (cptr<T>)(((uint64_t)hi << 32) | lo);
}
// (flat-scene kernels only: the hierarchy/texture kernels keep the loaded records)
//
// One-sample scene-specialized kernels built with RTX_BAKED_RECORDS carry the scene's object,
// material and light records in the code object (rtx_api.hip jit_baked_records: constant
// arrays rtx_baked::kObjs / kMats / kLights, defined ahead of this header). Reads at a
// compile-time index -- the unrolled object and light loops -- fold to literals, so no
// dependent scalar load precedes a wave's first ray; per-lane reads (the hit object, its
// material) load from the code object's read-only data. The values are the same bytes
// rtx_scene_create uploads, so the arithmetic is unchanged.
template <bool X>
RTX_HD SceneView sample_scene(const SceneView& S0) {
    SceneView S = S0;
#if defined(RTX_BAKED_RECORDS) && defined(__HIP_DEVICE_COMPILE__)
    if (!X) {
        S.objs = (cptr<DObj>)rtx_baked::kObjs;
        S.mats = (cptr<DMat>)rtx_baked::kMats;
        S.lights = (cptr<DLight>)rtx_baked::kLights;
        return S;
    }
#endif
#if defined(__HIP_DEVICE_COMPILE__)
    if (RTX_RELOAD_RECORDS && !X) {  // opaque to loop-invariant code motion
        S.objs = opaque_uniform(S.objs);
        if (RTX_RELOAD_RECORDS > 1) {
            S.mats = opaque_uniform(S.mats);
            S.lights = opaque_uniform(S.lights);
        }
    }
#endif
    return S;
}

// scene.py:47-79 for pixel p of the output block (host/device: the tests-only host
// emulation runs the same body).
template <bool MESH, bool SEC, bool X, bool COUNT, bool JIT>
RTX_HD void render_pixel(const KParams& P, float* fb, int32_t row0, int32_t rr, int32_t cc, Tally& tl,
                         const FrameStack& fs, const HStack& hs, int32_t bin = -1) {
    if (RTX_PROBE(14)) {  // cost probe only: store a constant (launch + framebuffer write)
        const int64_t p = (int64_t)rr * P.ncols + cc;
        put_channel(fb, 3 * p, 0.5f); put_channel(fb, 3 * p + 1, 0.25f); put_channel(fb, 3 * p + 2, 0.125f);
        return;
    }
    const int j = P.height - 1 - (row0 + rr);  // reference row index (y grows upward)
    const int32_t blane = bin >= 0 ? (((row0 + rr) & 7) << 3) | (cc & 7) : -1;  // the pixel in its tile
#if defined(RTX_PRIM_ORIGIN) && RTX_PRIM_ORIGIN && defined(RTX_FIXED_COUNTS)
    OriginTerms prim;  // the primary rays' origin-only terms (host-computed)
#pragma unroll
    for (int k = 0; k < RTX_FIXED_NP; ++k) prim.pnum[k] = P.po_pnum[k];
#pragma unroll
    for (int k = 0; k < RTX_FIXED_NS; ++k) {
        prim.soc[k] = ld3(P.po_soc[k]);
        prim.sq[k] = P.po_sq[k];
    }
    const OriginTerms* primp = &prim;
#else
    const OriginTerms* primp = nullptr;
#endif
    f3 colour = mk(0.0f, 0.0f, 0.0f);
    f3 jr_odd = mk(0.0f, 0.0f, 0.0f);  // the odd sample's jitter uniforms of the current pair
    // pinned counts must not unroll the loops (one cast_ray body per sample)
#pragma unroll 1
    for (int kd = 0; kd < RTX_NDOF(P); ++kd) {
        // the focal point is recomputed per DOF sample (the same fp32 operations) rather
        // than kept live across the loops (RTX_RELOAD_RECORDS)
        int32_t cc_k = cc, j_k = j;
#if defined(__HIP_DEVICE_COMPILE__)
        if (RTX_RELOAD_RECORDS) asm volatile("" : "+v"(cc_k), "+v"(j_k));
#endif
        const f3 focal = pixel_focal(P, cc_k, j_k);
        const f3 ddir = normalize(sub(focal, ld3(P.dof_o + 3 * kd)));  // scene.py:58
#pragma unroll 1
        for (int ka = 0; ka < RTX_NAA(P); ++ka) {
            // the Philox block of samples (2m, 2m + 1), computed at the even one; the odd
            // one's uniforms wait in jr
            const bool philox = JIT && RTX_JMODE(P) == RTX_JITTER_PHILOX && !RTX_PROBE(15);
            const bool odd = ((kd * RTX_NAA(P) + ka) & 1) != 0;
            f3 jr = jr_odd;
            if (philox && !odd) {
                uint32_t w[4];
                jitter_block(P, cc, j, (kd * RTX_NAA(P) + ka) >> 1, w);
                jr = jitter_rnd(w, 0);
                jr_odd = jitter_rnd(w, 1);
            }
            const f3 o = sample_origin<JIT>(P, cc, j, kd, ka, philox ? &jr : nullptr);
#pragma unroll 1
            for (int kt = 0; kt < RTX_NTIMES(P); ++kt)
                colour = add(colour, cast_ray<MESH, SEC, X, COUNT>(sample_scene<X>(P.S), o, ddir, P.times[kt], tl, fs, hs,
                                                                   bin, primp, blane));
        }
    }
    colour = mk(sample_mean(P, colour.x), sample_mean(P, colour.y), sample_mean(P, colour.z));
#if RTX_PROBE_ON == 11 && defined(__HIP_DEVICE_COMPILE__)
    {  // cost probe only: RTX_PAD extra VALU instructions per pixel in 4 independent chains
        float c0 = colour.x, c1 = colour.y, c2 = colour.z, c3 = (float)cc;
#pragma unroll
        for (int k = 0; k < RTX_PAD / 4; ++k)
            asm volatile("v_add_f32 %0, %4, %0\n v_add_f32 %1, %4, %1\n v_add_f32 %2, %4, %2\n v_add_f32 %3, %4, %3"
                         : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3) : "v"((float)j));
        colour = mk(c0, c1, c2 + c3 * 0.0f);
    }
#endif
    const int64_t p = (int64_t)rr * P.ncols + cc;
    put_channel(fb, 3 * p, colour.x);
    put_channel(fb, 3 * p + 1, colour.y);
    put_channel(fb, 3 * p + 2, colour.z);
}

// Chunk c of a heavy tile's primary-ray face list (SceneView::bin_heavy): for the tile's
// pixel `lane` (row * 8 + column of its 8x8 tile), the closest of the chunk's faces by
// closest_hit's tests -- the face's padded box, then the exact test, offered to the same
// total order -- as (t32 bits, stored face or -1). The primary ray is render_pixel's of a
// one-sample pinhole camera (the bins' cameras): aa_o[0] toward the pixel's focal point.
// Every lane of a wave calls it for the same chunk (the loop's votes are the wave's).
// (Measured slower: starting chunks c >= 1 from chunk 0's closest face, in a second launch
// after it, blob 1080p 0.275 -> 0.291 ms; two faces per step, 0.201 -> 0.208-0.212 ms.)
RTX_HD uint2 mesh_chunk(const KParams& P, int32_t bin, int32_t c, int lane) {
    const SceneView& S = P.S;
    const int32_t ty = bin / S.bins_x, tx = bin - ty * S.bins_x;
    const int32_t row = ty * 8 + (lane >> 3), cc = tx * 8 + (lane & 7);
    const bool active = row < P.height && cc < P.ncols;
    const int j = P.height - 1 - (active ? row : 0);
    const f3 d = normalize(sub(pixel_focal(P, active ? cc : 0, j), ld3(P.dof_o)));  // scene.py:58
    const f3 o = ld3(P.aa_o);  // scene.py:60-61 (one sample, no jitter)
    const int32_t oi = S.n_plane + S.n_sphere + S.n_box;  // the scene's one top-level mesh
    const DObj ob = S.objs[oi];
    const float time = P.times[0];
    const RayInv ri = ray_inv(o, d);
    Hit h{INFINITY, -1, 0};
    const int32_t q0 = S.bin_start[bin] + c * kHeavyChunk;
    const int32_t q1 = min(S.bin_start[bin + 1], q0 + kHeavyChunk);
    for (int32_t q = q0; q < q1; ++q) {
        if (RTX_ALL(!active || h.t32 < S.bin_zmin[q])) break;  // nearest first (closest_hit's exit)
        const int32_t f = S.bin_faces[q];
        const bool fmaybe = active && leaf_maybe_hit(RTX_FBOX(S, ob.tri_begin + f), o, ri, ob.cmax, h.t32);
        if (!RTX_ANY(fmaybe)) continue;
        float t32;
        const bool valid = tri_hit(RTX_TRI(S, ob.tri_begin + f), o, d, fmaybe, t32);
        offer(S, h, valid, t32, oi, f, o, d, time);
    }
    return make_uint2(__builtin_bit_cast(uint32_t, h.t32), h.obj >= 0 ? (uint32_t)h.sub : 0xFFFFFFFFu);
}

// mesh_chunk with the chunk's face records staged in LDS first (k_mesh_chunks mode bit 0,
// device only): one round of coalesced loads -- every lane fetches 16-byte words of the
// chunk's face records (its 32 face indices, then 96 B of triangle and 32 B of face box
// per face) -- instead of 2-3 dependent scalar loads per face inside the loop (the pass
// waited on memory 0.63 of its wave cycles, profiles/pmc_blob1080.json). The same tests,
// in the same order, as mesh_chunk.
#if defined(__HIP_DEVICE_COMPILE__)
struct ChunkLds {
    DTri tri[kHeavyChunk];
    DFaceBox box[kHeavyChunk];
    int32_t face[kHeavyChunk];
    float zmin[kHeavyChunk];
};
__device__ __forceinline__ uint2 mesh_chunk_lds(const KParams& P, int32_t bin, int32_t c, int lane, ChunkLds& sh) {
    const SceneView& S = P.S;
    const int32_t ty = bin / S.bins_x, tx = bin - ty * S.bins_x;
    const int32_t row = ty * 8 + (lane >> 3), cc = tx * 8 + (lane & 7);
    const bool active = row < P.height && cc < P.ncols;
    const int32_t oi = S.n_plane + S.n_sphere + S.n_box;  // the scene's one top-level mesh
    const DObj ob = S.objs[oi];
    const int32_t q0 = S.bin_start[bin] + c * kHeavyChunk;
    const int32_t n = min(S.bin_start[bin + 1], q0 + kHeavyChunk) - q0;
    if (lane < n) {
        sh.face[lane] = S.bin_faces[q0 + lane];
        sh.zmin[lane] = S.bin_zmin[q0 + lane];
    }
    __syncthreads();  // (one wave per block)
    constexpr int kTriW = (int)(sizeof(DTri) / 16), kBoxW = (int)(sizeof(DFaceBox) / 16), kW = kTriW + kBoxW;
    for (int w = lane; w < n * kW; w += 64) {
        const int i = w / kW, k = w - i * kW;
        const int64_t f = ob.tri_begin + sh.face[i];
        if (k < kTriW)
            reinterpret_cast<uint4*>(&sh.tri[i])[k] = reinterpret_cast<const uint4 RTX_CONST*>(&S.tris[f])[k];
        else
            reinterpret_cast<uint4*>(&sh.box[i])[k - kTriW] = reinterpret_cast<const uint4 RTX_CONST*>(&S.fboxes[f])[k - kTriW];
    }
    __syncthreads();
    const int j = P.height - 1 - (active ? row : 0);
    const f3 d = normalize(sub(pixel_focal(P, active ? cc : 0, j), ld3(P.dof_o)));  // scene.py:58
    const f3 o = ld3(P.aa_o);  // scene.py:60-61 (one sample, no jitter)
    const float time = P.times[0];
    const RayInv ri = ray_inv(o, d);
    Hit h{INFINITY, -1, 0};
    for (int i = 0; i < n; ++i) {
        if (RTX_ALL(!active || h.t32 < sh.zmin[i])) break;  // nearest first (closest_hit's exit)
        const DFaceBox B = sh.box[i];
        const bool fmaybe = active && leaf_maybe_hit(B, o, ri, ob.cmax, h.t32);
        if (!RTX_ANY(fmaybe)) continue;
        float t32;
        const bool valid = tri_hit(sh.tri[i], o, d, fmaybe, t32);
        offer(S, h, valid, t32, oi, sh.face[i], o, d, time);
    }
    return make_uint2(__builtin_bit_cast(uint32_t, h.t32), h.obj >= 0 ? (uint32_t)h.sub : 0xFFFFFFFFu);
}
#endif

// Blocks of a split chunk to render again in the one-kernel form (rtx_split.h): n == nullptr
// for every other launch. A listed block's flag is set; the launch that renders it clears it.
struct RedoList {
    const uint32_t* n;       // blocks listed
    const uint32_t* blocks;  // their indices
    uint32_t* flags;         // per block of the chunk
};

// The per-frame parameters live in device memory (uploaded by rtx_camera_set) and are
// read with scalar loads; only the per-call output block is passed by value.
struct Launch {
    float* fb;
    unsigned long long* counters;
    int32_t row0, nrows;
    // gstride > 0 (rtx_render_groups): the block's rows are the 8-row groups gphase,
    // gphase + gstride, ... of the image, packed in order
    int32_t gphase, gstride;
    // rtx_render_frames: blockIdx.y renders frame y of a batch into fb + y * fstride bytes
    int64_t fstride;
    uint32_t perm;  // RTX_TILE_ORDER 2: the wave permutation's multiplier
    int32_t pix0;   // split hierarchy passes (rtx_split.h): the chunk's first pixel of the block
    int32_t tperm;  // RTX_TILE_SCHED kernels: 1 = dispatch a whole frame's tiles by P.tile_perm
    int32_t tlog;   // RTX_TILE_SCHED kernels: 1 = record each wave's duration in P.tile_time
    int32_t xcd;    // 1 = XCD-aware block order (xcd_block; tile-mapped render_body)
    // render_body_spp as the split passes' fallback (rtx_split.h): render only the listed
    // blocks (chains that found the record pool full), pixels from pix0 on
    RedoList redo;
};

// This block's framebuffer (frame blockIdx.y of a batched launch; the only frame otherwise).
__device__ __forceinline__ float* frame_fb(const Launch& L) {
    return reinterpret_cast<float*>(reinterpret_cast<char*>(L.fb) + (int64_t)blockIdx.y * L.fstride);
}

// Image row (row 0 = top) of block row rr.
__host__ __device__ inline int32_t image_row(const Launch& L, int32_t rr) {
    return L.gstride > 0 ? ((rr >> 3) * L.gstride + L.gphase) * 8 + (rr & 7) : L.row0 + rr;
}

// The primary-ray face bin of the 8x8 pixel tile whose top-left pixel is (image row,
// strip column, a multiple of 8), or -1 when the camera has no bins or the tile straddles
// two bin rows (row blocks that start off the 8-row grid).
// Scene-specialized kernels of cameras without bins are compiled with RTX_PRIMARY_BINS=0
// (the bin code vanishes); the precompiled kernels check bins_on at run time.
#ifndef RTX_PRIMARY_BINS
#define RTX_PRIMARY_BINS 1
#endif
__host__ __device__ inline int32_t primary_bin(const SceneView& S, int32_t row, int32_t col) {
    return RTX_PRIMARY_BINS && S.bins_on && (row & 7) == 0 ? (row >> 3) * S.bins_x + (col >> 3) : -1;
}

// Occupancy request (waves per SIMD) by kernel variant: mesh kernels without secondary
// rays fit 128 VGPRs without scratch and gain from 4 waves/SIMD; the flat primary+shadow
// kernels from 5 (DepthOfField 4K 11.2 -> 10.2 ms; TwoSpheresPlane already fits); the
// secondary-ray kernels lose if forced below their natural allocation (measured,
// tools/ablate.sh: 6 and 8 waves are slower everywhere).
#ifndef RTX_LB_WAVES
#define RTX_LB_WAVES(MESH, SEC) ((SEC) ? 1 : ((MESH) ? 4 : 5))
#endif
#ifndef RTX_TILE
#define RTX_TILE 1
#endif
// Pixels per lane: each wave renders RTX_PPL 8x8 tiles in sequence (amortises the
// per-wave setup chain: parameters, tables, scene records).
#ifndef RTX_PPL
#define RTX_PPL 1
#endif

// Output pixel (row, column within the block) of this work-item. RTX_TILE=1 maps each
// 64-lane wave to an 8x8 pixel tile (coherent rays per wave); 0 maps waves to 64
// consecutive pixels of a row. The wave's tile is wave-uniform, so its coordinates are
// scalar 32-bit arithmetic.
struct PixelRC {
    int32_t r, c;
};
// The order in which a launch's waves visit the tiles (experiments): 0 row-major from the
// top, 1 reversed (bottom rows first), 2 a stride permutation w -> w * perm mod T (the
// host picks perm coprime to the launch's T waves, near T / golden ratio), so each
// stretch of the dispatch samples the whole image.
#ifndef RTX_TILE_ORDER
#define RTX_TILE_ORDER 0
#endif
// Measured tile schedule (scene-specialized kernels of scenes with secondary rays or
// meshes, rtx_api.hip tile_schedule): whole-frame launches can dispatch the tiles in a
// table's order (longest measured first) and record each wave's duration.
#ifndef RTX_TILE_SCHED
#define RTX_TILE_SCHED 0
#endif
// XCD-aware block order (Launch::xcd, option xcd_map): the dispatcher hands workgroups to the 8 XCDs
// round-robin, so consecutive blocks -- neighbouring tiles, whose bin lists, tile-schedule
// entries and scene lines share cache lines -- would land in 8 different L2s. Block b
// instead takes slot block xcd_block(b): each XCD's k-th run of 16 waves (g blocks of
// 16/g waves) takes 16 consecutive tiles. Blocks of the last incomplete round of 8 runs keep
// their own index, so the map is a bijection on [0, nb). Host and device share it (the
// tile schedule's table is laid out through it, rtx_api.hip tile_schedule). Off by default:
// it cuts the fabric reads of the bins, light grids and schedule table (TorusMesh 1080p
// 29.8 -> 28.9 MB per frame, TwoSpheresPlane 26.2 -> 25.5, DepthOfField 4K 111.7 -> 109.5)
// but not the time (TwoSpheresPlane 22.06 -> 22.42 us, the 81,920-face mesh +1 %,
// DepthOfField -0.6 %; profiles/r05/xcd/).
__host__ __device__ inline uint32_t xcd_block(uint32_t b, uint32_t nb, uint32_t waves_per_block) {
    const uint32_t lg = waves_per_block >= 16 ? 0u : (waves_per_block >= 4 ? 2u : (waves_per_block >= 2 ? 3u : 4u));
    const uint32_t g = 1u << lg, round = 8u * g;
    if (b >= nb / round * round) return b;
    const uint32_t x = b & 7u, k = b >> 3;
    return (((k >> lg) << 3) + x) * g + (k & (g - 1u));
}
__device__ __forceinline__ PixelRC pixel_rc(int32_t ncols, int sub, uint32_t perm = 1, int32_t xcd = 0,
                                            const int32_t RTX_CONST* tperm = nullptr, int* tile = nullptr) {
    const int lane = threadIdx.x & 63;
    const uint32_t blk = xcd ? xcd_block(blockIdx.x, gridDim.x, blockDim.x >> 6) : blockIdx.x;
    int wave = __builtin_amdgcn_readfirstlane((int)((blk * (blockDim.x >> 6) + (threadIdx.x >> 6)) * RTX_PPL + sub));
    const uint32_t T = gridDim.x * (blockDim.x >> 6) * RTX_PPL;
    if (RTX_TILE_SCHED && tperm != nullptr) wave = tperm[wave];
    if (tile) *tile = wave;
    if (RTX_TILE_ORDER == 1) wave = (int)T - 1 - wave;
    if (RTX_TILE_ORDER == 2) wave = (int)(((uint64_t)(uint32_t)wave * perm) % T);
    if (RTX_TILE == 0) {
        const int64_t p = (int64_t)wave * 64 + lane;
        const int32_t r = (int32_t)(p / ncols);
        return PixelRC{r, (int32_t)(p - (int64_t)r * ncols)};
    }
    const int tiles_x = (ncols + 7) >> 3;
    const int ty = wave / tiles_x, tx = wave - ty * tiles_x;
    return PixelRC{ty * 8 + (lane >> 3), tx * 8 + (lane & 7)};
}

__host__ __device__ inline int64_t launch_items(int32_t nrows, int32_t ncols) {
    const int64_t waves = RTX_TILE == 0 ? ((int64_t)nrows * ncols + 63) / 64
                                        : (int64_t)((ncols + 7) >> 3) * ((nrows + 7) >> 3);
    return (waves + RTX_PPL - 1) / RTX_PPL * 64;
}

// Block size: 256 threads, or one wave for the hierarchy/texture (X) variants, whose
// per-thread ray/point stacks (9 words per hierarchy level) share the CU's LDS.
// 64 and 128 measured equal to 256 within noise with matching JIT kernels (library and
// hiprtc kernels both built with the value; tools/ab_block.sh, profiles/r02/blk: TSP
// 28.7/29.1/29.0 us, TM 83.0/82.1/81.9, MR 51.6/52.8/52.2, DOF 7.23/7.21/7.28 ms for
// 256/64/128)
#ifndef RTX_BLOCK_FLAT  // threads per block of the flat-scene kernels (experiments)
#define RTX_BLOCK_FLAT 256
#endif
template <bool X>
constexpr int kBlock = X ? 64 : RTX_BLOCK_FLAT;

// The body of k_render, shared with the scene-specialized kernels compiled at run time
// (rtx_jit.cpp), which pin the scene's object and light counts.
// RTX_LDS_TRIS kernels: the block copies the scene's triangles, face boxes and BVH nodes
// into LDS (16-byte words, all lanes) before tracing (rtx_trace.h RTX_TRI / RTX_LEAF).
__device__ __forceinline__ void stage_mesh_lds(const SceneView& S) {
#if defined(RTX_LDS_TRIS) && defined(__HIP_DEVICE_COMPILE__)
    auto copy = [](void* dst, const void RTX_CONST* src, int words) {
        uint4* d = static_cast<uint4*>(dst);
        const uint4 RTX_CONST* s = static_cast<const uint4 RTX_CONST*>(src);
        for (int i = threadIdx.x; i < words; i += blockDim.x) d[i] = s[i];
    };
    copy(g_lds_tris, S.tris, RTX_LDS_TRIS * (int)(sizeof(DTri) / 16));
    copy(g_lds_fboxes, S.fboxes, RTX_LDS_TRIS * (int)(sizeof(DFaceBox) / 16));
    copy(g_lds_leaves, S.leaves, RTX_LDS_LEAVES * (int)(sizeof(DLeaf) / 16));
    __syncthreads();
#else
    (void)S;
#endif
}

// RTX_LDS_OBJS kernels: the block copies the object and material records into LDS.
__device__ __forceinline__ void stage_records_lds(const SceneView& S) {
#if defined(RTX_LDS_OBJS) && defined(__HIP_DEVICE_COMPILE__)
    auto copy = [](void* dst, const void RTX_CONST* src, int words) {
        uint4* d = static_cast<uint4*>(dst);
        const uint4 RTX_CONST* s = static_cast<const uint4 RTX_CONST*>(src);
        for (int i = threadIdx.x; i < words; i += blockDim.x) d[i] = s[i];
    };
    copy(g_lds_objs, S.objs, RTX_LDS_OBJS * (int)(sizeof(DObj) / 16));
    copy(g_lds_mats, S.mats, RTX_LDS_MATS * (int)(sizeof(DMat) / 16));
    __syncthreads();
#else
    (void)S;
#endif
}

// Wave timeline probe (experiment): the wave's start/end clock and where it ran.
#if defined(RTX_WAVE_LOG) && defined(__HIP_DEVICE_COMPILE__)
struct WaveClock {
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    __device__ void done(const KParams* Pp) const {
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        if ((threadIdx.x & 63) == 0 && Pp->wave_log != nullptr) {
            const uint64_t w = ((uint64_t)blockIdx.y * gridDim.x + blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6);
            const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
            const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
            unsigned long long* o = Pp->wave_log + 4 * w;
            o[0] = t0;
            o[1] = t1;
            o[2] = hw;
            o[3] = xcc;
        }
    }
};
#define RTX_WAVE_CLOCK_BEGIN const WaveClock wclk_;
#define RTX_WAVE_CLOCK_END wclk_.done(Pp);
#else
#define RTX_WAVE_CLOCK_BEGIN
#define RTX_WAVE_CLOCK_END
#endif

template <bool MESH, bool SEC, bool X, bool COUNT, bool JIT>
__device__ __forceinline__ void render_body(const KParams* __restrict__ Pp, const Launch L) {
    constexpr int B = kBlock<X>;
    RTX_WAVE_CLOCK_BEGIN
    if (MESH) stage_mesh_lds(Pp->S);
    stage_records_lds(Pp->S);
#ifdef RTX_FIXED_NCOLS  // scene-specialized kernels pin the strip width (tile index math by constants)
    const int32_t ncols = RTX_FIXED_NCOLS;
#else
    const int32_t ncols = Pp->ncols;
#endif
    Tally tl = {};
    // secondary-ray frames: [frame][word][thread] in LDS (40 KB per 256-thread block; 30 KB
    // with RTX_FRAME_MATBITS)
    __shared__ float frames[SEC ? kFrameLds * kFrameWords * B : 1];
    extern __shared__ float hstack[];  // X: [level][9][thread] (dynamic size)
    const FrameStack fs{frames + threadIdx.x, B};
    const HStack hs{hstack + threadIdx.x, B};
    bool any_active = false;
#if RTX_TILE_SCHED && defined(__HIP_DEVICE_COMPILE__)
    static_assert(RTX_TILE == 1 && RTX_PPL == 1, "the tile schedule orders whole 8x8 tiles");
    const unsigned long long tclk0 = L.tlog ? __builtin_amdgcn_s_memrealtime() : 0ull;
    int tile = 0;
#endif
    for (int sub = 0; sub < RTX_PPL; ++sub) {
#if RTX_TILE_SCHED && defined(__HIP_DEVICE_COMPILE__)
        const PixelRC px = pixel_rc(ncols, sub, L.perm, L.xcd, L.tperm ? Pp->tile_perm : nullptr, &tile);
#else
        const PixelRC px = pixel_rc(ncols, sub, L.perm, L.xcd);
#endif
        const bool active = px.r < L.nrows && px.c < ncols;
        any_active = any_active || active;
        // primary-ray face bin of the wave's 8x8 tile (its top-left pixel)
        const int32_t bin = RTX_TILE == 1 ? primary_bin(Pp->S, image_row(L, px.r & ~7), px.c & ~7) : -1;
        // render_pixel's image row is row0 + rr: pass the image row of px.r as that sum
        if (active)
            render_pixel<MESH, SEC, X, COUNT, JIT>(*Pp, frame_fb(L), image_row(L, px.r) - px.r, px.r, px.c, tl, fs, hs, bin);
    }
    flush_tally<COUNT>(tl, L.counters, any_active);
#if RTX_TILE_SCHED && defined(__HIP_DEVICE_COMPILE__)
    if (L.tlog && (threadIdx.x & 63) == 0 && tile < Pp->tile_n)
        Pp->tile_time[tile] = (unsigned int)(__builtin_amdgcn_s_memrealtime() - tclk0);
#endif
    RTX_WAVE_CLOCK_END
}

// n / d and n % d for 0 <= n < 2^22, d >= 1 (rd = fl32(1 / d)): the fp32 quotient is
// off by at most one, which the remainder test corrects. Full-rate 24-bit multiplies.
__device__ __forceinline__ int udiv_small(int n, int d, float rd, int& rem) {
    int q = (int)((float)n * rd);
    int r = n - (int)__umul24((unsigned)q, (unsigned)d);
    if (r >= d) { ++q; r -= d; }
    if (r < 0) { --q; r += d; }
    rem = r;
    return q;
}

// Pixels per block of the sample-parallel mapping (host and device agree on it).
__host__ __device__ inline int spp_pixels_per_block(int spp, int block) { return spp >= block ? 1 : block / spp; }

// Sample-parallel mapping for high sample counts (rtx_render picks it for the hierarchy /
// texture kernels when a pixel has >= RTX_SPP_MIN samples): the B lanes of a block trace the samples of P = B / spp
// consecutive pixels (row-major within the output block), or the samples of one pixel
// in ceil(spp / B) rounds, so a wave's rays start from one pixel (coherent) and a wave
// lasts one sample instead of all of them. Each lane puts its sample's colour in LDS;
// per (pixel, channel) one owner lane then adds them in the reference's order
// (dof, aa, time; scene.py:57-70) starting from +0 -- the same fp32 sums as
// render_pixel -- and writes the mean. Samples s map to (kd, ka, kt) with kt fastest.
template <bool MESH, bool SEC, bool X, bool COUNT, bool JIT>
__device__ __forceinline__ void render_block_spp(const KParams* __restrict__ Pp, const Launch& L, int64_t blk, Tally& tl,
                                                 bool& any_active) {
    constexpr int B = kBlock<X>;
    const KParams& P = *Pp;
    const int32_t ncols = P.ncols;
    const int nt = RTX_NTIMES(P), na = RTX_NAA(P);
    const int S = RTX_NDOF(P) * na * nt;
    const int PPB = spp_pixels_per_block(S, B);
    const int rounds = (PPB * S + B - 1) / B;
    const float rS = 1.0f / (float)S, rT = 1.0f / (float)nt, rA = 1.0f / (float)na;
    __shared__ float frames[SEC ? kFrameLds * kFrameWords * B : 1];
    __shared__ float sbuf[3 * B];
    extern __shared__ float hstack[];  // X: [level][9][thread] (dynamic size)
    const FrameStack fs{frames + threadIdx.x, B};
    const HStack hs{hstack + threadIdx.x, B};
    const int64_t npix = (int64_t)L.nrows * ncols;
    const int64_t pix0 = L.pix0 + blk * PPB;
    const int tid = threadIdx.x;
    float acc = 0.0f;  // rounds > 1 (one pixel per block): lane ch < 3 sums channel ch
    for (int rd = 0; rd < rounds; ++rd) {
        const int flat = rd * B + tid;  // the block's sample index
        int s;
        const int lp = udiv_small(flat, S, rS, s);
        const int64_t p = pix0 + lp;
        const bool active = lp < PPB && p < npix;
        f3 c = mk(0.0f, 0.0f, 0.0f);
        if (active) {
            any_active = true;
            const int32_t rr = (int32_t)(p / ncols), cc = (int32_t)(p - (int64_t)rr * ncols);
            const int j = P.height - 1 - image_row(L, rr);
            int kt, ka;
            const int da = udiv_small(s, nt, rT, kt);
            const int kd = udiv_small(da, na, rA, ka);
            const f3 focal = pixel_focal(P, cc, j);
            const f3 ddir = normalize(sub(focal, ld3(P.dof_o + 3 * kd)));  // scene.py:58
            const f3 o = sample_origin<JIT>(P, cc, j, kd, ka);
            c = cast_ray<MESH, SEC, X, COUNT>(P.S, o, ddir, P.times[kt], tl, fs, hs);
        }
        sbuf[tid] = c.x;
        sbuf[B + tid] = c.y;
        sbuf[2 * B + tid] = c.z;
        __syncthreads();
        if (rounds == 1) {  // (pixel, channel) pairs, each summed in order by one lane
            for (int q = tid; q < 3 * PPB; q += B) {
                const int pp = q / 3, ch = q - 3 * (q / 3);
                if (pix0 + pp < npix) {
                    const float* src = sbuf + ch * B + pp * S;
                    float a = 0.0f;
                    for (int k = 0; k < S; ++k) a += src[k];
                    put_channel(frame_fb(L), 3 * (pix0 + pp) + ch, sample_mean(P, a));
                }
            }
        } else if (tid < 3) {  // this round's samples of the block's pixel
            const int hi = min(S - rd * B, B);
            const float* src = sbuf + tid * B;
            for (int k = 0; k < hi; ++k) acc += src[k];
        }
        __syncthreads();  // sbuf is reused by the next round (or block)
    }
    if (rounds > 1 && tid < 3 && pix0 < npix) put_channel(frame_fb(L), 3 * pix0 + tid, sample_mean(P, acc));
}

template <bool MESH, bool SEC, bool X, bool COUNT, bool JIT>
__device__ __forceinline__ void render_body_spp(const KParams* __restrict__ Pp, const Launch L) {
    Tally tl = {};
    bool any_active = false;
    // one block, or (the split passes' redo list) the grid strides over the listed blocks;
    // one call site either way
    const bool listed = L.redo.n != nullptr;
    const uint32_t nb = listed ? *L.redo.n : 1u;
    for (uint32_t i = listed ? blockIdx.x : 0u; i < nb; i += listed ? gridDim.x : 1u) {
        const uint32_t b = listed ? L.redo.blocks[i] : blockIdx.x;
        render_block_spp<MESH, SEC, X, COUNT, JIT>(Pp, L, (int64_t)b, tl, any_active);
        if (listed && threadIdx.x == 0) L.redo.flags[b] = 0u;
    }
    flush_tally<COUNT>(tl, L.counters, any_active);
}

#ifndef RTX_LB_XWAVES  // hierarchy/texture kernels: waves per SIMD requested (experiments)
#define RTX_LB_XWAVES 1
#endif
#define RTX_RENDER_BOUNDS(MESH, SEC, X) __launch_bounds__(rtx::kBlock<X>, (X) ? RTX_LB_XWAVES : RTX_LB_WAVES(MESH, SEC))

#if !defined(__HIPCC_RTC__)
template <bool MESH, bool SEC, bool X, bool COUNT, bool JIT>
__global__ RTX_RENDER_BOUNDS(MESH, SEC, X) void k_render(const KParams* __restrict__ Pp, const Launch L) {
    render_body<MESH, SEC, X, COUNT, JIT>(Pp, L);
}

template <bool MESH, bool SEC, bool X, bool COUNT, bool JIT>
__global__ RTX_RENDER_BOUNDS(MESH, SEC, X) void k_render_spp(const KParams* __restrict__ Pp, const Launch L) {
    render_body_spp<MESH, SEC, X, COUNT, JIT>(Pp, L);
}

template <bool MESH, bool X>
__global__ __launch_bounds__(256) void k_intersect(SceneView S, int64_t n, const float* __restrict__ ro,
                                                   const float* __restrict__ rd, float time, double* t_out,
                                                   int32_t* obj_out, int32_t* mat_out, float* n_out, float* p_out) {
    extern __shared__ float hstack[];
    const HStack hs{hstack + threadIdx.x, (int)blockDim.x};
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const f3 o = mk(ro[i], ro[n + i], ro[2 * n + i]);
    const f3 d = mk(rd[i], rd[n + i], rd[2 * n + i]);
    Tally tl = {};
    HHit hh;
    const Hit h = closest_hit<MESH, X, false>(S, o, d, time, tl, hs, hh);
    int32_t mat = -1;
    f3 nn = mk(0.0f, 0.0f, 0.0f), pp = mk(0.0f, 0.0f, 0.0f);
    const bool hit = h.obj != -1;
    if (hit) {
        const Surface sf = resolve_hit<MESH, X>(S, h, hh, o, d, time);
        mat = sf.mat;
        nn = sf.normal;
        pp = sf.position;
    }
    if (t_out) t_out[i] = !hit ? (double)INFINITY : h.obj == kHierHit ? hh.t64 : hit_t64(S, h.obj, h.sub, o, d, time);
    if (obj_out) obj_out[i] = !hit ? -1 : h.obj == kHierHit ? h.sub : S.objs[h.obj].oid;
    if (mat_out) mat_out[i] = mat;
    if (n_out) { n_out[i] = nn.x; n_out[n + i] = nn.y; n_out[2 * n + i] = nn.z; }
    if (p_out) { p_out[i] = pp.x; p_out[n + i] = pp.y; p_out[2 * n + i] = pp.z; }
}

template <bool MESH, bool X>
__global__ __launch_bounds__(256) void k_occluded(SceneView S, int64_t n, const float* __restrict__ ro,
                                                  const float* __restrict__ rd, const double* __restrict__ tmax,
                                                  float time, uint8_t* occ) {
    extern __shared__ float hstack[];
    const HStack hs{hstack + threadIdx.x, (int)blockDim.x};
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const f3 o = mk(ro[i], ro[n + i], ro[2 * n + i]);
    const f3 d = mk(rd[i], rd[n + i], rd[2 * n + i]);
    Tally tl = {};
    occ[i] = occluded<MESH, X, false>(S, o, d, tmax[i], time, tl, hs) ? 1 : 0;
}

#if !defined(RTX_EXT_TU)  // defined once, in rtx_api.hip
// The heavy tiles' chunks (one wave per chunk, launched as one-wave blocks), before the
// render kernel: items (bin, chunk). A launch of rows (row0, nrows) or 8-row groups
// (gphase + k gstride) runs only the chunks of its tiles. mode (option chunk_mode):
// bit 0 stages each chunk's face records in LDS first (mesh_chunk_lds); bit 1 hands the
// items to the XCDs in runs of 16 consecutive chunks (xcd_block: the dispatcher deals
// blocks round-robin to the 8 XCDs, so neighbouring chunks -- which share faces -- would
// otherwise pull the same records into all eight L2s).
__global__ __launch_bounds__(64) void k_mesh_chunks(const KParams* __restrict__ Pp, const Launch L,
                                                    const int2* __restrict__ items, int32_t n, uint2* __restrict__ out,
                                                    int32_t mode) {
#if defined(__HIP_DEVICE_COMPILE__)
    __shared__ ChunkLds sh;
#endif
    const uint32_t b = (mode & 2) ? xcd_block(blockIdx.x, gridDim.x, 1) : blockIdx.x;
    const int32_t w = __builtin_amdgcn_readfirstlane((int32_t)b);
    if (w >= n) return;
    const int2 it = items[w];
    const int32_t ty = it.x / Pp->S.bins_x;  // the tile's 8-row group
    const bool mine = L.gstride > 0 ? (ty >= L.gphase && (ty - L.gphase) % L.gstride == 0)
                                    : (ty * 8 + 8 > L.row0 && ty * 8 < L.row0 + L.nrows);
    if (!mine) return;
    const int lane = threadIdx.x & 63;
    const int64_t slot = Pp->S.bin_heavy[it.x];
#if defined(__HIP_DEVICE_COMPILE__)
    if (mode & 1) {
        out[(slot + it.y) * 64 + lane] = mesh_chunk_lds(*Pp, it.x, it.y, lane, sh);
        return;
    }
#endif
    out[(slot + it.y) * 64 + lane] = mesh_chunk(*Pp, it.x, it.y, lane);
}
// (v * 255.0) truncated to uint8, four values per thread: one 16-byte load and one 4-byte
// store (fb 16-byte and out 4-byte aligned; rtx_fb_to_rgb8 checks), the tail one by one.
__device__ __forceinline__ uint8_t to_u8(float v) { return (uint8_t)(int)((double)v * 255.0); }
__global__ __launch_bounds__(256) void k_to_rgb8(const float* __restrict__ fb, uint8_t* __restrict__ out, int64_t n) {
    const int64_t i = 4 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
    if (i + 4 <= n) {
        const float4 v = *reinterpret_cast<const float4*>(fb + i);
        *reinterpret_cast<uchar4*>(out + i) = make_uchar4(to_u8(v.x), to_u8(v.y), to_u8(v.z), to_u8(v.w));
    } else {
        for (int64_t k = i; k < n; ++k) out[k] = to_u8(fb[k]);
    }
}
// Shadow-grid cells from their objects' rectangles (rtx_api.hip dir_shadow_grids): cell c of
// grid `off` ORs the bits of every rectangle of that grid holding it -- the host loop's
// result, without the host filling (and uploading) 2 MB per light.
__global__ __launch_bounds__(256) void k_dsg_fill(const DSRect* __restrict__ r, int32_t nr, DSCell* __restrict__ cells,
                                                  int64_t ncells, int32_t G) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= ncells) return;
    const int64_t gg = (int64_t)G * G, off = c / gg * gg;
    const int32_t q = (int32_t)(c - off), jy = q / G, ix = q - jy * G;
    DSCell v{0u, 0u};
    // the rectangles come grid by grid (off ascending, dir_shadow_grids): this grid's range
    int32_t lo = 0, hi = nr;
    while (lo < hi) {
        const int32_t mid = (lo + hi) >> 1;
        if (r[mid].off < off) lo = mid + 1;
        else hi = mid;
    }
    for (int32_t k = lo; k < nr && r[k].off == off; ++k) {
        const DSRect R = r[k];
        if (ix >= R.i0 && ix <= R.i1 && jy >= R.j0 && jy <= R.j1) {
            v.obj |= R.bit;
            v.root |= R.root;
        }
    }
    cells[c] = v;
}

// Camera uploads (rtx_api.hip pinned_upload): 16-byte words from the scene's pinned host
// buffer, read over the bus by the kernel itself -- no copy engine.
__global__ __launch_bounds__(256) void k_stage_copy(const uint4* __restrict__ src, uint4* __restrict__ dst, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

__global__ __launch_bounds__(256) void k_to_rgb8_unaligned(const float* __restrict__ fb, uint8_t* __restrict__ out,
                                                           int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = to_u8(fb[i]);
}
#endif
#endif  // !__HIPCC_RTC__

}  // namespace rtx
