// rtx_split.h — the hierarchy/texture (X) scenes' render in three passes. The one-kernel
// form (render_body_spp) carries the closest-hit traversal of the hierarchies, their
// shadow traversal and the shading in one register allocation (~195 VGPRs, 2 waves/SIMD).
// The chain of cast_ray (scene.py:81-116) does not depend on the lighting: the next ray
// of a mirror or refractive hit comes from the hit alone (scene.py:97-108), and
// _compute_regular_lighting (scene.py:140-187) only fills the frame that the unwinding
// blends. So the work splits into
//   A (trace):  every sample's chain of closest hits -> one shade-point record per hit;
//   B (shadow): every record's shadow rays (one per light) -> an occlusion bit mask;
//   C (shade):  every sample's lighting from its records (no ray is traced), the unwind
//               of its chain and the pixel's ordered sum (as render_body_spp).
// Each pass is a kernel of its own with its own (smaller) register allocation. The
// arithmetic is the one-kernel form's, operation for operation, so the frame is
// bit-identical (tests/test_gpu_split.py runs the hierarchy scenes both ways).
//
// Records (round 5): structure of arrays, 4-byte words, so every pass reads only what it
// needs and a wave's accesses are coalesced (level-0 records sit at the sample's index;
// deeper ones are appended in wave order):
//   pass B reads  pos (12 B) + meta (4 B)                       and writes occ (4 B);
//   pass C reads  pos, meta, normal (12 B), gobj, next, occ     (40 B).
// The ray direction that hit a record is not stored: C recomputes it walking down the
// chain (the camera ray, then reflect / refract of the parent's stored normal, the same
// fp32 operations as A), so a record is 40 B instead of 64 B.
// The deeper records come from a pool sized by use (rtx_api.hip render_split learns the
// frame's chain depth), not by the worst case of ten levels per sample. A hit that finds
// the pool full marks its pixel block in `redo`, and the block is rendered again by the
// one-kernel form after pass C (render_body_spp with L.redo): the same bytes, so an
// undersized pool costs time, never a wrong pixel.
#pragma once

#include "rtx_kernels.h"

// Occupancy requests (waves per SIMD) of the trace and shadow passes.
// (trace: 4 keeps it at <= 128 VGPRs without spills, as in round 4; the SoA record stores
// had taken it to 129 VGPRs, 3 waves/SIMD)
#ifndef RTX_LB_SPLIT_A
#define RTX_LB_SPLIT_A 4
#endif
#ifndef RTX_LB_SPLIT_B
#define RTX_LB_SPLIT_B 1
#endif

namespace rtx {

// The record arrays of a chunk, each `cap` words.
enum SpArray : int { kSpPx, kSpPy, kSpPz, kSpMeta, kSpNx, kSpNy, kSpNz, kSpGobj, kSpNext, kSpOcc, kSpArrays };
constexpr int64_t kSpBytes = 4 * kSpArrays;  // bytes per record
// meta: 0 = no hit (black); else kSpHit | kSpChain (a mirror / refractive hit whose child
// ray was cast) | the motion-time index << 2 | the material << kSpMatShift.
constexpr uint32_t kSpHit = 1u, kSpChain = 2u;
constexpr int kSpTimeBits = 10, kSpMatShift = 2 + kSpTimeBits;
// (the split path serves scenes within these: rtx_api.hip render_launch)
constexpr int64_t kSpMaxTimes = 1 << kSpTimeBits, kSpMaxMats = 1 << 16;

struct SplitBuf {
    uint32_t* w;          // kSpArrays arrays of cap words
    unsigned int* count;  // deeper records appended in this chunk (zero before A)
    uint32_t* redo_n;     // shade blocks listed for the redo launch (zero before A)
    uint32_t* redo_list;  // their indices
    uint32_t* redo_flag;  // per shade block of the chunk: listed (cleared by the redo launch)
    int64_t nsamp;        // samples of the chunk (= its level-0 records)
    int64_t cap;          // records the arrays hold
    RTX_HD uint32_t* u(int a) const { return w + a * cap; }
    RTX_HD float* f(int a) const { return reinterpret_cast<float*>(w + a * cap); }
    RTX_HD int32_t* i(int a) const { return reinterpret_cast<int32_t*>(w + a * cap); }
};

// Sample q of the chunk (q = pixel * spp + s, the reference's dof -> aa -> time order with
// time fastest, as render_body_spp): pixel and sample indices.
struct SampleIx {
    int32_t qp;  // the chunk's pixel
    int32_t rr, cc, j, kd, ka, kt;
};
RTX_HD SampleIx sample_ix(const KParams& P, const Launch& L, int64_t q, int S, int nt, int na) {
    SampleIx x;
    const uint32_t qp = (uint32_t)q / (uint32_t)S;  // (chunks hold < 2^31 samples)
    const int s = (int)((uint32_t)q - qp * (uint32_t)S);
    const int64_t p = L.pix0 + (int64_t)qp;
    x.qp = (int32_t)qp;
    x.rr = (int32_t)(p / P.ncols);
    x.cc = (int32_t)(p - (int64_t)x.rr * P.ncols);
    x.j = P.height - 1 - image_row(L, x.rr);
    const int da = s / nt;
    x.kt = s - da * nt;
    x.kd = da / na;
    x.ka = da - x.kd * na;
    return x;
}

// Lists shade block b for the redo launch (once).
RTX_HD void list_redo(const SplitBuf& sb, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (atomicExch(&sb.redo_flag[b], 1u) == 0u) sb.redo_list[atomicAdd(sb.redo_n, 1u)] = b;
#else
    if (__atomic_exchange_n(&sb.redo_flag[b], 1u, __ATOMIC_RELAXED) == 0u)
        sb.redo_list[__atomic_fetch_add(sb.redo_n, 1u, __ATOMIC_RELAXED)] = b;
#endif
}

// The camera ray's direction of a sample (scene.py:58).
RTX_HD f3 sample_dir(const KParams& P, const SampleIx& x) {
    return normalize(sub(pixel_focal(P, x.cc, x.j), ld3(P.dof_o + 3 * x.kd)));
}

// Pass A for sample q: the chain of closest hits (cast_ray's loop without the lighting).
// alloc(hit) returns the appended record of a deeper hit (every lane of the wave calls it
// at the same level; lanes without a hit get -1, lanes whose hit finds the pool full -2).
template <bool MESH, bool SEC, bool COUNT, bool JIT, class Alloc>
RTX_HD void trace_sample(const KParams& P, const Launch& L, const SplitBuf& sb, int64_t q, Tally& tl,
                         const HStack& hs, Alloc& alloc) {
    const SceneView& S = P.S;
    const int nt = RTX_NTIMES(P), na = RTX_NAA(P);
    const int Sn = RTX_NDOF(P) * na * nt;
    const SampleIx x = sample_ix(P, L, q, Sn, nt, na);
    f3 d = sample_dir(P, x);
    f3 o = sample_origin<JIT>(P, x.cc, x.j, x.kd, x.ka);
    const float time = P.times[x.kt];
    // the primary-ray bin of the wave's pixels when they share one (rtx_api.hip primary_bins)
    int32_t bin = -1;
#if !(defined(RTX_PRIMARY_BINS) && !RTX_PRIMARY_BINS)
    if (S.bins_on) {
        const int32_t b = (image_row(L, x.rr) >> 3) * S.bins_x + (x.cc >> 3);
        const int32_t b0 = wave_uniform(b);
        bin = RTX_ALL(b == b0) ? b0 : -1;
    }
#endif
    int64_t slot = q, parent = -1;
    bool in_shape = false;
    for (int level = 0; level < (SEC ? kMaxDepth : 1); ++level) {
        if (COUNT) tl.cast[level]++;
        HHit hh;
        const Hit h = closest_hit<MESH, true, COUNT>(S, o, d, time, tl, hs, hh, level == 0 ? bin : -1);
        const bool hit = h.obj != -1;
        if (level > 0) {  // a deeper hit is appended and linked from its parent
            slot = alloc(hit);
            if (slot >= 0) {
                sb.i(kSpNext)[parent] = (int32_t)slot;
            } else if (hit) {  // the pool is full: the one-kernel form renders the block again
                list_redo(sb, (uint32_t)x.qp / (uint32_t)spp_pixels_per_block(Sn, kBlock<true>));
                return;
            }
        }
        if (!hit) {
            if (level == 0) sb.u(kSpMeta)[q] = 0u;  // miss -> black
            return;
        }
        const Surface sf = resolve_hit<MESH, true>(S, h, hh, o, d, time);
        const DMat m = RTX_MAT(S, sf.mat);
        f3 n = sf.normal;
        bool chain = false, tir = false;
        f3 next_o = o, next_d = d;
        if (SEC && m.type == MAT_MIRROR) {  // reflect; child with in_shape = False
            const f3 rdir = reflect(d, n);
            next_o = add(sf.position, scale(rdir, 0.01f));
            next_d = rdir;
            chain = true;
        } else if (SEC && m.type == MAT_REFRACTIVE) {  // the negated normal also shades
            const float eta = in_shape ? m.eta_in : m.eta_out;
            if (in_shape) n = neg(n);
            const f3 rdir = refract(d, n, eta);
            tir = is_zero(rdir);
            next_o = add(sf.position, scale(rdir, 0.0001f));
            next_d = rdir;
            chain = true;
        }
        sb.f(kSpPx)[slot] = sf.position.x;
        sb.f(kSpPy)[slot] = sf.position.y;
        sb.f(kSpPz)[slot] = sf.position.z;
        sb.u(kSpMeta)[slot] = kSpHit | (chain ? kSpChain : 0u) | ((uint32_t)x.kt << 2) | ((uint32_t)sf.mat << kSpMatShift);
        sb.f(kSpNx)[slot] = n.x;
        sb.f(kSpNy)[slot] = n.y;
        sb.f(kSpNz)[slot] = n.z;
        sb.i(kSpGobj)[slot] = sf.gobj;
        sb.i(kSpNext)[slot] = -1;
        if (!SEC || !chain || tir) return;
        in_shape = m.type == MAT_REFRACTIVE ? !in_shape : false;
        o = next_o;
        d = next_d;
        parent = slot;
    }
}

// Pass B for one shading point: its shadow rays (regular_lighting's per-light rays,
// scene.py:148-164) -> occlusion mask.
template <bool MESH, bool COUNT>
RTX_HD uint32_t shadow_mask(const SceneView& S, f3 pos, float time, Tally& tl, const HStack& hs) {
    tally_inc<COUNT>(tl, &Tally::shade);
    uint32_t occm = 0u;
    for (int li = 0; li < RTX_NLIGHTS(S); ++li) {
        const DLight Lt = S.lights[li];
        f3 sdir;
        double t_max;
        if (Lt.type == LIGHT_POINT) {
            sdir = sub(ld3(Lt.vec), pos);
            t_max = 1.0;
        } else {
            sdir = ld3(Lt.negvec);
            t_max = INFINITY;
        }
        tally_inc<COUNT>(tl, &Tally::shadow);
        if (occluded<MESH, true, COUNT>(S, pos, sdir, t_max, time, tl, hs, nullptr, li)) occm |= 1u << li;
    }
    return occm;
}

// Pass C for the sample q (whose level-0 record is q): cast_ray's value (scene.py:97-116)
// from its chain of records. Walking down the `next` links it recomputes each record's
// incoming ray direction and lights the record (regular_lighting with the record's
// occlusion mask; no ray traced); the lighting and material of every level that blends
// with a child go to a frame stack (LDS on the device), the deepest level's stays in
// registers; then it blends bottom-up -- the unwinding order.
// The stack: per frame three floats and a 16-bit material index (the split path serves
// scenes with at most 2^16 materials), [frame][word][lane] so lanes hit distinct banks.
struct ShadeStack {
    float* f;     // [kMaxDepth - 1][3][stride]
    uint16_t* m;  // [kMaxDepth - 1][stride]
    int stride;
    RTX_HD void put(int k, f3 L, int32_t mat) const {
        float* p = f + 3 * k * stride;
        p[0] = L.x;
        p[stride] = L.y;
        p[2 * stride] = L.z;
        m[k * stride] = (uint16_t)mat;
    }
    RTX_HD f3 get(int k, int32_t& mat) const {
        const float* p = f + 3 * k * stride;
        mat = m[k * stride];
        return f3{p[0], p[stride], p[2 * stride]};
    }
};
constexpr int kShadeFrames = kMaxDepth - 1;  // the deepest level never blends with a child

template <bool MESH, bool SEC>
RTX_HD f3 shade_sample(const KParams& P, const Launch& L, const SplitBuf& sb, int64_t q, const ShadeStack& fs) {
    const SceneView& S = P.S;
    uint32_t meta = sb.u(kSpMeta)[q];
    if (!(meta & kSpHit)) return mk(0.0f, 0.0f, 0.0f);  // miss -> black
    const int nt = RTX_NTIMES(P), na = RTX_NAA(P);
    const int Sn = RTX_NDOF(P) * na * nt;
    const SampleIx x = sample_ix(P, L, q, Sn, nt, na);
    const float time = P.times[x.kt];
    f3 d = sample_dir(P, x);
    int nfr = 0;  // frames on the stack (levels whose colour blends with a child's)
    bool in_shape = false;
    int64_t r = q;
    Tally tl = {};
    const HStack hs{nullptr, 1};
    f3 tail = mk(0.0f, 0.0f, 0.0f);
    for (int k = 0; k < (SEC ? kMaxDepth : 1); ++k) {
        const int32_t mi = (int32_t)(meta >> kSpMatShift);
        const DMat m = RTX_MAT(S, mi);
        const f3 pos = mk(sb.f(kSpPx)[r], sb.f(kSpPy)[r], sb.f(kSpPz)[r]);
        const f3 n = mk(sb.f(kSpNx)[r], sb.f(kSpNy)[r], sb.f(kSpNz)[r]);
        const int32_t gobj = sb.i(kSpGobj)[r];
        const f3 diffuse = gobj >= 0 ? get_diffuse(S, S.objs[gobj], pos, time) : ld3(m.diffuse);
        const f3 lit = regular_lighting<MESH, true, false>(S, d, pos, n, m, diffuse, time, tl, hs, (int64_t)sb.u(kSpOcc)[r]);
        if (!SEC || !(meta & kSpChain)) {  // a diffuse hit ends the chain with its clamped colour
            tail = clamp01(lit);
            break;
        }
        const int32_t nx = sb.i(kSpNext)[r];
        if (nx < 0) {  // the child ray missed, or total internal reflection: black child
            tail = clamp01(add(scale(lit, m.tint), scale(tail, m.omt)));
            break;
        }
        fs.put(nfr++, lit, mi);
        // the child's ray, as trace_sample cast it (the stored normal is already negated
        // inside a refractive object)
        if (m.type == MAT_MIRROR) {
            d = reflect(d, n);
            in_shape = false;
        } else {
            d = refract(d, n, in_shape ? m.eta_in : m.eta_out);
            in_shape = !in_shape;
        }
        r = nx;
        meta = sb.u(kSpMeta)[r];
    }
    // from the deepest blending level up: colour = clamp(L * tint + child * (1 - tint))
    for (int k = nfr - 1; k >= 0; --k) {
        int32_t mi;
        const f3 lit = fs.get(k, mi);
        const DMat m = RTX_MAT(S, mi);
        tail = clamp01(add(scale(lit, m.tint), scale(tail, m.omt)));
    }
    return tail;
}

// Pass A: work item = sample; a wave's lanes are consecutive samples (coherent rays for
// the wave-uniform culling). Deeper hits take appended records, one atomic per wave.
template <bool MESH, bool SEC, bool COUNT, bool JIT>
__device__ __forceinline__ void split_trace(const KParams* __restrict__ Pp, const Launch L, SplitBuf sb) {
    constexpr int B = kBlock<true>;
    extern __shared__ float hstack[];
    const HStack hs{hstack + threadIdx.x, B};
    Tally tl = {};
    const int64_t q = (int64_t)blockIdx.x * B + threadIdx.x;
    const bool active = q < sb.nsamp;
    if (active) {
        auto alloc = [&](bool hit) -> int64_t {
#if defined(__HIP_DEVICE_COMPILE__)
            const uint64_t want = __builtin_amdgcn_ballot_w64(hit);
            uint32_t base = 0;
            if (want) {
                const int lead = __builtin_ctzll(want);
                if ((int)(threadIdx.x & 63) == lead) base = atomicAdd(sb.count, (unsigned)__builtin_popcountll(want));
                base = __builtin_amdgcn_readlane(base, lead);
            }
            if (!hit) return -1;
            const int64_t slot = sb.nsamp + base +
                                 (int64_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(want >> 32),
                                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)want, 0u));
            return slot < sb.cap ? slot : -2;
#else
            (void)hit;
            return -1;
#endif
        };
        trace_sample<MESH, SEC, COUNT, JIT>(*Pp, L, sb, q, tl, hs, alloc);
    }
    flush_tally<COUNT>(tl, L.counters, active);
}

// Pass B: records in index order (level 0 in sample order, then the appended deeper
// hits), grid-stride over the chunk's records.
template <bool MESH, bool COUNT>
__device__ __forceinline__ void split_shadow(const KParams* __restrict__ Pp, const Launch L, SplitBuf sb) {
    constexpr int B = kBlock<true>;
    extern __shared__ float hstack[];
    const HStack hs{hstack + threadIdx.x, B};
    Tally tl = {};
    const SceneView S = Pp->S;
    const int64_t n = min(sb.nsamp + (int64_t)*sb.count, sb.cap);  // (appends past cap were refused)
    bool any = false;
    for (int64_t r = (int64_t)blockIdx.x * B + threadIdx.x; r - (int64_t)threadIdx.x < n;
         r += (int64_t)gridDim.x * B) {
        const uint32_t meta = r < n ? sb.u(kSpMeta)[r] : 0u;
        const bool hit = (meta & kSpHit) != 0u;
        if (!RTX_ANY(hit)) continue;
        any = true;
        if (hit) {
            const f3 pos = mk(sb.f(kSpPx)[r], sb.f(kSpPy)[r], sb.f(kSpPz)[r]);
            const float time = Pp->times[(meta >> 2) & (kSpMaxTimes - 1)];
            sb.u(kSpOcc)[r] = shadow_mask<MESH, COUNT>(S, pos, time, tl, hs);
        }
    }
    flush_tally<COUNT>(tl, L.counters, any);
}

// Pass C: render_body_spp's mapping and ordered sums, with shade_sample for cast_ray.
template <bool MESH, bool SEC>
__device__ __forceinline__ void split_shade(const KParams* __restrict__ Pp, const Launch L, SplitBuf sb) {
    constexpr int B = kBlock<true>;
    const KParams& P = *Pp;
    const int nt = RTX_NTIMES(P), na = RTX_NAA(P);
    const int Sn = RTX_NDOF(P) * na * nt;
    const int PPB = spp_pixels_per_block(Sn, B);
    const int rounds = (PPB * Sn + B - 1) / B;
    const float rS = 1.0f / (float)Sn;  // (a block's samples < 2^22: udiv_small)
    // LDS: the frame stacks (SEC: 9 x 14 B per lane, 8,064 B per one-wave block, so 20
    // blocks share a CU's 160 KB: 5 waves/SIMD) and, aliased onto them, the colours of the
    // block's samples, written after every lane's stack is dead (one wave per block)
    constexpr int kStackWords = SEC ? kShadeFrames * 3 * B + kShadeFrames * B / 2 : 0;
    __shared__ float lds[kStackWords > 3 * B ? kStackWords : 3 * B];
    float* const sbuf = lds;
    static_assert(!SEC || B == 64, "the aliased colour buffer needs one wave per block");
    const ShadeStack fs{lds + threadIdx.x, reinterpret_cast<uint16_t*>(lds + kShadeFrames * 3 * B) + threadIdx.x, B};
    const int64_t npix = sb.nsamp / Sn;  // the chunk's pixels
    const int64_t pix0 = (int64_t)blockIdx.x * PPB;
    const int tid = threadIdx.x;
    float acc = 0.0f;
    for (int rd = 0; rd < rounds; ++rd) {
        const int flat = rd * B + tid;
        int s;
        const int lp = udiv_small(flat, Sn, rS, s);
        const int64_t p = pix0 + lp;
        f3 c = mk(0.0f, 0.0f, 0.0f);
        if (lp < PPB && p < npix) c = shade_sample<MESH, SEC>(P, L, sb, p * Sn + s, fs);
        sbuf[tid] = c.x;
        sbuf[B + tid] = c.y;
        sbuf[2 * B + tid] = c.z;
        __syncthreads();
        if (rounds == 1) {
            for (int qq = tid; qq < 3 * PPB; qq += B) {
                const int pp = qq / 3, ch = qq - 3 * (qq / 3);
                if (pix0 + pp < npix) {
                    const float* src = sbuf + ch * B + pp * Sn;
                    float a = 0.0f;
                    for (int k = 0; k < Sn; ++k) a += src[k];
                    put_channel(frame_fb(L), 3 * (L.pix0 + pix0 + pp) + ch, sample_mean(P, a));
                }
            }
        } else if (tid < 3) {
            const int hi = min(Sn - rd * B, B);
            const float* src = sbuf + tid * B;
            for (int k = 0; k < hi; ++k) acc += src[k];
        }
        if (rounds > 1) __syncthreads();
    }
    if (rounds > 1 && tid < 3 && pix0 < npix) put_channel(frame_fb(L), 3 * (L.pix0 + pix0) + tid, sample_mean(P, acc));
}

// Chunking of a frame (host; rtx_api.hip render_split and the host emulation share it):
// a chunk is whole shade blocks of pixels; its record arrays hold one level-0 record per
// sample plus `ratio` deeper records per sample, within `budget` bytes.
struct SplitPlan {
    int64_t chunk;  // pixels per chunk (a multiple of the shade block unless it is the whole frame)
    int64_t cap;    // records per chunk
};
#if !defined(__HIPCC_RTC__)
inline SplitPlan split_plan(int64_t npix, int spp, int ppb, double ratio, int64_t budget) {
    const double per_pix = (double)spp * (1.0 + ratio) * (double)kSpBytes;
    int64_t chunk = std::max<int64_t>(1, (int64_t)((double)budget / per_pix));
    if (chunk < npix) chunk = std::max<int64_t>(ppb, chunk / ppb * ppb);
    chunk = std::min(chunk, npix);
    const int64_t nsamp = chunk * spp;
    return SplitPlan{chunk, nsamp + (int64_t)std::ceil((double)nsamp * ratio)};
}
#endif

#if !defined(__HIPCC_RTC__)
template <bool MESH, bool SEC, bool COUNT, bool JIT>
__global__ __launch_bounds__(kBlock<true>, RTX_LB_SPLIT_A) void k_split_trace(const KParams* __restrict__ Pp,
                                                                              const Launch L, SplitBuf sb) {
    split_trace<MESH, SEC, COUNT, JIT>(Pp, L, sb);
}
template <bool MESH, bool COUNT>
__global__ __launch_bounds__(kBlock<true>, RTX_LB_SPLIT_B) void k_split_shadow(const KParams* __restrict__ Pp,
                                                                               const Launch L, SplitBuf sb) {
    split_shadow<MESH, COUNT>(Pp, L, sb);
}
// (shade: 5 waves/SIMD, which its LDS stacks allow, needs <= 96 VGPRs)
template <bool MESH, bool SEC>
__global__ __launch_bounds__(kBlock<true>, 5) void k_split_shade(const KParams* __restrict__ Pp, const Launch L,
                                                              SplitBuf sb) {
    split_shade<MESH, SEC>(Pp, L, sb);
}
#endif

}  // namespace rtx
