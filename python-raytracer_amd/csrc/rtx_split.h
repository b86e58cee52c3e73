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
// bit-identical (tests/test_gpu_parity.py runs the hierarchy scenes both ways).
// A frame is processed in chunks of whole pixels, so the records fit a fixed buffer
// (rtx_api.hip render_split).
#pragma once

#include "rtx_kernels.h"

// Occupancy requests (waves per SIMD) of the trace and shadow passes.
#ifndef RTX_LB_SPLIT_A
#define RTX_LB_SPLIT_A 1
#endif
#ifndef RTX_LB_SPLIT_B
#define RTX_LB_SPLIT_B 1
#endif

namespace rtx {

// One hit of a sample's chain (64 B, written by A, its mask by B, read by C).
struct alignas(16) ShadePt {
    float pos[3];
    float time;
    float n[3];     // the normal the lighting uses (negated inside a refractive object)
    int32_t mat;
    float d[3];     // the ray direction that hit (the specular half vector)
    int32_t gobj;   // DObj whose get_diffuse shades the hit, or -1
    int32_t next;   // the record of the child's hit, or -1 (black child / none)
    uint32_t flags; // kSpHit | kSpChain
    uint32_t occ;   // B: bit li = light li's shadow ray is occluded
    int32_t prev;   // the parent's record (the hit whose reflect/refract ray this is), or -1
};
constexpr uint32_t kSpHit = 1u, kSpChain = 2u;

// The chunk's record buffer: level-0 records at [0, nsamp) (one per sample, in sample
// order), the chain's deeper hits appended at nsamp + (*count)++.
struct SplitBuf {
    ShadePt* rec;
    unsigned int* count;  // appended records (reset before A)
    int64_t nsamp;        // samples of the chunk
    int64_t cap;          // records the buffer holds
};

// Sample q of the chunk (q = pixel * spp + s, the reference's dof -> aa -> time order with
// time fastest, as render_body_spp): pixel and sample indices.
struct SampleIx {
    int32_t rr, cc, j, kd, ka, kt;
};
RTX_HD SampleIx sample_ix(const KParams& P, const Launch& L, int64_t q, int S, int nt, int na) {
    SampleIx x;
    const uint32_t qp = (uint32_t)q / (uint32_t)S;  // (chunks hold < 2^31 samples)
    const int s = (int)((uint32_t)q - qp * (uint32_t)S);
    const int64_t p = L.pix0 + (int64_t)qp;
    x.rr = (int32_t)(p / P.ncols);
    x.cc = (int32_t)(p - (int64_t)x.rr * P.ncols);
    x.j = P.height - 1 - image_row(L, x.rr);
    const int da = s / nt;
    x.kt = s - da * nt;
    x.kd = da / na;
    x.ka = da - x.kd * na;
    return x;
}

// Pass A for sample q: the chain of closest hits (cast_ray's loop without the lighting).
// alloc(hit) returns the appended record of a deeper hit (every lane of the wave calls it
// at the same level; lanes without a hit get -1).
template <bool MESH, bool SEC, bool COUNT, bool JIT, class Alloc>
RTX_HD void trace_sample(const KParams& P, const Launch& L, const SplitBuf& sb, int64_t q, Tally& tl,
                         const HStack& hs, Alloc& alloc) {
    const SceneView& S = P.S;
    const int nt = RTX_NTIMES(P), na = RTX_NAA(P);
    const int Sn = RTX_NDOF(P) * na * nt;
    const SampleIx x = sample_ix(P, L, q, Sn, nt, na);
    const f3 focal = pixel_focal(P, x.cc, x.j);
    f3 d = normalize(sub(focal, ld3(P.dof_o + 3 * x.kd)));  // scene.py:58
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
            if (slot >= 0) sb.rec[parent].next = (int32_t)slot;
        }
        if (!hit) {
            if (level == 0) sb.rec[q].flags = 0u;  // miss -> black
            return;
        }
        if (slot < 0) return;  // (cannot happen: the chunk's buffer holds every level)
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
        ShadePt r;
        r.pos[0] = sf.position.x; r.pos[1] = sf.position.y; r.pos[2] = sf.position.z;
        r.time = time;
        r.n[0] = n.x; r.n[1] = n.y; r.n[2] = n.z;
        r.mat = sf.mat;
        r.d[0] = d.x; r.d[1] = d.y; r.d[2] = d.z;
        r.gobj = sf.gobj;
        r.next = -1;
        r.flags = kSpHit | (chain ? kSpChain : 0u);
        r.occ = 0u;
        r.prev = (int32_t)parent;
        sb.rec[slot] = r;
        if (!SEC || !chain || tir) return;
        in_shape = m.type == MAT_REFRACTIVE ? !in_shape : false;
        o = next_o;
        d = next_d;
        parent = slot;
    }
}

// Pass B for one record: its shadow rays (regular_lighting's per-light rays, scene.py:
// 148-164) -> occlusion mask.
template <bool MESH, bool COUNT>
RTX_HD uint32_t shadow_record(const SceneView& S, const ShadePt& R, Tally& tl, const HStack& hs) {
    const f3 pos = mk(R.pos[0], R.pos[1], R.pos[2]);
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
        if (occluded<MESH, true, COUNT>(S, pos, sdir, t_max, R.time, tl, hs, nullptr, li)) occm |= 1u << li;
    }
    return occm;
}

// The lighting of one record (scene.py:140-187 with its occlusion mask; no ray traced).
template <bool MESH>
RTX_HD f3 record_lighting(const SceneView& S, const ShadePt& R, const DMat& m) {
    Tally tl = {};
    const HStack hs{nullptr, 1};
    const f3 pos = mk(R.pos[0], R.pos[1], R.pos[2]);
    const f3 diffuse = R.gobj >= 0 ? get_diffuse(S, S.objs[R.gobj], pos, R.time) : ld3(m.diffuse);
    return regular_lighting<MESH, true, false>(S, mk(R.d[0], R.d[1], R.d[2]), pos, mk(R.n[0], R.n[1], R.n[2]), m,
                                               diffuse, R.time, tl, hs, (int64_t)R.occ);
}

// Pass C for the sample whose level-0 record is r: cast_ray's value (scene.py:97-116)
// from its chain of records. The chain is walked to its deepest record by the `next`
// links, then back up by the `prev` links, lighting each record on the way up and
// blending it into the child's colour -- the unwinding order, with no frame stack.
template <bool MESH, bool SEC>
RTX_HD f3 shade_sample(const SceneView& S, const SplitBuf& sb, int64_t r) {
    if (!(sb.rec[r].flags & kSpHit)) return mk(0.0f, 0.0f, 0.0f);  // miss -> black
    if (SEC)
        for (int32_t nx = sb.rec[r].next; nx >= 0; nx = sb.rec[r].next) r = nx;
    // from the deepest record up: a diffuse hit ends the chain with its own clamped
    // colour; a mirror / refractive one blends its lighting with its child's colour (black
    // when the child ray was not traced or missed: TIR, the depth limit)
    f3 tail = mk(0.0f, 0.0f, 0.0f);
    bool deepest = true;
    for (int64_t p = r; p >= 0;) {
        const ShadePt R = sb.rec[p];
        const DMat m = RTX_MAT(S, R.mat);
        const f3 L = record_lighting<MESH>(S, R, m);
        tail = (deepest && !(R.flags & kSpChain)) ? clamp01(L) : clamp01(add(scale(L, m.tint), scale(tail, m.omt)));
        deepest = false;
        p = SEC ? R.prev : -1;
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
            return slot < sb.cap ? slot : -1;
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
// hits), grid-stride over the chunk's count.
template <bool MESH, bool COUNT>
__device__ __forceinline__ void split_shadow(const KParams* __restrict__ Pp, const Launch L, SplitBuf sb) {
    constexpr int B = kBlock<true>;
    extern __shared__ float hstack[];
    const HStack hs{hstack + threadIdx.x, B};
    Tally tl = {};
    const SceneView S = Pp->S;
    const int64_t n = sb.nsamp + (int64_t)*sb.count;
    bool any = false;
    for (int64_t r = (int64_t)blockIdx.x * B + threadIdx.x; r - (int64_t)threadIdx.x < n;
         r += (int64_t)gridDim.x * B) {
        const bool hit = r < n && (sb.rec[r].flags & kSpHit);
        if (!RTX_ANY(hit)) continue;
        any = true;
        if (hit) sb.rec[r].occ = shadow_record<MESH, COUNT>(S, sb.rec[r], tl, hs);
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
    __shared__ float sbuf[3 * B];
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
        if (lp < PPB && p < npix) c = shade_sample<MESH, SEC>(P.S, sb, p * Sn + s);
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
template <bool MESH, bool SEC>
__global__ __launch_bounds__(kBlock<true>) void k_split_shade(const KParams* __restrict__ Pp, const Launch L,
                                                              SplitBuf sb) {
    split_shade<MESH, SEC>(Pp, L, sb);
}
#endif

}  // namespace rtx
