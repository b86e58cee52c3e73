// rtx_api.hip — MI355X (gfx950) render kernels and the C ABI of librtx.so (include/rtx.h).
//
// Kernels
//   k_render      one work-item per output pixel; loops the pixel's DOF x AA x motion
//                 samples in the reference's order (scene.py:57-73) so the fp32 colour
//                 sum is accumulated exactly as the reference does; each sample runs the
//                 iterative cast_ray of rtx_trace.h. Scene records are read with
//                 wave-uniform indices (scalar loads through the constant cache).
//   k_intersect   closest hit of SoA rays (Geometry.intersect + min, scene.py:86-94)
//   k_occluded    shadow any-hit of SoA rays (Geometry.shadow_intersect, scene.py:160-164)
//   k_to_rgb8     (v * 255.0) truncated to uint8 (main.py:327)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rtx.h"
#include "rtx_trace.h"

using namespace rtx;

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

#define RTX_HIP(call)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (call);                                                           \
        if (e_ != hipSuccess)                                                             \
            return fail(RTX_ERR_HIP, std::string(#call ": ") + hipGetErrorString(e_));    \
    } while (0)

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

// scene.py:47-79 for pixel p of the output block (host/device: the tests-only host
// emulation runs the same body).
template <bool MESH, bool SEC, bool COUNT, bool JIT>
RTX_HD void render_pixel(const KParams& P, float* fb, int32_t row0, int32_t rr, int32_t cc, Tally& tl,
                         const FrameStack& fs) {
    const int64_t p = (int64_t)rr * P.ncols + cc;
    const int j = P.height - 1 - (row0 + rr);  // reference row index (y grows upward)
    const float fx = P.xs[cc];
    const float fy = P.ys[j];
    // base_ray_direction = normalize(x * u + y * v - d * w)  (scene.py:54)
    const f3 bdir = normalize(sub(add(scale(ld3(P.u), fx), scale(ld3(P.v), fy)), ld3(P.dw)));
    const f3 focal = add(ld3(P.pos), scale(bdir, P.focal));  // scene.py:55
    f3 colour = mk(0.0f, 0.0f, 0.0f);
    for (int kd = 0; kd < P.n_dof; ++kd) {
        const f3 ddir = normalize(sub(focal, ld3(P.dof_o + 3 * kd)));  // scene.py:58
        for (int ka = 0; ka < P.n_aa; ++ka) {
            f3 o = ld3(P.aa_o + 3 * (kd * P.n_aa + ka));
            if (JIT) {  // scene.py:63-65
                f3 rnd;
                if (P.jitter == RTX_JITTER_REPLAY) {
                    const int64_t idx = (((int64_t)cc * P.height + j) * P.n_dof + kd) * P.n_aa + ka;
                    rnd = ld3(P.noise + 3 * idx);
                } else {
                    uint32_t ctr[4] = {(uint32_t)(P.col0 + cc), (uint32_t)j, (uint32_t)(kd * P.n_aa + ka), 0u};
                    philox4x32(ctr, P.seed_lo, P.seed_hi);
                    rnd = mk((float)(ctr[0] >> 8) * 0x1p-24f, (float)(ctr[1] >> 8) * 0x1p-24f,
                             (float)(ctr[2] >> 8) * 0x1p-24f);
                }
                o = add(o, scale(normalize(rnd), P.jscale));
            }
            for (int kt = 0; kt < P.n_times; ++kt)
                colour = add(colour, cast_ray<MESH, SEC, COUNT>(P.S, o, ddir, P.times[kt], tl, fs));
        }
    }
    // colour / (samples * dof_samples * len(motion_times)) (scene.py:73); for a power of
    // two the exact reciprocal multiply gives the identical correctly rounded result.
    if (P.div_pow2) colour = scale(colour, P.inv_divisor);
    else colour = divs(colour, P.divisor);
    float* out = fb + 3 * p;
    out[0] = colour.x;
    out[1] = colour.y;
    out[2] = colour.z;
}

// The per-frame parameters live in device memory (uploaded by rtx_camera_set) and are
// read with scalar loads; only the per-call output block is passed by value.
struct Launch {
    float* fb;
    unsigned long long* counters;
    int32_t row0, nrows;
};

// Occupancy request (waves per SIMD) by kernel variant: mesh kernels without secondary
// rays fit 128 VGPRs without scratch and gain from 4 waves/SIMD; the others spill if
// forced below their natural allocation (measured, tools/ablate.sh).
#ifndef RTX_LB_WAVES
#define RTX_LB_WAVES(MESH, SEC) ((MESH) && !(SEC) ? 4 : 1)
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
__device__ __forceinline__ PixelRC pixel_rc(int32_t ncols, int sub) {
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(
        (int)((blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * RTX_PPL + sub));
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

template <bool MESH, bool SEC, bool COUNT, bool JIT>
__global__ __launch_bounds__(256, RTX_LB_WAVES(MESH, SEC)) void k_render(const KParams* __restrict__ Pp, const Launch L) {
    const int32_t ncols = Pp->ncols;
    Tally tl = {};
    // secondary-ray frames: [frame][word][thread] in LDS (40 KB per 256-thread block)
    __shared__ float frames[SEC ? kMaxDepth * 4 * 256 : 1];
    const FrameStack fs{frames + threadIdx.x, 256};
    bool any_active = false;
    for (int sub = 0; sub < RTX_PPL; ++sub) {
        const PixelRC px = pixel_rc(ncols, sub);
        const bool active = px.r < L.nrows && px.c < ncols;
        any_active = any_active || active;
        if (active) render_pixel<MESH, SEC, COUNT, JIT>(*Pp, L.fb, L.row0, px.r, px.c, tl, fs);
    }
    flush_tally<COUNT>(tl, L.counters, any_active);
}

template <bool MESH>
__global__ __launch_bounds__(256) void k_intersect(SceneView S, int64_t n, const float* __restrict__ ro,
                                                   const float* __restrict__ rd, float time, double* t_out,
                                                   int32_t* obj_out, int32_t* mat_out, float* n_out, float* p_out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const f3 o = mk(ro[i], ro[n + i], ro[2 * n + i]);
    const f3 d = mk(rd[i], rd[n + i], rd[2 * n + i]);
    Tally tl = {};
    const Hit h = closest_hit<MESH, false>(S, o, d, time, tl);
    int32_t mat = -1;
    f3 nn = mk(0.0f, 0.0f, 0.0f), pp = mk(0.0f, 0.0f, 0.0f);
    if (h.obj >= 0) {
        const Surface sf = resolve_hit<MESH>(S, h, o, d, time);
        mat = sf.mat;
        nn = sf.normal;
        pp = sf.position;
    }
    if (t_out) t_out[i] = h.obj >= 0 ? hit_t64(S, h.obj, h.sub, o, d, time) : (double)INFINITY;
    if (obj_out) obj_out[i] = h.obj >= 0 ? S.objs[h.obj].oid : -1;
    if (mat_out) mat_out[i] = mat;
    if (n_out) { n_out[i] = nn.x; n_out[n + i] = nn.y; n_out[2 * n + i] = nn.z; }
    if (p_out) { p_out[i] = pp.x; p_out[n + i] = pp.y; p_out[2 * n + i] = pp.z; }
}

template <bool MESH>
__global__ __launch_bounds__(256) void k_occluded(SceneView S, int64_t n, const float* __restrict__ ro,
                                                  const float* __restrict__ rd, const double* __restrict__ tmax,
                                                  float time, uint8_t* occ) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const f3 o = mk(ro[i], ro[n + i], ro[2 * n + i]);
    const f3 d = mk(rd[i], rd[n + i], rd[2 * n + i]);
    Tally tl = {};
    occ[i] = occluded<MESH, false>(S, o, d, tmax[i], time, tl) ? 1 : 0;
}

__global__ __launch_bounds__(256) void k_to_rgb8(const float* __restrict__ fb, uint8_t* __restrict__ out, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = (uint8_t)(int)((double)fb[i] * 255.0);
}

}  // namespace

// ------------------------------------------------------------------ host-side conversion
// rtx_*_desc (ABI) -> device records. Pure host code with no HIP calls, shared with the
// tests-only host emulation build (tests/native/rtx_hostemu.hip).
namespace {

void set3(float* dst, const float* s) { dst[0] = s[0]; dst[1] = s[1]; dst[2] = s[2]; dst[3] = 0.0f; }
void set3(float* dst, f3 s) { dst[0] = s.x; dst[1] = s.y; dst[2] = s.z; dst[3] = 0.0f; }
bool finite3(const float* v) { return std::isfinite(v[0]) && std::isfinite(v[1]) && std::isfinite(v[2]); }

struct HostScene {
    std::vector<DObj> objs;
    std::vector<DTri> tris;
    std::vector<DTriN> trins;
    std::vector<DLeaf> leaves;
    std::vector<int32_t> tri_orig;
    std::vector<DMat> mats;
    std::vector<DLight> lights;
    bool has_mesh = false, has_secondary = false;
    int32_t n_objs = 0, n_lights = 0;
    int32_t n_plane = 0, n_sphere = 0, n_box = 0, n_mesh = 0;
    int32_t pow_bits = 0;
    float ambient[4] = {0, 0, 0, 0};
};

int convert_scene(const rtx_scene_desc* desc, HostScene& H) {
    if (!desc) return fail(RTX_ERR_INVALID, "rtx_scene_create: null argument");
    if (desc->n_objects < 0 || desc->n_materials < 0 || desc->n_lights < 0 || desc->n_triangles < 0)
        return fail(RTX_ERR_INVALID, "rtx_scene_create: negative count");
    if ((desc->n_objects && !desc->objects) || (desc->n_materials && !desc->materials) ||
        (desc->n_lights && !desc->lights) || (desc->n_triangles && !desc->triangles))
        return fail(RTX_ERR_INVALID, "rtx_scene_create: null array with non-zero count");
    H.objs.assign(desc->n_objects, DObj{});
    H.tris.assign(desc->n_triangles, DTri{});
    H.trins.assign(desc->n_triangles, DTriN{});
    H.mats.assign(desc->n_materials, DMat{});
    H.lights.assign(desc->n_lights, DLight{});

    for (int i = 0; i < desc->n_materials; ++i) {
        const rtx_material& m = desc->materials[i];
        DMat& d = H.mats[i];
        std::memset(&d, 0, sizeof(d));
        set3(d.diffuse, m.diffuse);
        set3(d.specular, m.specular);
        d.type = m.type;
        if (m.type < RTX_MAT_DIFFUSE || m.type > RTX_MAT_REFRACTIVE)
            return fail(RTX_ERR_INVALID, "material " + std::to_string(i) + ": bad type");
        if (m.type != RTX_MAT_DIFFUSE) H.has_secondary = true;
        d.tint = (float)m.tint;                  // colour * mat.tint
        d.omt = (float)(1.0 - m.tint);           // reflection * (1 - mat.tint), fp64 then fp32
        d.eta_in = (float)m.refr_index;          // eta = refr_index (in_shape)
        d.eta_out = (float)(1.0 / m.refr_index); // eta = 1.0 / refr_index
        d.hardness = m.hardness;
        d.hard_is_int = (m.hardness >= 0.0 && m.hardness <= 4096.0 && std::floor(m.hardness) == m.hardness) ? 1 : 0;
        d.hard_int = d.hard_is_int ? (int32_t)m.hardness : 0;
        // specular lobe provably zero: +0 specular (so +0 * pow(...) = +0 for the finite,
        // non-negative pow) and +0-or-positive diffuse (so lambert >= +0 and lambert + 0 == lambert)
        auto pos_zero = [](float v) { return v == 0.0f && !std::signbit(v); };
        auto nonneg = [](float v) { return v > 0.0f || (v == 0.0f && !std::signbit(v)); };
        d.spec_zero = pos_zero(m.specular[0]) && pos_zero(m.specular[1]) && pos_zero(m.specular[2]) &&
                      nonneg(m.diffuse[0]) && nonneg(m.diffuse[1]) && nonneg(m.diffuse[2]) &&
                      m.hardness >= 0.0 && m.hardness <= 1e6;  // pow(base <= 1 + eps, h) stays finite
        for (int b = 0; b < 31; ++b)
            if ((d.hard_int >> b) && H.pow_bits < b + 1) H.pow_bits = b + 1;
    }
    for (int i = 0; i < desc->n_lights; ++i) {
        const rtx_light& l = desc->lights[i];
        DLight& d = H.lights[i];
        std::memset(&d, 0, sizeof(d));
        if (l.type != RTX_LIGHT_POINT && l.type != RTX_LIGHT_DIRECTIONAL)
            return fail(RTX_ERR_INVALID, "light " + std::to_string(i) + ": bad type");
        d.type = l.type;
        set3(d.vec, l.vector);
        f3 nv = neg(ld3(l.vector));
        set3(d.negvec, nv);
        set3(d.ndir, normalize(nv));
        set3(d.cp, scale(ld3(l.colour), (float)l.power));  // light.colour * light.power
    }
    for (int i = 0; i < desc->n_triangles; ++i) {
        const rtx_triangle& t = desc->triangles[i];
        DTri& d = H.tris[i];
        f3 v0 = ld3(t.v0), v1 = ld3(t.v1), v2 = ld3(t.v2);
        for (int k = 0; k < 3; ++k) { d.v0[k] = t.v0[k]; d.v1[k] = t.v1[k]; d.v2[k] = t.v2[k]; }
        f3 e01 = sub(v1, v0), e12 = sub(v2, v1), e20 = sub(v0, v2);
        f3 nu = cross(sub(v1, v0), sub(v2, v0));  // mesh.py:84-86 / :130-134
        f3 n = normalize(nu);
        const f3 src[4] = {e01, e12, e20, n};
        float* dst[4] = {d.e01, d.e12, d.e20, d.n};
        for (int q = 0; q < 4; ++q) { dst[q][0] = src[q].x; dst[q][1] = src[q].y; dst[q][2] = src[q].z; }
        d.nu[0] = nu.x; d.nu[1] = nu.y; d.nu[2] = nu.z;
        set3(H.trins[i].n0, t.n0);
        set3(H.trins[i].n1, t.n1);
        set3(H.trins[i].n2, t.n2);
    }
    for (int i = 0; i < desc->n_objects; ++i) {
        const rtx_object& o = desc->objects[i];
        DObj& d = H.objs[i];
        std::memset(&d, 0, sizeof(d));
        const std::string tag = "object " + std::to_string(i) + ": ";
        d.type = o.type;
        d.nmat = o.n_mats;
        if (o.n_mats < 1) return fail(RTX_ERR_INVALID, tag + "no material (the reference raises IndexError)");
        for (int k = 0; k < (o.n_mats < 2 ? o.n_mats : 2); ++k)
            if (o.mat[k] < 0 || o.mat[k] >= desc->n_materials) return fail(RTX_ERR_INVALID, tag + "material index out of range");
        d.mat0 = o.mat[0];
        d.mat1 = o.n_mats >= 2 ? o.mat[1] : o.mat[0];
        d.has_speed = o.has_speed ? 1 : 0;
        set3(d.speed, o.speed);
        set3(d.a, o.a);
        set3(d.b, o.b);
        switch (o.type) {
            case RTX_SPHERE:
                d.r2 = std::pow(o.radius, 2.0);  // self.radius ** 2
                break;
            case RTX_PLANE: {
                // Plane.__init__ axes (simple_geometry.py:93-103), exact vec3 compares
                f3 n = ld3(o.b);
                auto eq = [&](float x, float y, float z) { return n.x == x && n.y == y && n.z == z; };
                f3 wa;
                if (eq(0, 1, 0) || eq(0, -1, 0) || eq(0, 0, 1)) wa = mk(1, 0, 0);
                else if (eq(0, 0, -1)) wa = mk(-1, 0, 0);
                else if (eq(1, 0, 0)) wa = mk(0, 0, -1);
                else if (eq(-1, 0, 0)) wa = mk(0, 0, 1);
                else wa = normalize(cross(n, mk(0, 0, 1)));
                set3(d.c, wa);
                set3(d.e, normalize(cross(wa, n)));
                break;
            }
            case RTX_BOX:
                break;
            case RTX_MESH:
                if (o.tri_begin < 0 || o.tri_count < 0 || (int64_t)o.tri_begin + o.tri_count > desc->n_triangles)
                    return fail(RTX_ERR_INVALID, tag + "triangle range out of bounds");
                if (o.bv_type != RTX_BV_AABB && o.bv_type != RTX_BV_SPHERE)
                    return fail(RTX_ERR_INVALID, tag + "bad bounding volume type");
                H.has_mesh = true;
                d.tri_begin = o.tri_begin;
                d.tri_count = o.tri_count;
                d.bv_type = o.bv_type;
                d.flat = o.flat ? 1 : 0;
                set3(d.bv_a, o.bv_a);
                set3(d.bv_b, o.bv_b);
                d.bv_r2 = std::pow(o.bv_radius, 2.0);  // BoundingSphere: self.radius ** 2
                break;
            default:
                return fail(RTX_ERR_INVALID, tag + "bad type");
        }
    }
    // Group by type (planes, spheres, boxes, meshes), keeping scene order within a group;
    // `oid` remembers the scene-order position for closest-hit ties.
    std::vector<DObj> grouped;
    grouped.reserve(H.objs.size());
    const int32_t order[4] = {RTX_PLANE, RTX_SPHERE, RTX_BOX, RTX_MESH};
    int32_t counts[4] = {0, 0, 0, 0};
    for (int g = 0; g < 4; ++g)
        for (int i = 0; i < desc->n_objects; ++i)
            if (H.objs[i].type == order[g]) {
                DObj d = H.objs[i];
                d.oid = i;
                grouped.push_back(d);
                counts[g]++;
            }
    H.objs.swap(grouped);
    H.n_plane = counts[0]; H.n_sphere = counts[1]; H.n_box = counts[2]; H.n_mesh = counts[3];
    // Mesh face clusters: reorder each mesh's faces into spatially coherent leaves of <= 8
    // faces (median splits on face centroids) and record each face's OBJ order index.
    H.tri_orig.assign(desc->n_triangles, 0);
    for (DObj& d : H.objs) {
        if (d.type != RTX_MESH) continue;
        const int32_t b0 = d.tri_begin, n = d.tri_count;
        std::vector<int32_t> idx(n);
        for (int32_t i = 0; i < n; ++i) idx[i] = i;
        auto centroid = [&](int32_t i, int ax) {
            const DTri& t = H.tris[b0 + i];
            return (double)t.v0[ax] + (double)t.v1[ax] + (double)t.v2[ax];
        };
        const int32_t leaf0 = (int32_t)H.leaves.size();
        std::vector<std::pair<int32_t, int32_t>> stack{{0, n}};
        std::vector<std::pair<int32_t, int32_t>> ranges;
        while (!stack.empty()) {
            auto [a, e] = stack.back();
            stack.pop_back();
            if (e - a <= 8) { ranges.push_back({a, e}); continue; }
            double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
            for (int32_t k = a; k < e; ++k)
                for (int ax = 0; ax < 3; ++ax) {
                    const double c = centroid(idx[k], ax);
                    lo[ax] = std::min(lo[ax], c);
                    hi[ax] = std::max(hi[ax], c);
                }
            int ax = 0;
            for (int q = 1; q < 3; ++q)
                if (hi[q] - lo[q] > hi[ax] - lo[ax]) ax = q;
            const int32_t mid = (a + e) / 2;
            std::nth_element(idx.begin() + a, idx.begin() + mid, idx.begin() + e,
                             [&](int32_t x, int32_t y) { return centroid(x, ax) < centroid(y, ax); });
            stack.push_back({mid, e});
            stack.push_back({a, mid});
        }
        std::vector<DTri> tris(n);
        std::vector<DTriN> trins(n);
        float cmax = 0.0f;
        for (auto [a, e] : ranges) {
            DLeaf L;
            L.first = a;
            L.count = e - a;
            for (int ax = 0; ax < 3; ++ax) { L.lo[ax] = INFINITY; L.hi[ax] = -INFINITY; }
            for (int32_t k = a; k < e; ++k) {
                const DTri& t = H.tris[b0 + idx[k]];
                tris[k] = t;
                trins[k] = H.trins[b0 + idx[k]];
                H.tri_orig[b0 + k] = idx[k];
                for (const float* v : {t.v0, t.v1, t.v2})
                    for (int ax = 0; ax < 3; ++ax) {
                        L.lo[ax] = std::min(L.lo[ax], v[ax]);
                        L.hi[ax] = std::max(L.hi[ax], v[ax]);
                        cmax = std::max(cmax, std::fabs(v[ax]));
                    }
            }
            H.leaves.push_back(L);
        }
        std::copy(tris.begin(), tris.end(), H.tris.begin() + b0);
        std::copy(trins.begin(), trins.end(), H.trins.begin() + b0);
        d.leaf_begin = leaf0;
        d.leaf_count = (int32_t)H.leaves.size() - leaf0;
        d.cmax = cmax;
    }
    H.n_objs = desc->n_objects;
    H.n_lights = desc->n_lights;
    set3(H.ambient, desc->ambient);
    return RTX_OK;
}

// Validates the camera and fills the scalar part of KParams; table pointers are left for
// the caller (device uploads, or host arrays in the emulation build).
int convert_camera(const rtx_camera_desc* c, KParams& k) {
    if (!c) return fail(RTX_ERR_INVALID, "rtx_camera_set: null argument");
    if (c->width < 1 || c->height < 1 || c->ncols < 1 || c->col0 < 0 || (int64_t)c->col0 + c->ncols > c->width)
        return fail(RTX_ERR_INVALID, "rtx_camera_set: bad image/strip size");
    if (c->n_dof < 1 || c->n_aa < 1 || c->n_times < 1)
        return fail(RTX_ERR_INVALID, "rtx_camera_set: sample counts must be >= 1");
    if (!c->xs || !c->ys || !c->dof_origins || !c->aa_origins || !c->times)
        return fail(RTX_ERR_INVALID, "rtx_camera_set: null table");
    if (c->jitter < RTX_JITTER_OFF || c->jitter > RTX_JITTER_REPLAY)
        return fail(RTX_ERR_INVALID, "rtx_camera_set: bad jitter mode");
    if (c->jitter == RTX_JITTER_REPLAY && !c->noise)
        return fail(RTX_ERR_INVALID, "rtx_camera_set: replay jitter needs a noise table");
    if (!finite3(c->position) || !finite3(c->u) || !finite3(c->v) || !finite3(c->w))
        return fail(RTX_ERR_INVALID, "rtx_camera_set: non-finite camera basis");
    const int64_t nsamp = (int64_t)c->n_dof * c->n_aa;
    if (nsamp * c->n_times > ((int64_t)1 << 24)) return fail(RTX_ERR_INVALID, "rtx_camera_set: too many samples per pixel");
    std::memset(&k, 0, sizeof(k));
    set3(k.pos, c->position);
    set3(k.u, c->u);
    set3(k.v, c->v);
    set3(k.dw, scale(ld3(c->w), (float)c->d));  // self.vc.d * self.vc.w
    k.focal = (float)c->focal_length;
    k.divisor = (float)(nsamp * c->n_times);     // samples * dof_samples * len(motion_times)
    const int64_t nd = nsamp * c->n_times;
    k.div_pow2 = (nd & (nd - 1)) == 0 ? 1 : 0;
    k.inv_divisor = 1.0f / k.divisor;
    k.jscale = (float)c->jitter_scale;
    k.width = c->width; k.height = c->height; k.col0 = c->col0; k.ncols = c->ncols;
    k.n_dof = c->n_dof; k.n_aa = c->n_aa; k.n_times = c->n_times; k.jitter = c->jitter;
    k.seed_lo = (uint32_t)c->seed; k.seed_hi = (uint32_t)(c->seed >> 32);
    return RTX_OK;
}

}  // namespace

// ------------------------------------------------------------------ scene object
struct rtx_scene {
    int device = 0;
    SceneView view{};
    bool has_mesh = false, has_secondary = false;
    void* d_objs = nullptr;
    void* d_tris = nullptr;
    void* d_trins = nullptr;
    void* d_mats = nullptr;
    void* d_lights = nullptr;
    void* d_leaves = nullptr;
    void* d_tri_orig = nullptr;
    // camera
    bool cam_set = false;
    KParams kp{};
    float* d_xs = nullptr;
    float* d_ys = nullptr;
    float* d_dof = nullptr;
    float* d_aa = nullptr;
    float* d_times = nullptr;
    float* d_noise = nullptr;
    KParams* d_kp = nullptr;
};

namespace {

template <class T>
int upload(void** dptr, const std::vector<T>& v) {
    if (v.empty()) { *dptr = nullptr; return RTX_OK; }
    RTX_HIP(hipMalloc(dptr, sizeof(T) * v.size()));
    RTX_HIP(hipMemcpy(*dptr, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice));
    return RTX_OK;
}

void free_camera(rtx_scene* s) {
    for (float* p : {s->d_xs, s->d_ys, s->d_dof, s->d_aa, s->d_times, s->d_noise}) (void)hipFree(p);
    (void)hipFree(s->d_kp);
    s->d_xs = s->d_ys = s->d_dof = s->d_aa = s->d_times = s->d_noise = nullptr;
    s->d_kp = nullptr;
    s->cam_set = false;
}

void free_scene(rtx_scene* s) {
    free_camera(s);
    for (void* p : {s->d_objs, s->d_tris, s->d_trins, s->d_mats, s->d_lights, s->d_leaves, s->d_tri_orig})
        (void)hipFree(p);
    delete s;
}

}  // namespace

extern "C" {

int rtx_abi_version(void) { return RTX_ABI_VERSION; }

const char* rtx_last_error(void) { return g_last_error.c_str(); }

int rtx_scene_create(const rtx_scene_desc* desc, rtx_scene** out) {
    if (!out) return fail(RTX_ERR_INVALID, "rtx_scene_create: null argument");
    *out = nullptr;
    HostScene H;
    int rc = convert_scene(desc, H);
    if (rc) return rc;
    rtx_scene* s = new rtx_scene();
    if (hipGetDevice(&s->device) != hipSuccess) { delete s; return fail(RTX_ERR_HIP, "hipGetDevice failed"); }
    if ((rc = upload(&s->d_objs, H.objs)) || (rc = upload(&s->d_tris, H.tris)) || (rc = upload(&s->d_trins, H.trins)) ||
        (rc = upload(&s->d_mats, H.mats)) || (rc = upload(&s->d_lights, H.lights)) ||
        (rc = upload(&s->d_leaves, H.leaves)) || (rc = upload(&s->d_tri_orig, H.tri_orig))) {
        free_scene(s);
        return rc;
    }
    s->has_mesh = H.has_mesh;
    s->has_secondary = H.has_secondary;
    SceneView& v = s->view;
    v.objs = (cptr<DObj>)s->d_objs;
    v.tris = (cptr<DTri>)s->d_tris;
    v.trins = (cptr<DTriN>)s->d_trins;
    v.mats = (cptr<DMat>)s->d_mats;
    v.lights = (cptr<DLight>)s->d_lights;
    v.leaves = (cptr<DLeaf>)s->d_leaves;
    v.tri_orig = (cptr<int32_t>)s->d_tri_orig;
    v.n_objs = H.n_objs;
    v.n_lights = H.n_lights;
    v.n_plane = H.n_plane; v.n_sphere = H.n_sphere; v.n_box = H.n_box; v.n_mesh = H.n_mesh;
    v.pow_bits = H.pow_bits;
    std::memcpy(v.ambient, H.ambient, sizeof(v.ambient));
    *out = s;
    return RTX_OK;
}

int rtx_scene_destroy(rtx_scene* s) {
    if (!s) return fail(RTX_ERR_INVALID, "rtx_scene_destroy: null scene");
    free_scene(s);
    return RTX_OK;
}

int rtx_camera_set(rtx_scene* s, const rtx_camera_desc* c) {
    if (!s) return fail(RTX_ERR_INVALID, "rtx_camera_set: null scene");
    KParams k;
    int rc = convert_camera(c, k);
    if (rc) return rc;
    free_camera(s);
    const size_t nsamp = (size_t)c->n_dof * c->n_aa;
    std::vector<float> times(c->n_times);
    for (int i = 0; i < c->n_times; ++i) times[i] = (float)c->times[i];  // current_time * speed casts to fp32
    auto up = [&](float** d, const float* h, size_t n) -> int {
        RTX_HIP(hipMalloc((void**)d, sizeof(float) * n));
        RTX_HIP(hipMemcpy(*d, h, sizeof(float) * n, hipMemcpyHostToDevice));
        return RTX_OK;
    };
    if ((rc = up(&s->d_xs, c->xs, c->ncols)) || (rc = up(&s->d_ys, c->ys, c->height)) ||
        (rc = up(&s->d_dof, c->dof_origins, 3 * (size_t)c->n_dof)) || (rc = up(&s->d_aa, c->aa_origins, 3 * nsamp)) ||
        (rc = up(&s->d_times, times.data(), times.size())))
        return rc;
    if (c->jitter == RTX_JITTER_REPLAY && (rc = up(&s->d_noise, c->noise, 3 * (size_t)c->ncols * c->height * nsamp)))
        return rc;
    k.S = s->view;
    k.xs = (cptr<float>)s->d_xs; k.ys = (cptr<float>)s->d_ys; k.dof_o = (cptr<float>)s->d_dof;
    k.aa_o = (cptr<float>)s->d_aa; k.times = (cptr<float>)s->d_times; k.noise = (cptr<float>)s->d_noise;
    RTX_HIP(hipMalloc((void**)&s->d_kp, sizeof(KParams)));
    RTX_HIP(hipMemcpy(s->d_kp, &k, sizeof(KParams), hipMemcpyHostToDevice));
    s->kp = k;
    s->cam_set = true;
    return RTX_OK;
}

int rtx_render(rtx_scene* s, int32_t row0, int32_t nrows, float* fb_dev, uint64_t* counters_dev, void* stream) {
    if (!s) return fail(RTX_ERR_INVALID, "rtx_render: null scene");
    if (!s->cam_set) return fail(RTX_ERR_STATE, "rtx_render: rtx_camera_set was not called");
    if (row0 < 0 || nrows < 0 || (int64_t)row0 + nrows > s->kp.height)
        return fail(RTX_ERR_INVALID, "rtx_render: row range outside the image");
    if (nrows == 0) return RTX_OK;
    if (!fb_dev) return fail(RTX_ERR_INVALID, "rtx_render: null framebuffer");
    Launch L;
    L.fb = fb_dev;
    L.row0 = row0;
    L.nrows = nrows;
    L.counters = reinterpret_cast<unsigned long long*>(counters_dev);
    const int64_t items = launch_items(nrows, s->kp.ncols);
    const dim3 grid((unsigned)((items + 255) / 256)), block(256);
    hipStream_t st = (hipStream_t)stream;
    const bool cnt = counters_dev != nullptr;
    const bool jit = s->kp.jitter != RTX_JITTER_OFF;
    const int sel = (s->has_mesh ? 8 : 0) | (s->has_secondary ? 4 : 0) | (cnt ? 2 : 0) | (jit ? 1 : 0);
    const KParams* kp = s->d_kp;
#define RTX_LAUNCH(M, S, C, J) \
    hipLaunchKernelGGL((k_render<M, S, C, J>), grid, block, 0, st, kp, L)
    switch (sel) {
        case 0: RTX_LAUNCH(false, false, false, false); break;
        case 1: RTX_LAUNCH(false, false, false, true); break;
        case 2: RTX_LAUNCH(false, false, true, false); break;
        case 3: RTX_LAUNCH(false, false, true, true); break;
        case 4: RTX_LAUNCH(false, true, false, false); break;
        case 5: RTX_LAUNCH(false, true, false, true); break;
        case 6: RTX_LAUNCH(false, true, true, false); break;
        case 7: RTX_LAUNCH(false, true, true, true); break;
        case 8: RTX_LAUNCH(true, false, false, false); break;
        case 9: RTX_LAUNCH(true, false, false, true); break;
        case 10: RTX_LAUNCH(true, false, true, false); break;
        case 11: RTX_LAUNCH(true, false, true, true); break;
        case 12: RTX_LAUNCH(true, true, false, false); break;
        case 13: RTX_LAUNCH(true, true, false, true); break;
        case 14: RTX_LAUNCH(true, true, true, false); break;
        case 15: RTX_LAUNCH(true, true, true, true); break;
    }
#undef RTX_LAUNCH
    RTX_HIP(hipGetLastError());
    return RTX_OK;
}

int rtx_intersect(rtx_scene* s, int64_t n, const float* ro, const float* rd, double time, double* t_dev,
                  int32_t* obj_dev, int32_t* mat_dev, float* normal_dev, float* position_dev, void* stream) {
    if (!s || n < 0 || (n > 0 && (!ro || !rd))) return fail(RTX_ERR_INVALID, "rtx_intersect: bad argument");
    if (n == 0) return RTX_OK;
    const dim3 grid((unsigned)((n + 255) / 256)), block(256);
    if (s->has_mesh)
        hipLaunchKernelGGL(k_intersect<true>, grid, block, 0, (hipStream_t)stream, s->view, n, ro, rd, (float)time,
                           t_dev, obj_dev, mat_dev, normal_dev, position_dev);
    else
        hipLaunchKernelGGL(k_intersect<false>, grid, block, 0, (hipStream_t)stream, s->view, n, ro, rd, (float)time,
                           t_dev, obj_dev, mat_dev, normal_dev, position_dev);
    RTX_HIP(hipGetLastError());
    return RTX_OK;
}

int rtx_occluded(rtx_scene* s, int64_t n, const float* ro, const float* rd, const double* tmax, double time,
                 uint8_t* occ, void* stream) {
    if (!s || n < 0 || (n > 0 && (!ro || !rd || !tmax || !occ))) return fail(RTX_ERR_INVALID, "rtx_occluded: bad argument");
    if (n == 0) return RTX_OK;
    const dim3 grid((unsigned)((n + 255) / 256)), block(256);
    if (s->has_mesh)
        hipLaunchKernelGGL(k_occluded<true>, grid, block, 0, (hipStream_t)stream, s->view, n, ro, rd, tmax, (float)time, occ);
    else
        hipLaunchKernelGGL(k_occluded<false>, grid, block, 0, (hipStream_t)stream, s->view, n, ro, rd, tmax, (float)time, occ);
    RTX_HIP(hipGetLastError());
    return RTX_OK;
}

int rtx_fb_to_rgb8(const float* fb, uint8_t* out, int64_t n, void* stream) {
    if (n < 0 || (n > 0 && (!fb || !out))) return fail(RTX_ERR_INVALID, "rtx_fb_to_rgb8: bad argument");
    if (n == 0) return RTX_OK;
    hipLaunchKernelGGL(k_to_rgb8, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, fb, out, n);
    RTX_HIP(hipGetLastError());
    return RTX_OK;
}

}  // extern "C"
