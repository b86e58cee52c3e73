// rtx_trace.h — per-ray math of the MI355X render path (device code; also compiled for
// the host in the tests-only emulation build, tests/native/).
//
// Numerics contract: PyGLM vec3 arithmetic is IEEE fp32, Python
// scalars are fp64. Every expression below keeps the reference's operation order and
// is compiled with -ffp-contract=off, so no multiply-add is fused. Citations are to
// SpacewaIker/python-raytracer @ 2025-02-14.
#pragma once

#if !defined(__HIPCC_RTC__)  // hiprtc (scene-specialized kernels) brings its own runtime header
#include <hip/hip_runtime.h>
#include <stdint.h>
#else
using __hip_internal::int32_t;
using __hip_internal::int64_t;
using __hip_internal::uint8_t;
using __hip_internal::uint16_t;
using __hip_internal::uint32_t;
using __hip_internal::uint64_t;
#ifndef INFINITY
#define INFINITY __builtin_inff()
#endif
#endif

#define RTX_HD __host__ __device__ __forceinline__

#include "rtx_fastmath.h"

// Read-only scene and camera tables are addressed as the AMDGPU constant address space in
// device code: wave-uniform reads of them become scalar (s_load) reads through the
// constant cache. The host-emulation build (tests only) sees plain pointers.
#if defined(__HIP_DEVICE_COMPILE__)
#define RTX_CONST __attribute__((address_space(4)))
#else
#define RTX_CONST
#endif

namespace rtx {

constexpr int kMaxDepth = 10;  // cast_ray(max_recursion=10) (scene.py:81)
// (a library build knob, forwarded to the hiprtc kernels): chunks of 16 faces measured
// 3-4 % faster than 32 on the 81,920-face mesh (0.1560 -> 0.1498 ms, three rounds on one
// box, profiles/r06/s8/), 64 slower (0.173 ms, profiles/r06/s6/)
#ifndef RTX_HEAVY_CHUNK
#define RTX_HEAVY_CHUNK 16
#endif
constexpr int kHeavyChunk = RTX_HEAVY_CHUNK;  // faces per chunk of a heavy tile's primary-ray list (SceneView::bin_heavy)

// Cost probes (tools/ablate.sh, tools/ab_jitflags.sh): a tools build of the library
// (-DRTX_TOOLS_BUILD, tools/build_lib_variant.sh) compiles kernels with -DRTX_ABLATE=n that
// drop or fake one part of the work so that part can be timed. librtx.so is not a tools
// build: RTX_PROBE(n) is false in it and in every kernel it compiles at run time (its
// hiprtc sources undefine RTX_TOOLS_BUILD), whatever flags they are given.
#ifndef RTX_ABLATE
#define RTX_ABLATE 0
#endif
#if defined(RTX_TOOLS_BUILD)
#define RTX_PROBE(n) (RTX_ABLATE == (n))
#define RTX_PROBE_ON RTX_ABLATE
#else
#define RTX_PROBE(n) false
#define RTX_PROBE_ON 0
#endif

// ------------------------------------------------------------------ fp32 vec3 (PyGLM)
struct f3 {
    float x, y, z;
};
RTX_HD f3 mk(float x, float y, float z) { return f3{x, y, z}; }
RTX_HD f3 ld3(const float* p) { return f3{p[0], p[1], p[2]}; }
#if defined(__HIP_DEVICE_COMPILE__)
RTX_HD f3 ld3(const float RTX_CONST* p) { return f3{p[0], p[1], p[2]}; }
#endif
RTX_HD f3 add(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
RTX_HD f3 sub(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
RTX_HD f3 mul(f3 a, f3 b) { return f3{a.x * b.x, a.y * b.y, a.z * b.z}; }
RTX_HD f3 scale(f3 a, float s) { return f3{a.x * s, a.y * s, a.z * s}; }
RTX_HD f3 divs(f3 a, float s) { return f3{a.x / s, a.y / s, a.z / s}; }
RTX_HD f3 neg(f3 a) { return f3{-a.x, -a.y, -a.z}; }
// glm::dot: tmp = a * b; tmp.x + tmp.y + tmp.z (left to right)
RTX_HD float dot(f3 a, f3 b) {
    float px = a.x * b.x, py = a.y * b.y, pz = a.z * b.z;
    float s = px + py;
    return s + pz;
}
RTX_HD f3 cross(f3 a, f3 b) {
    return f3{a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y};
}
// Wave votes as one ballot of the predicate's lane mask (no bool -> int -> compare round
// trip through a VGPR): true if the predicate holds in ANY / ALL active lanes; the host
// emulation runs a single lane.
#if defined(__HIP_DEVICE_COMPILE__)
#define RTX_ANY(p) (__builtin_amdgcn_ballot_w64((bool)(p)) != 0)
#define RTX_ALL(p) (__builtin_amdgcn_ballot_w64((bool)(p)) == __builtin_amdgcn_ballot_w64(true))
#else
#define RTX_ANY(p) ((bool)(p))
#define RTX_ALL(p) ((bool)(p))
#endif

// Marks the start of a rarely taken wave-uniform branch: an asm statement cannot be
// speculated, so the compiler keeps the block behind the branch instead of computing it
// in every wave and selecting (if-conversion of the IEEE normalize fallback and of the
// spheres' second roots cost TwoSpheresPlane 4 %, DepthOfField 3 %).
#ifndef RTX_NORM_BRANCH
#define RTX_NORM_BRANCH 1
#endif
RTX_HD void unspeculated() {
#if defined(__HIP_DEVICE_COMPILE__)
    if (RTX_NORM_BRANCH) asm volatile("");
#endif
}

// glm::normalize = v * inversesqrt(dot(v, v)), inversesqrt(x) = 1 / sqrt(x)
RTX_HD f3 normalize(f3 v) {
    const float q = dot(v, v);
#if RTX_PROBE_ON == 6 && defined(__HIP_DEVICE_COMPILE__)
    float inv = __builtin_amdgcn_rsqf(q);  // cost probe only
#else
#if defined(__HIP_DEVICE_COMPILE__)
    // the same IEEE results from the hardware approximations (rtx_fastmath.h) when every
    // active lane's dot is in range -- the common case; the compiler's sequence otherwise
    const bool fast = q >= fm::kLo && q < fm::kHi;  // false for NaN
    if (RTX_ALL(fast)) return scale(v, fm::rcp_rn(fm::sqrt_rn(q)));
    unspeculated();
#endif
    float inv = 1.0f / sqrtf(q);
#endif
    return scale(v, inv);
}
RTX_HD bool is_zero(f3 v) { return v.x == 0.0f && v.y == 0.0f && v.z == 0.0f; }
// glm::reflect(I, N) = I - N * dot(N, I) * 2
RTX_HD f3 reflect(f3 I, f3 N) { return sub(I, scale(scale(N, dot(N, I)), 2.0f)); }
// glm::refract(I, N, eta), T = float
RTX_HD f3 refract(f3 I, f3 N, float eta) {
    float d = dot(N, I);
    float k = 1.0f - eta * eta * (1.0f - d * d);
    if (!(k >= 0.0f)) return f3{0.0f, 0.0f, 0.0f};
    float s = eta * d + sqrtf(k);
    return sub(scale(I, eta), scale(N, s));
}
// Python max(0.0, x) and the clamp max(0.0, min(1.0, x)) of scene.py:113-115
RTX_HD float pos_part(float x) { return x > 0.0f ? x : 0.0f; }
RTX_HD float clamp01(float x) {
    float m = x < 1.0f ? x : 1.0f;
    return m > 0.0f ? m : 0.0f;
}
RTX_HD f3 clamp01(f3 c) { return f3{clamp01(c.x), clamp01(c.y), clamp01(c.z)}; }

// ------------------------------------------------------------------ device scene records
// Library-internal layouts (not ABI). Derived values are computed once on the host by
// rtx_api.hip with the same fp32 operation order as the reference computes them per ray.
// Objects are stored grouped by type (planes, spheres, boxes, meshes); `oid` is the
// object's position in the scene list, which decides closest-hit ties.
struct alignas(16) DObj {
    int32_t type, nmat, mat0, mat1;
    int32_t has_speed, tri_begin, tri_count, bv_type;
    int32_t flat, oid, leaf_begin, leaf_count;   // mesh: BVH nodes (DLeaf range, preorder)
    float cmax;                                  // mesh: max |vertex coordinate|
    int32_t face_cull;                           // mesh: test each face's box before its exact test
    float r2f;                                   // sphere: (float)(radius ** 2), the fp32 filters' input
    int32_t pad5;
    float a[4];       // sphere centre | plane point | box minpos
    float b[4];       // plane normal | box maxpos
    float c[4];       // plane width axis
    float e[4];       // plane height axis
    float speed[4];
    float bv_a[4];    // mesh BV AABB min | sphere centre
    float bv_b[4];    // mesh BV AABB max
    double r2;        // sphere radius ** 2
    double bv_r2;     // mesh BV sphere radius ** 2
    double radius;    // sphere radius (is_inside, simple_geometry.py:80)
    double tex_scale; // plane texture_scale (scene_parser.py:226)
    int32_t has_tex, tex_off, tex_w, tex_h;   // texture: texels [tex_off, + w * h), RGBA8
};

struct alignas(16) DTri {
    float v0[3], v1[3], v2[3];
    float e01[3], e12[3], e20[3];  // v1 - v0, v2 - v1, v0 - v2 (mesh.py:99-101)
    float n[3];                    // normalize(cross(v1 - v0, v2 - v0)) (mesh.py:86)
    float nu[3];                   // cross(v1 - v0, v2 - v0) (mesh.py:134)
};

// A face's bounds, for the conservative per-face skip of small meshes (DObj::face_cull).
struct alignas(16) DFaceBox {
    float lo[3], pad0;
    float hi[3], pad1;
};

struct alignas(16) DTriN {
    float n0[4], n1[4], n2[4];     // smooth vertex normals (mesh.py:53-70)
};

// A mesh BVH node in preorder: the bounds of the vertices of its faces; a leaf holds a
// cluster of <= 8 spatially sorted faces (count > 0), an internal node's children follow
// it. Used only to skip faces conservatively (see leaf_maybe_hit); faces keep their
// original index for tie breaks (tri_orig).
struct alignas(16) DLeaf {
    float lo[3];
    int32_t first;                 // leaf: into the mesh's (cluster-ordered) faces
    float hi[3];
    int32_t count;                 // 0: internal node
    int32_t skip, pad0, pad1, pad2;  // the node after this subtree (relative to the mesh's first)
};

struct alignas(16) DMat {
    float diffuse[4];
    float specular[4];
    float tint, omt;               // f32(tint), f32(1 - tint)       (scene.py:104,108)
    float eta_in, eta_out;         // f32(refr_index), f32(1 / refr_index) (scene.py:191,194)
    int32_t type, hard_int, hard_is_int, spec_zero;
    double hardness;
};

struct alignas(16) DLight {
    int32_t type, pad0, pad1, pad2;
    float vec[4];                  // light.vector
    float negvec[4];               // -light.vector
    float ndir[4];                 // normalize(-light.vector) (directional, scene.py:173)
    float cp[4];                   // light.colour * f32(light.power) (scene.py:183)
};

enum : int32_t { OBJ_SPHERE = 0, OBJ_PLANE = 1, OBJ_BOX = 2, OBJ_MESH = 3 };
enum : int32_t { MAT_DIFFUSE = 0, MAT_MIRROR = 1, MAT_REFRACTIVE = 2 };
enum : int32_t { LIGHT_POINT = 0, LIGHT_DIRECTIONAL = 1 };
enum : int32_t { BV_AABB = 0, BV_SPHERE = 1 };

// Hierarchy nodes (hierarchy.py:11-146), flattened in preorder: the subtree of node i is
// [i, end), a node's children follow it in child order. Leaves point at a DObj.
enum : int32_t { HN_UNION = 0, HN_INTER = 1, HN_DIFF = 2, HN_OTHER = 3, HN_LEAF = 4 };
struct alignas(16) DNode {
    int32_t kind, parent, cidx, depth;  // depth 0 = a top-level object
    int32_t end, pkind, obj, mat0;      // pkind: parent's kind; obj: leaf DObj; mat0: materials[0] or -1
    int32_t oid, pad0, pad1, pad2;      // oid: the root's position in Scene.objects
    float M[16];                        // glm mat4, [column][row]
    float Minv[16];
};
constexpr int kMaxHLevels = 16;  // hierarchy depth limit (levels of the ray/point stacks)

// On the device a node is split by use, so the traversal's scalar working set stays small
// (the scalar data cache is 16 KB): the fields every step reads (48 B), and the matrices
// (128 B) read only when a ray or point descends into the node.
struct alignas(16) DNodeHot {
    int32_t kind, parent, cidx, depth;
    int32_t end, pkind, obj, mat0;
    int32_t oid, pad0, pad1, pad2;
};
struct alignas(16) DNodeMat {
    float M[16];
    float Minv[16];
};

// Conservative regions of a hierarchy subtree, in its parent's frame, for the frame's
// motion-time range (computed on the host, padded far beyond fp32 rounding): every
// intersect() hit of the subtree that also passes its parent's filter lies in h,
// is_inside() can only be true in i, and shadow_intersect() can only be true for a ray
// that meets s. Empty: lo > hi.
struct alignas(16) DBound {
    float hlo[4], hhi[4];
    float ilo[4], ihi[4];
    float slo[4], shi[4];
};
// On the device the three kinds of box live in three arrays (a traversal reads one kind).
struct alignas(16) DBox {
    float lo[4], hi[4];
};

// Light grid of a point light (rtx_api.hip light_grids): the directions from the light
// to the scene's one mesh form a cone (axis a, padded half angle with cos^2 = cos2); its
// gnomonic plane (x, y) = (w.u, w.v) / w.a, |x|, |y| <= tmax, is cut into G x G cells,
// and cell c lists every face whose padded footprint covers it. A shadow ray from p to
// the light (and beyond it: Mesh.shadow_intersect has no t_max) can only hit faces listed
// in the cell of w = p - L (the line's points all lie in the directions +-w from L).
// Within a cell, faces come by a lower bound of their distance from L along a: when the
// mesh is on p's side of the light (w.a > 0) only the part of the line between p and L
// meets it, so faces farther along a than |w| cannot occlude and the list stops there.
struct alignas(16) DLGrid {
    float L[3];
    int32_t G;           // cells per side; 0 = no grid for this light
    float a[3], cos2;
    float u[3], tmax;
    float v[3], scale;   // G / (2 tmax)
    float r2min, r2max;  // |w|^2 outside [r2min, r2max]: walk the BVH instead
    int32_t start_off, pad0;  // this light's G*G + 1 entries of lg_start
};

// Shadow grid of a directional light (rtx_api.hip dir_shadow_grids, per camera). The
// light's shadow rays are parallel, so the spheres, boxes and hierarchies one of them can
// meet follow from where its origin p projects on a plane across the light: cell
// (floor((p.e1 - u0) su), floor((p.e2 - v0) sv)) of G x G lists them (DSCell: obj bits =
// spheres 0-15, boxes 16-31; root bits = hierarchy roots 0-31 in order). `always`: what
// every ray tests (objects beyond the 16th of a kind, roots with unbounded shadow boxes);
// origins off the grid test only those, origins with max |p_i| > pmax test everything.
struct DSCell {
    uint32_t obj, root;
};
// One object's cell rectangle of a shadow grid (rtx_api.hip dir_shadow_grids; the device
// fills the cells from these, k_dsg_fill): cells [i0, i1] x [j0, j1] of the grid at `off`.
struct DSRect {
    int32_t off, i0, i1, j0, j1;
    uint32_t bit, root, pad;
};
struct alignas(16) DSGrid {
    float e1[3];
    int32_t G;  // cells per side; 0 = no grid for this light
    float e2[3];
    float pmax;
    float u0, v0, su, sv;
    int32_t off;  // this light's G * G cells in dsg_cells
    uint32_t always, always_root;
    // boxes (bits 16-31) whose own shadow test a camera ray's hit point on them may skip:
    // it cannot pass (rtx_api.hip dir_shadow_grids)
    uint32_t self_boxes;
};

template <class T>
using cptr = const T RTX_CONST*;
template <class T>
using cref = const T RTX_CONST&;  // a record read field by field where it is used

struct SceneView {
    cptr<DObj> objs;   // [planes | spheres | boxes | meshes]
    cptr<DTri> tris;
    cptr<DTriN> trins;
    cptr<DFaceBox> fboxes;           // per stored face (meshes with face_cull)
    cptr<DMat> mats;
    cptr<DLight> lights;
    cptr<DLeaf> leaves;
    cptr<int32_t> tri_orig;          // original face index (within its mesh) of each stored face
    int32_t n_objs, n_lights;
    int32_t n_plane, n_sphere, n_box, n_mesh;
    int32_t pow_bits, pad0, pad1, pad2;   // bit length of the largest integer hardness
    float ambient[4];
    cptr<DNodeHot> nodes;            // hierarchy nodes (roots: 0, nodes[0].end, ...)
    cptr<DNodeMat> nmat;             // their matrices
    cptr<uint32_t> texels;           // all textures, RGBA8 (A unused)
    cptr<float> lut255;              // fl32(k / 255) (simple_geometry.py:169)
    cptr<DBox> hbox, ibox, sbox;     // per node, for the current motion-time range (DBound)
    int32_t n_nodes, hlevels;        // hlevels: stack levels the hierarchies need
    int32_t n_tris, n_leaves;        // all triangles / mesh BVH nodes
    // Primary-ray face bins of the camera (rtx_api.hip primary_bins): for each 8x8 pixel
    // bin, the faces of the scene's one mesh that a primary ray of a tile whose top-left
    // pixel lies in the bin may hit (conservative). bins_on = 0: walk the BVH.
    cptr<int32_t> bin_start;         // [bins + 1]
    cptr<int32_t> bin_faces;         // stored face indices (within the mesh), nearest first
    cptr<float> bin_zmin;            // per entry: a lower bound of any hit t on that face
    cptr<uint32_t> bin_objmask;      // per bin: spheres (bits 0-15) and boxes (16-31) a ray may hit
    cptr<uint32_t> bin_rootmask;     // per bin: hierarchy roots (bit q: the q-th; later ones always)
    int32_t bins_x, bins_on, mesh_bins, pad5;
    // Heavy tiles (rtx_api.hip heavy_chunks): a bin whose face list is longer than
    // kHeavyChunk faces is tested in chunks of kHeavyChunk faces by a pass of its own
    // (k_mesh_chunks, one wave per chunk, before the render kernel of each frame), which
    // leaves per chunk and pixel of the tile the chunk's closest face; the render kernel
    // then offers those instead of walking the list. bin_heavy[b]: the bin's first chunk
    // (its chunks are consecutive), or -1. mesh_hits: [chunk][64 pixels of the 8x8 tile]
    // (t32 bits, stored face or -1). null: no heavy tiles.
    cptr<int32_t> bin_heavy;
    const uint2* mesh_hits;
    int32_t n_objs_all, n_mats, pad6, pad7;  // object records (incl. hierarchy leaves), materials
    // Light grids (per light; shadow rays of point lights against the scene's one mesh)
    cptr<DLGrid> lgrid;
    cptr<int32_t> lg_start;          // per light: [G * G + 1] offsets into lg_faces
    cptr<int32_t> lg_faces;          // stored face indices (within the mesh), by lg_d2
    cptr<float> lg_d2;               // per entry: (a lower bound of the face's distance along a)^2
    int32_t lgrid_on, pad8, pad9, pad10;
    // Shadow grids (per light; directional lights against the spheres and boxes)
    cptr<DSGrid> dsgrid;
    cptr<DSCell> dsg_cells;
    int32_t dsg_on, pad11, pad12, pad13;
    // Self tests of planes (per camera; rtx_api.hip plane_self_limits): [light][plane < 4]
    // the largest max |p_i| of a camera ray's hit point p on that plane whose own shadow
    // test toward the light cannot pass (-1: none); null: no skips
    cptr<float> plane_self;
};

// Mesh records read by the hot BVH walks (closest_hit / occluded). Scene-specialized
// kernels built with RTX_LDS_TRIS / RTX_LDS_LEAVES (the scene's triangle and BVH-node
// counts; rtx_api.hip, RTX_MESH_LDS=1) stage them in LDS once per block (render_body) and
// read them from there; everything else reads them through the constant cache.
#if defined(RTX_LDS_TRIS) && defined(__HIP_DEVICE_COMPILE__)
__shared__ DTri g_lds_tris[RTX_LDS_TRIS];
__shared__ DFaceBox g_lds_fboxes[RTX_LDS_TRIS];
__shared__ DLeaf g_lds_leaves[RTX_LDS_LEAVES];
#define RTX_TRI(S, i) (g_lds_tris[i])
#define RTX_FBOX(S, i) (g_lds_fboxes[i])
#define RTX_LEAF(S, i) (g_lds_leaves[i])
#else
#define RTX_TRI(S, i) ((S).tris[i])
#define RTX_FBOX(S, i) ((S).fboxes[i])
#define RTX_LEAF(S, i) ((S).leaves[i])
#endif

// A primary-ray tile's face list staged in LDS (RTX_BIN_LDS, scene-specialized mesh
// kernels; option bin_lds): kHeavyChunk faces at a time, their indices, depth bounds and
// records fetched by the wave's active lanes with coalesced 16-byte loads, then read from
// LDS by the closest-hit loop -- one round of memory latency per 32 faces instead of two
// or three dependent scalar loads per face. One slot per wave of the block.
#if defined(RTX_BIN_LDS) && RTX_BIN_LDS && defined(__HIP_DEVICE_COMPILE__)
struct BinLds {
    DTri tri[kHeavyChunk];
    DFaceBox box[kHeavyChunk];
    int32_t face[kHeavyChunk];
    float zmin[kHeavyChunk];
};
#ifdef RTX_BLOCK_FLAT
__shared__ BinLds g_bin_lds[RTX_BLOCK_FLAT / 64];
#else
__shared__ BinLds g_bin_lds[4];  // (256-thread blocks, rtx_kernels.h kBlock)
#endif
// rocPRIM's wave_barrier: LDS written by some lanes is read by others of the same wave
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
#endif

// Object and material records fetched with a per-lane index (the hit object of each lane,
// its material): scene-specialized kernels built with RTX_LDS_OBJS / RTX_LDS_MATS (the
// scene's record counts) copy both tables into LDS once per block (render_body), so these
// gathers are LDS reads instead of L2 round trips on the shading path. Loops over objects
// with a wave-uniform index keep their scalar loads.
#if defined(RTX_LDS_OBJS) && defined(__HIP_DEVICE_COMPILE__)
__shared__ DObj g_lds_objs[RTX_LDS_OBJS];
__shared__ DMat g_lds_mats[RTX_LDS_MATS];
#define RTX_OBJ(S, i) (g_lds_objs[i])
#define RTX_MAT(S, i) (g_lds_mats[i])
#else
#define RTX_OBJ(S, i) ((S).objs[i])
#define RTX_MAT(S, i) ((S).mats[i])
#endif

// ------------------------------------------------------------------ counters
struct Tally {
    uint32_t cast[kMaxDepth];
    uint32_t shadow, shade, tri;
};

template <bool COUNT>
RTX_HD void tally_inc(Tally& t, uint32_t Tally::*field) {
    if (COUNT) (t.*field)++;
}

// ------------------------------------------------------------------ geometry helpers
template <class O, class P>
RTX_HD f3 moved(const O& o, P p, float time) {
    // `p + self.speed * self.scene.current_time` (simple_geometry.py:21-24, :106-109, :189-194)
    f3 q = ld3(p);
#if defined(RTX_FIXED_STATIC) && RTX_FIXED_STATIC
    (void)o;
    (void)time;  // scene-specialized kernel of a scene without speeds
#else
    if (o.has_speed) q = add(q, scale(ld3(o.speed), time));
#endif
    return q;
}

// Ray.getPoint(t) = origin + direction * t, t cast to fp32 (helperclasses.py:21-22)
RTX_HD f3 get_point(f3 o, f3 d, double t) { return add(o, scale(d, (float)t)); }

// ------------------------------------------------------------------ materials, normals
// math.floor(a - b) of two floats, where the reference subtracts in fp64 (exactly). The
// fp32 difference d = fl32(a - b) lies in [k, k + 1] when floor(a - b) = k (k and k + 1
// are floats below 2^23), so floorf(d) is exact unless d is an integer: then use fp64.
RTX_HD int32_t floor_diff(float a, float b) {
    const float d = a - b;
    const float f = floorf(d);
    if (fabsf(d) < 0x1p23f && d != f) return (int32_t)f;
    unspeculated();
    return (int32_t)(int64_t)floor((double)a - (double)b);
}

// Plane.get_material (simple_geometry.py:133-148): checker by floor of the projected
// coordinates, Python modulo.
template <class O>
RTX_HD int32_t plane_material(const O& ob, f3 point, float time) {
    if (ob.nmat == 1) return ob.mat0;
    f3 position = moved(ob, ob.a, time);
    f3 n = ld3(ob.b);
    point = sub(point, scale(n, dot(sub(point, position), n)));
    float x = dot(sub(point, position), ld3(ob.c));
    float z = dot(sub(point, position), ld3(ob.e));
    const int32_t s = floor_diff(position.x, x) + floor_diff(position.z, z);
    return (s & 1) ? ob.mat1 : ob.mat0;  // (dx + dz) % 2 with Python modulo
}

// Barycentric smooth normal (mesh.py:103-113; igl.barycentric_coordinates_tri on fp32 rows).
template <class TT>
RTX_HD f3 smooth_normal(const TT& T, const DTriN& N, f3 p) {
    f3 a = ld3(T.v0), b = ld3(T.v1), c = ld3(T.v2);
    f3 v0 = sub(b, a), v1 = sub(c, a), v2 = sub(p, a);
    float d00 = dot(v0, v0), d01 = dot(v0, v1), d11 = dot(v1, v1);
    float d20 = dot(v2, v0), d21 = dot(v2, v1);
    float den = d00 * d11 - d01 * d01;
    float v = (d11 * d20 - d01 * d21) / den;
    float w = (d00 * d21 - d01 * d20) / den;
    float u = (1.0f - v) - w;
    f3 n = add(add(scale(ld3(N.n0), u), scale(ld3(N.n1), v)), scale(ld3(N.n2), w));
    return normalize(n);
}


// ------------------------------------------------------------------ exact fp32 proxies
// Every `t` the reference compares is an fp64 value t64. We carry t32 = fl32(t64):
//  * for plane/triangle hits t64 = fl64(num / den) of two floats, and fl32(fl64(q)) =
//    fl32(q) (double rounding is innocuous when 53 >= 2*24 + 2), so t32 is one IEEE fp32
//    division and getPoint(t64) = o + d * t32 exactly;
//  * fl32 is monotone and equal t64 give equal t32, so t32a < t32b implies t64a < t64b
//    and t32 > fl32(T) implies t64 > T. Only EQUAL proxies need the fp64 values.
// 1e-4 and 1e-3 are not floats: |x| > 1e-4 for a float x  <=>  |x| >= kEps4Up.
constexpr float kEps4Up = 0x1.a36e3p-14f;      // smallest float > 1e-4
constexpr float kEps4Near = 1e-4f;             // fl32(1e-4) (< 1e-4)
constexpr float kEps3Near = 1e-3f;             // fl32(1e-3)

// Wave-uniform predicates: RTX_ANY / RTX_ALL (defined with normalize above).

// A value every active lane holds, as a wave-uniform (scalar) value.
RTX_HD int32_t wave_uniform(int32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_readfirstlane(x);
#else
    return x;
#endif
}

// Closest-hit record: t as its fp32 proxy, the object (index into the type-grouped
// array, -1 = none) and a sub-index (sphere: root; box: entry slab label; mesh: face).
// The exact fp64 t is recomputed from (obj, sub) when two proxies tie.
struct Hit {
    float t32;
    int32_t obj;
    int32_t sub;
};

// t64 > T for t64 = fl64(num / den), with T32 = fl32(T).
RTX_HD bool quot_gt(float t32, float num, float den, double T, float T32) {
    if (t32 != T32) return t32 > T32;
    unspeculated();  // (the fp64 quotient only for lanes at the threshold's float)
    return (double)num / (double)den > T;
}
RTX_HD bool quot_lt(float t32, float num, float den, double T, float T32) {
    if (t32 != T32) return t32 < T32;
    unspeculated();
    return (double)num / (double)den < T;
}
// t64 >= 0 and t64 < 0 for t64 = fl64(num / den), den != 0, from t32 = fl32(num / den):
// a quotient that underflows to +-0 in fp32 keeps its sign in fp64; NaN compares false.
RTX_HD bool quot_signs_differ(float num, float den) { return num != 0.0f && ((num < 0.0f) != (den < 0.0f)); }
RTX_HD bool quot_nonneg(float t32, float num, float den) {
    return t32 > 0.0f || (t32 == 0.0f && !quot_signs_differ(num, den));
}
RTX_HD bool quot_neg(float t32, float num, float den) {
    return t32 < 0.0f || (t32 == 0.0f && quot_signs_differ(num, den));
}

// Sphere quadratic (simple_geometry.py:29-39); returns false when disc < 0.
// The same with oc = o - c and q = dot(oc, oc) given (shared by a shading point's lights).
RTX_HD bool sphere_roots_oc(f3 d, f3 oc, float q, double r2, double& b, double& s, double& two_a) {
    double a = (double)dot(d, d);
    b = 2.0 * (double)dot(d, oc);
    double cc = (double)q - r2;
    double disc = b * b - 4.0 * a * cc;
    if (disc < 0.0) return false;
    s = sqrt(disc);
    two_a = 2.0 * a;
    return true;
}
RTX_HD bool sphere_roots(f3 o, f3 d, f3 c, double r2, double& b, double& s, double& two_a) {
    if (RTX_PROBE(4)) {  // cost probe only: fp32 quadratic (not parity-correct)
        float a = dot(d, d);
        f3 oc = sub(o, c);
        float bf = 2.0f * dot(d, oc);
        float cf = dot(oc, oc) - (float)r2;
        float disc = bf * bf - 4.0f * a * cf;
        if (disc < 0.0f) return false;
        b = bf; s = sqrtf(disc); two_a = 2.0f * a;
        return true;
    }
    const f3 oc = sub(o, c);
    return sphere_roots_oc(d, oc, dot(oc, oc), r2, b, s, two_a);
}

// fp32 filter for the sign of the reference's fp64 discriminant (simple_geometry.py:29-34):
// returns -1 (certainly < 0), +1 (certainly > 0) or 0 (undecided: use sphere_roots).
// With h = dot(d, o - c) (b = 2h exactly), a = dot(d, d), q = dot(o - c, o - c), the
// quarter discriminant h^2 - a (q - r^2) is evaluated in fp32; its error is below
// 2^-21 (h^2 + a (q + r^2) + |D|), which also covers the reference's own fp64 rounding.
RTX_HD int sphere_disc_sign_oc(f3 d, f3 oc, float q, float r2f) {
    const float a = dot(d, d), h = dot(d, oc);
    const float hh = h * h;
    const float D = hh - a * (q - r2f);
    const float E = 0x1p-21f * (hh + a * (q + r2f) + fabsf(D));
    if (D < -E) return -1;
    if (D > E) return 1;
    return 0;  // also NaN/inf inputs: the exact path reproduces the reference
}
// Sphere.shadow_intersect's decision (simple_geometry.py:48-72: a root t with
// 1e-3 < t < t_max) in fp32 where error bounds allow: 1 hit, 0 no hit, -1 undecided (run
// the fp64 roots). With D within E of the exact discriminant H^2 - A C (the bound
// sphere_disc_sign_oc uses), s = sqrtf(D) is within E / s + 2^-22 s of sqrt(H^2 - A C),
// and the roots (-H -+ s) / A -- the reference's (-b -+ sqrt(disc)) / 2a with b = 2H --
// within m of the computed ones (every other rounding, and the reference's own fp64
// rounding, is below 2^-20 (|H| + s) / A). 1e-3 < t <=> t >= fl32(1e-3) for a float t.
#ifndef RTX_SHADOW_F32
#define RTX_SHADOW_F32 0  // measured slower (TSP 28.5 -> 30.4 us, DOF 7.23 -> 7.37 ms): off
#endif
// [tmax_dn, tmax_up]: the floats around t_max (equal when t_max is one, as 1.0 and inf are)
RTX_HD int sphere_shadow_f32(f3 d, f3 oc, float q, float r2f, float tmax_dn, float tmax_up) {
    const float a = dot(d, d), h = dot(d, oc);
    const float hh = h * h;
    const float D = hh - a * (q - r2f);
    const float E = 0x1p-21f * (hh + a * (q + r2f) + fabsf(D));
    if (D < -E) return 0;  // no real root
    if (!(D > E) || !(a > 0.0f)) return -1;
    const float s = sqrtf(D);
    const float inva = 1.0f / a;
    const float m = (E / s + 0x1p-21f * s) * inva + 0x1p-20f * ((fabsf(h) + s) * inva);
    auto decide = [&](float t) {
        const float lo = t - m, hi = t + m;
        if (lo >= kEps3Near && hi < tmax_dn) return 1;
        if (hi < kEps3Near || lo >= tmax_up) return 0;
        return -1;
    };
    const int h1 = decide((-h - s) * inva), h2 = decide((-h + s) * inva);
    if (h1 == 1 || h2 == 1) return 1;
    return h1 == 0 && h2 == 0 ? 0 : -1;
}
RTX_HD int sphere_disc_sign(f3 o, f3 d, f3 c, float r2f) {
    const f3 oc = sub(o, c);
    return sphere_disc_sign_oc(d, oc, dot(oc, oc), r2f);
}

// AABB slabs (simple_geometry.py:196-226; bounding_volumes.py:61-91). Returns false if
// a zero-direction slab rejects the ray; otherwise the entry start (max of starts, first
// wins), its label, and the exit end (min of ends, first wins), all fp64.
RTX_HD bool box_slabs(f3 o, f3 d, f3 mn, f3 mx, double& start, int& label, double& end) {
    const float ro[3] = {o.x, o.y, o.z};
    const float rd[3] = {d.x, d.y, d.z};
    const float lo[3] = {mn.x, mn.y, mn.z};
    const float hi[3] = {mx.x, mx.y, mx.z};
    double s_best = 0.0, e_best = 0.0;
    int l_best = 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        double s, e;
        if (rd[k] == 0.0f) {
            if (!((double)lo[k] < (double)ro[k] && (double)ro[k] < (double)hi[k])) return false;
            s = -INFINITY;
            e = INFINITY;
        } else {
            double t1 = ((double)lo[k] - (double)ro[k]) / (double)rd[k];
            double t2 = ((double)hi[k] - (double)ro[k]) / (double)rd[k];
            s = t2 < t1 ? t2 : t1;  // AAInterval: start = min(t1, t2)
            e = t2 > t1 ? t2 : t1;  //             end = max(t1, t2)
        }
        if (k == 0) {
            s_best = s; e_best = e; l_best = 0;
        } else {
            if (s > s_best) { s_best = s; l_best = k; }
            if (e < e_best) e_best = e;
        }
    }
    start = s_best;
    label = l_best;
    end = e_best;
    return true;
}

RTX_HD float rcp_approx(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rcpf(x);
#else
    return 1.0f / x;
#endif
}
// Per-ray reciprocals of the direction (v_rcp_f32), shared by the conservative box and
// cluster tests and the fp32 slab intervals.
struct RayInv {
    f3 inv;
    float pad_rel;
};
RTX_HD RayInv ray_inv(f3 o, f3 d) {
    auto safe = [](float v) { return fabsf(v) < 1e-30f ? copysignf(1e-30f, v) : v; };
    RayInv r;
    // v_rcp_f32 (1 ulp): its error moves a slab by <= 2^-23 |bound - o|, far inside the pad
    r.inv = f3{rcp_approx(safe(d.x)), rcp_approx(safe(d.y)), rcp_approx(safe(d.z))};
    r.pad_rel = fmaxf(fabsf(o.x), fmaxf(fabsf(o.y), fabsf(o.z)));
    return r;
}
// The fp64 slabs as the rare fallback of the fp32 decisions below, out of line: inlined,
// the compiler hoists their loop-invariant fp64 numerators (bound - origin) out of the
// shading loops, where they hold VGPRs for the whole kernel (TorusMesh: 40 B/lane of
// spills for its bounding volume's six numerators).
// (The result comes back by value, in registers: out-parameters of an out-of-line call
// would live in scratch, and every caller would store their initial values there on
// each visit -- 20 B/lane per box test, DepthOfField's extra HBM writes.)
struct SlabFar {
    double start, end;
    int label;
    bool valid;
};
__host__ __device__ __attribute__((noinline)) inline SlabFar box_slabs_far(f3 o, f3 d, f3 mn, f3 mx) {
    SlabFar r;
    r.valid = box_slabs(o, d, mn, mx, r.start, r.label, r.end);
    return r;
}

// The same slabs decided in fp32, with box_slabs as the fallback. Each reference quotient
// t = fl64((bound - o) / d) is estimated as q = fl32(bound - o) * rcp(d): three fp32
// roundings and v_rcp_f32's 1 ulp give |q - t| <= 2^-22 |q|, so q +- (2^-20 |q| + 2^-100)
// holds t. Start and end are then known to lie in [s_lo, s_hi] and [e_lo, e_hi], and the
// entry label is known when the first maximal start is separated from the other axes'.
// Slabs with 0 < |d| < 2^-20 or a quotient beyond 2^100 (or NaN) leave the lane undecided
// (so a flushed subnormal numerator, <= 2^-126 * 2^20, stays inside the 2^-100 term).
struct SlabIv {
    float s_lo, s_hi, e_lo, e_hi;
    int label;
    bool reject;  // certain: a d == 0 slab does not contain the origin (exact comparison)
    bool sure;    // the intervals and the label hold
};
// ri: the ray's reciprocals when the caller has them (the same v_rcp_f32 of every |d| >=
// 1e-30; smaller slabs are undecided anyway), else they are computed here.
RTX_HD SlabIv box_slabs_iv(f3 o, f3 d, f3 mn, f3 mx, const RayInv* ri = nullptr) {
    const float ro[3] = {o.x, o.y, o.z};
    const float rd[3] = {d.x, d.y, d.z};
    const float lo[3] = {mn.x, mn.y, mn.z};
    const float hi[3] = {mx.x, mx.y, mx.z};
    const float rr[3] = {ri ? ri->inv.x : 0.0f, ri ? ri->inv.y : 0.0f, ri ? ri->inv.z : 0.0f};
    float sc[3], ec[3], w[3];
    SlabIv r;
    r.reject = false;
    r.sure = true;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        if (rd[k] == 0.0f) {
            r.reject = r.reject || !(lo[k] < ro[k] && ro[k] < hi[k]);
            sc[k] = -INFINITY;
            ec[k] = INFINITY;
            w[k] = 0.0f;
        } else {
            const float rc = ri ? rr[k] : rcp_approx(rd[k]);
            const float q1 = (lo[k] - ro[k]) * rc, q2 = (hi[k] - ro[k]) * rc;
            sc[k] = fminf(q1, q2);
            ec[k] = fmaxf(q1, q2);
            const float m = fmaxf(fabsf(q1), fabsf(q2));
            w[k] = m * 0x1p-20f + 0x1p-100f;
            r.sure = r.sure && fabsf(rd[k]) >= 0x1p-20f && m < 0x1p100f;  // false for NaN
        }
    }
    int l = 0;  // max(..., key=start) keeps the first maximum
    if (sc[1] > sc[l]) l = 1;
    if (sc[2] > sc[l]) l = 2;
    r.label = l;
    r.s_lo = sc[l] - w[l];
    r.s_hi = sc[l] + w[l];
#pragma unroll
    for (int k = 0; k < 3; ++k)
        if (k != l) r.sure = r.sure && sc[k] + w[k] < r.s_lo;  // false if every d is 0
    r.e_lo = fminf(fminf(ec[0] - w[0], ec[1] - w[1]), ec[2] - w[2]);
    r.e_hi = fminf(fminf(ec[0] + w[0], ec[1] + w[1]), ec[2] + w[2]);
    return r;
}
// The reference's start for entry axis k: min(t1, t2) of that axis, i.e. the bound the
// ray meets first (fl64 division is monotone, so the exact order decides).
RTX_HD double slab_start64(f3 o, f3 d, f3 mn, f3 mx, int k) {
    const float ok = k == 0 ? o.x : (k == 1 ? o.y : o.z);
    const float dk = k == 0 ? d.x : (k == 1 ? d.y : d.z);
    const float lk = k == 0 ? mn.x : (k == 1 ? mn.y : mn.z);
    const float hk = k == 0 ? mx.x : (k == 1 ? mx.y : mx.z);
    const float b = ((hk > lk) == (dk > 0.0f)) ? lk : hk;
    return ((double)b - (double)ok) / (double)dk;
}
// Box entry as the closest-hit test needs it (simple_geometry.py:188-226: valid iff no
// zero-direction slab rejects, start <= end and start >= 0): fp32 decision, one fp64
// division for the entry t, the full fp64 slabs for undecided lanes.
RTX_HD bool box_entry_iv(f3 o, f3 d, f3 mn, f3 mx, const SlabIv& iv, bool live, double& start, int& label) {
    const bool yes = live && iv.sure && !iv.reject && iv.s_hi < iv.e_lo && iv.s_lo > 0.0f;
    const bool no = !live || iv.reject || (iv.sure && (iv.s_lo > iv.e_hi || iv.s_hi < 0.0f));
    label = iv.label;
    start = 0.0;
    if (yes) start = slab_start64(o, d, mn, mx, iv.label);
    bool valid = yes;
    const bool und = !yes && !no;
    if (RTX_ANY(und)) {
        if (und) {
            const SlabFar f = box_slabs_far(o, d, mn, mx);
            start = f.start;
            label = f.label;
            valid = f.valid && !(f.start > f.end || f.start < 0.0);
        }
    }
    return valid;
}
RTX_HD bool box_entry(f3 o, f3 d, f3 mn, f3 mx, bool live, double& start, int& label, const RayInv* ri = nullptr) {
    return box_entry_iv(o, d, mn, mx, box_slabs_iv(o, d, mn, mx, ri), live, start, label);
}
// From the fp32 intervals alone: the lane's ray certainly misses the box, or enters it
// only after tcap (its start cannot win or tie against a best hit whose fp32 proxy is
// tcap: start >= s_lo > tcap gives fl32(start) > tcap).
RTX_HD bool box_iv_out(const SlabIv& iv, float tcap) {
    return iv.reject || (iv.sure && (iv.s_lo > iv.e_hi || iv.s_hi < 0.0f || iv.s_lo > tcap));
}
// Experiment knob: 1 drops the padded pre-test and lets the slab intervals (which share
// its reciprocals and quotients) decide which lanes go on. Measured slower (DepthOfField 4K
// 7.06 -> 7.85 ms, profiles/r03/box_iv/): the cheap pre-test culls most lanes -- rays
// already ending on the floor in front of a box, tiles that miss it -- before any
// interval is needed.
#ifndef RTX_BOX_IV_CULL
#define RTX_BOX_IV_CULL 0
#endif
// Box shadow test (simple_geometry.py:251-294): 1e-4 < start < t_max and start <= end.
RTX_HD bool box_shadow_iv(f3 o, f3 d, f3 mn, f3 mx, const SlabIv& iv, double t_max) {
    const bool yes = iv.sure && !iv.reject && iv.s_hi < iv.e_lo && iv.s_lo >= kEps4Up && (double)iv.s_hi < t_max;
    const bool no = iv.reject ||
                    (iv.sure && (iv.s_lo > iv.e_hi || iv.s_hi < kEps4Up || (double)iv.s_lo >= t_max));
    bool occ = yes;
    const bool und = !yes && !no;
    if (RTX_ANY(und)) {
        if (und) {
            const SlabFar f = box_slabs_far(o, d, mn, mx);
            occ = f.valid && !(f.start > f.end) && 1e-4 < f.start && f.start < t_max;
        }
    }
    return occ;
}
RTX_HD bool box_shadow(f3 o, f3 d, f3 mn, f3 mx, double t_max, const RayInv* ri = nullptr) {
    return box_shadow_iv(o, d, mn, mx, box_slabs_iv(o, d, mn, mx, ri), t_max);
}

// Mesh bounding volume (bounding_volumes.py:18-37 sphere, :49-83 AABB).
template <class O>
RTX_HD bool mesh_bv(const O& ob, f3 o, f3 d) {
    if (ob.bv_type == BV_AABB) {
        // valid iff start <= end and start >= 0 (the fp64 slabs only for undecided lanes)
        const f3 mn = ld3(ob.bv_a), mx = ld3(ob.bv_b);
        const SlabIv iv = box_slabs_iv(o, d, mn, mx);
        const bool yes = iv.sure && !iv.reject && iv.s_hi < iv.e_lo && iv.s_lo > 0.0f;
        const bool no = iv.reject || (iv.sure && (iv.s_lo > iv.e_hi || iv.s_hi < 0.0f));
        if (yes || no) return yes;
        const SlabFar f = box_slabs_far(o, d, mn, mx);
        return f.valid && !(f.start > f.end || f.start < 0.0);
    }
    double b, s, two_a;
    if (!sphere_roots(o, d, ld3(ob.bv_a), ob.bv_r2, b, s, two_a)) return false;
    if ((-b - s) / two_a > 0.0) return true;
    return (-b + s) / two_a > 0.0;
}

// Conservative ray/cluster test. A face whose exact test passes has its computed point
// o + d*t32 inside the triangle up to fp32 rounding, i.e. within ~2^-22 (|o| + cmax) of
// the cluster box; the box is padded by 2^-16 (|o|_max + cmax) per ray, far above every
// rounding term, so a cluster is skipped only if none of its faces can pass.
// tcap: the ray's current best t (closest hit) -- a face beyond it cannot win; the
// padded box's entry precedes every face hit inside it.
template <class L_>
RTX_HD bool leaf_maybe_hit(const L_& L, f3 o, const RayInv& ri, float cmax, float tcap = INFINITY) {
    const float pad = 0x1p-16f * (ri.pad_rel + cmax);
    const float tx1 = (L.lo[0] - pad - o.x) * ri.inv.x, tx2 = (L.hi[0] + pad - o.x) * ri.inv.x;
    const float ty1 = (L.lo[1] - pad - o.y) * ri.inv.y, ty2 = (L.hi[1] + pad - o.y) * ri.inv.y;
    const float tz1 = (L.lo[2] - pad - o.z) * ri.inv.z, tz2 = (L.hi[2] + pad - o.z) * ri.inv.z;
    const float tn = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fminf(tz1, tz2));
    const float tf = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fmaxf(tz1, tz2));
    return tf >= tn && tf >= 0.0f && tn <= tcap;
}

// Per-face skip of a mesh: DObj::face_cull, or a constant when every mesh of the scene
// agrees (scene-specialized kernels: RTX_FACE_CULL_MODE 0 = never, 1 = always).
#ifndef RTX_FACE_CULL_MODE
#define RTX_FACE_CULL_MODE 2
#endif
template <class O>
RTX_HD bool face_cull(const O& ob) {
    return RTX_FACE_CULL_MODE == 2 ? ob.face_cull != 0 : RTX_FACE_CULL_MODE == 1;
}

// A box's conservative pre-test (same bound as the clusters'): false only when no exact
// slab test of the ray against [mn, mx] can pass with start <= tcap.
struct Box3 {
    float lo[3], hi[3];
};
RTX_HD bool box_maybe_hit(f3 mn, f3 mx, f3 o, const RayInv& ri, float tcap) {
    // the slabs are symmetric in (min, max): a box given with min > max on an axis
    // (NovelScene2's trails) spans [max, min] there
    const Box3 B{{fminf(mn.x, mx.x), fminf(mn.y, mx.y), fminf(mn.z, mx.z)},
                 {fmaxf(mn.x, mx.x), fmaxf(mn.y, mx.y), fmaxf(mn.z, mx.z)}};
    const float cm = fmaxf(fmaxf(fmaxf(fabsf(mn.x), fabsf(mn.y)), fmaxf(fabsf(mn.z), fabsf(mx.x))),
                           fmaxf(fabsf(mx.y), fabsf(mx.z)));
    return leaf_maybe_hit(B, o, ri, cm, tcap);
}

// The same pre-test from a box's record: a static box carries its sorted corners and max
// |coordinate| (rtx_api.hip convert_scene: c = lo, e = hi, c[3] = max), so the per-ray test
// skips the wave-uniform min / max / abs work (VALU on scalar values); a moving box forms
// them from its moved corners.
template <class O>
RTX_HD bool box_maybe_hit_obj(const O& ob, f3 mn, f3 mx, f3 o, const RayInv& ri, float tcap) {
#if !(defined(RTX_FIXED_STATIC) && RTX_FIXED_STATIC)
    if (ob.has_speed) return box_maybe_hit(mn, mx, o, ri, tcap);
#endif
    const Box3 B{{ob.c[0], ob.c[1], ob.c[2]}, {ob.e[0], ob.e[1], ob.e[2]}};
    return leaf_maybe_hit(B, o, ri, ob.c[3], tcap);
}

// Conservative pre-test of a mesh's bounding volume: false only when the exact test
// (mesh_bv) cannot pass with an entry at or before tcap. An AABB volume passes only rays
// that enter it at start >= 0, and every face hit inside it lies beyond that entry, so the
// padded box of the clusters' bound (box_maybe_hit) decides; sphere volumes always pass.
template <class O>
RTX_HD bool bv_maybe(const O& ob, f3 o, const RayInv& ri, float tcap) {
    // (the record carries the sorted corners and max |coordinate|, as for boxes)
    return ob.bv_type != BV_AABB ||
           leaf_maybe_hit(Box3{{ob.c[0], ob.c[1], ob.c[2]}, {ob.e[0], ob.e[1], ob.e[2]}}, o, ri, ob.c[3], tcap);
}

// Exact fp64 t of a candidate, recomputed from the object exactly as during its test
// (used only when two fp32 proxies tie; out of line to keep the hot loop's registers low).
// (RTX_HIT_T64_INLINE, scene-specialized kernels: inlined, with only the object kinds the
// scene has -- no call in the kernel, whose ABI constrains the whole kernel's registers)
#if defined(RTX_FIXED_COUNTS) && defined(RTX_HIT_T64_INLINE) && RTX_HIT_T64_INLINE
#define RTX_T64_ATTR __forceinline__
#define RTX_T64_HAS_BOX (RTX_FIXED_NB > 0)
#define RTX_T64_HAS_TRI (RTX_FIXED_NM > 0)
#else
#define RTX_T64_ATTR __attribute__((noinline))
#define RTX_T64_HAS_BOX 1
#define RTX_T64_HAS_TRI 1
#endif
__host__ __device__ RTX_T64_ATTR inline double hit_t64(const SceneView& S, int32_t obj, int32_t sb, f3 o, f3 d, float time) {
    const DObj ob = S.objs[obj];
    if (ob.type == OBJ_PLANE) {
        const f3 n = ld3(ob.b);
        return (double)dot(sub(moved(ob, ob.a, time), o), n) / (double)dot(d, n);
    }
    if (ob.type == OBJ_SPHERE) {
        double b = 0.0, s = 0.0, two_a = 1.0;
        sphere_roots(o, d, moved(ob, ob.a, time), ob.r2, b, s, two_a);
        return sb == 0 ? (-b - s) / two_a : (-b + s) / two_a;
    }
    if (RTX_T64_HAS_BOX && ob.type == OBJ_BOX) {
        double start = 0.0, end = 0.0;
        int label = 0;
        box_slabs(o, d, moved(ob, ob.a, time), moved(ob, ob.b, time), start, label, end);
        return start;
    }
    if (!RTX_T64_HAS_TRI) return INFINITY;  // (no other kind in the scene)
    const DTri T = S.tris[ob.tri_begin + sb];
    const f3 n = ld3(T.n);
    return (double)dot(sub(ld3(T.v0), o), n) / (double)dot(d, n);
}

// min(intersections, key=time) keeps the FIRST minimum of the list, which is ordered by
// object and then by hit within the object (scene.py:86-94). Candidates are offered in
// any object order but in hit order within an object; a candidate replaces the record
// iff its t is smaller, or equal with a smaller scene-order id. Proxies decide unless
// they are equal; then the exact fp64 values (and the ids) do.
// The tie rule in one out-of-line call (RTX_TIE_CALL, the secondary-ray kernels with
// hit_t64 inlined: one call site per offer instead of two -- MirrorRefraction 35.6 ->
// 35.0 us; in the one-sample kernel the call's register constraints spilled 400 B/lane,
// profiles/r05/noslp/ab_tie_call.log): whether candidate (obj, sb) takes the tie from h.
__host__ __device__ __attribute__((noinline)) inline bool tie_takes(const SceneView& S, const Hit& h, int32_t obj,
                                                                  int32_t sb, f3 o, f3 d, float time) {
    const double a = hit_t64(S, obj, sb, o, d, time);
    if (h.obj < 0) return a < INFINITY;
    const double b = hit_t64(S, h.obj, h.sub, o, d, time);
    const DObj oa = S.objs[obj], ob = S.objs[h.obj];
    const int32_t fa = oa.type == OBJ_MESH ? S.tri_orig[oa.tri_begin + sb] : 0;
    const int32_t fb = ob.type == OBJ_MESH ? S.tri_orig[ob.tri_begin + h.sub] : 0;
    return a < b || (a == b && (oa.oid < ob.oid || (oa.oid == ob.oid && fa < fb)));
}
RTX_HD void offer(const SceneView& S, Hit& h, bool valid, float t32, int32_t obj, int32_t sb, f3 o, f3 d,
                  float time) {
    bool take = valid && t32 < h.t32;
    const bool tie = valid && t32 == h.t32;
#if defined(RTX_TIE_CALL) && RTX_TIE_CALL
    if (tie) take = tie_takes(S, h, obj, sb, o, d, time);
    if (false) {
#else
    if (tie) {
#endif
        const double a = hit_t64(S, obj, sb, o, d, time);
        if (h.obj < 0) {
            take = a < INFINITY;
        } else {
            const double b = hit_t64(S, h.obj, h.sub, o, d, time);
            // equal t: earlier object, then (same mesh) earlier face in OBJ order
            const DObj oa = S.objs[obj], ob = S.objs[h.obj];
            const int32_t fa = oa.type == OBJ_MESH ? S.tri_orig[oa.tri_begin + sb] : 0;
            const int32_t fb = ob.type == OBJ_MESH ? S.tri_orig[ob.tri_begin + h.sub] : 0;
            take = a < b || (a == b && (oa.oid < ob.oid || (oa.oid == ob.oid && fa < fb)));
        }
    }
    h.t32 = take ? t32 : h.t32;
    h.obj = take ? obj : h.obj;
    h.sub = take ? sb : h.sub;
}

// ------------------------------------------------------------------ textures
// Python `x % m` (float_rem: the result takes the sign of m).
RTX_HD double py_mod(double x, double m) {
    double r = fmod(x, m);
    if (r != 0.0) {
        if ((m < 0.0) != (r < 0.0)) r += m;
    } else {
        r = copysign(0.0, m);
    }
    return r;
}
// texture.getpixel((i, j)) with int() / float truncation; the reference raises for an
// index outside the image (only reachable through `x % w == w` rounding or NaN), the
// device reads texel 0 of that row/column instead.
template <class O>
RTX_HD f3 texel(const SceneView& S, const O& ob, double fi, double fj) {
    const int i = (fi > -1.0 && fi < (double)ob.tex_w) ? (int)fi : 0;
    const int j = (fj > -1.0 && fj < (double)ob.tex_h) ? (int)fj : 0;
    const uint32_t t = S.texels[ob.tex_off + j * ob.tex_w + i];
    return f3{S.lut255[t & 255u], S.lut255[(t >> 8) & 255u], S.lut255[(t >> 16) & 255u]};
}
// Plane.get_diffuse (simple_geometry.py:150-173); the projection uses the unmoved point.
template <class O>
RTX_HD f3 plane_diffuse(const SceneView& S, const O& ob, f3 point, float time) {
    if (!ob.has_tex) return ld3(S.mats[plane_material(ob, point, time)].diffuse);
    const f3 position = moved(ob, ob.a, time);
    const f3 n = ld3(ob.b);
    point = sub(point, scale(n, dot(sub(point, ld3(ob.a)), n)));
    const double u = (double)dot(sub(point, position), ld3(ob.c)) * 1000.0 / ob.tex_scale;
    const double v = (double)dot(sub(point, position), ld3(ob.e)) * 1000.0 / ob.tex_scale;
    return texel(S, ob, trunc(py_mod(u, (double)ob.tex_w)), trunc(py_mod(v, (double)ob.tex_h)));
}
// AABB.get_diffuse (simple_geometry.py:312-355), fp64 like the reference's Python floats.
template <class O>
RTX_HD f3 box_diffuse(const SceneView& S, const O& ob, f3 point, float time) {
    if (!ob.has_tex) return ld3(S.mats[ob.mat0].diffuse);
    const f3 mn = moved(ob, ob.a, time), mx = moved(ob, ob.b, time);
    const double px = point.x, py = point.y, pz = point.z;
    const double x = (px - mn.x) / ((double)mx.x - mn.x);
    const double y = (py - mn.y) / ((double)mx.y - mn.y);
    const double z = (pz - mn.z) / ((double)mx.z - mn.z);
    const double W = ob.tex_w, H = ob.tex_h, e = 1e-4;
    double i = 0.0, j = 0.0;
    if (fabs(px - mn.x) < e) { i = z * W; j = (1 - y) * H; }
    else if (fabs(px - mx.x) < e) { i = (1 - z) * W; j = (1 - y) * H; }
    else if (fabs(py - mn.y) < e) { i = x * W; j = (1 - z) * H; }
    else if (fabs(py - mx.y) < e) { i = x * W; j = z * H; }
    else if (fabs(pz - mn.z) < e) { i = (1 - x) * W; j = (1 - y) * H; }
    else if (fabs(pz - mx.z) < e) { i = x * W; j = (1 - y) * H; }
    // min(max(0, i), width - 1): Python keeps the first argument unless the second wins
    i = i > 0.0 ? i : 0.0;
    j = j > 0.0 ? j : 0.0;
    i = W - 1 < i ? W - 1 : i;
    j = H - 1 < j ? H - 1 : j;
    return texel(S, ob, i, j);
}
// Geometry.get_diffuse as _compute_regular_lighting calls it for Plane/AABB hits
// (scene.py:143-146); other geometry uses the hit material's diffuse.
template <class O>
RTX_HD f3 get_diffuse(const SceneView& S, const O& ob, f3 point, float time) {
    return ob.type == OBJ_PLANE ? plane_diffuse(S, ob, point, time) : box_diffuse(S, ob, point, time);
}

// ------------------------------------------------------------------ hierarchies (CSG)
// Hierarchy.intersect / shadow_intersect / is_inside / get_material (hierarchy.py:42-138)
// without recursion. R[k] is the ray handed to the nodes and leaves at depth k (R[0] =
// the world ray); a node at depth k hands R[k + 1] = Minv * R[k] to its children
// (hierarchy.py:43-45). P[k] is a point in the frame of the children of the depth-k node
// whose is_inside is being evaluated. Both stacks live in LDS on the device ([slot]
// [thread], 9 words per level), a local array in the host emulation.
struct HStack {
    float* base;
    int stride;
    RTX_HD void put_ray(int k, f3 o, f3 d) const {
        float* p = base + k * 9 * stride;
        p[0] = o.x; p[stride] = o.y; p[2 * stride] = o.z;
        p[3 * stride] = d.x; p[4 * stride] = d.y; p[5 * stride] = d.z;
    }
    RTX_HD void get_ray(int k, f3& o, f3& d) const {
        const float* p = base + k * 9 * stride;
        o = f3{p[0], p[stride], p[2 * stride]};
        d = f3{p[3 * stride], p[4 * stride], p[5 * stride]};
    }
    RTX_HD void put_pt(int k, f3 q) const {
        float* p = base + (k * 9 + 6) * stride;
        p[0] = q.x; p[stride] = q.y; p[2 * stride] = q.z;
    }
    RTX_HD f3 get_pt(int k) const {
        const float* p = base + (k * 9 + 6) * stride;
        return f3{p[0], p[stride], p[2 * stride]};
    }
};

// glm.vec3(m * glm.vec4(p, w)): GLM's mat4 * vec4 is (m[0] x + m[1] y) + (m[2] z + m[3] w).
template <class P>
RTX_HD f3 xform(P m, f3 p, float w) {
    float r[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) r[k] = (m[k] * p.x + m[4 + k] * p.y) + (m[8 + k] * p.z + m[12 + k] * w);
    return f3{r[0], r[1], r[2]};
}
// glm.normalize(glm.transpose(Minv) * glm.vec4(n, 0)).xyz (hierarchy.py:76): the
// normalisation is over all four components (vec4 dot = (x*x + y*y) + (z*z + w*w)).
template <class P>
RTX_HD f3 normal_xform(P mi, f3 n) {
    float o[4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
        o[r] = (mi[4 * r] * n.x + mi[4 * r + 1] * n.y) + (mi[4 * r + 2] * n.z + mi[4 * r + 3] * 0.0f);
    const float d2 = (o[0] * o[0] + o[1] * o[1]) + (o[2] * o[2] + o[3] * o[3]);
    const float inv = 1.0f / sqrtf(d2);
    return f3{o[0] * inv, o[1] * inv, o[2] * inv};
}

// AABB hit normal from the entry-slab label and the direction's sign (simple_geometry.py:231-242)
RTX_HD f3 box_normal(int label, f3 d) {
    const float dl = label == 0 ? d.x : (label == 1 ? d.y : d.z);
    const float sgn = dl < 0.0f ? 1.0f : (dl > 0.0f ? -1.0f : 0.0f);
    return f3{label == 0 ? sgn : 0.0f, label == 1 ? sgn : 0.0f, label == 2 ? sgn : 0.0f};
}

// Every hit of one leaf, in the reference's list order, with fp64 t (leaves of
// hierarchies are few: no fp32 proxies). emit(t64, position, normal, material).
// Spheres, planes and boxes emit through ONE call site (a loop over their <= 2 hits), so
// the walk-up the caller's emit inlines is compiled once per leaf_hits, not once per hit
// kind.
// SURF = false (shadow enumerations, diff_shadow): the hit's normal and material are not
// needed, so they are not computed (emit receives zeros and -1).
template <bool MESH, class O, class Emit, bool SURF = true>
RTX_HD void leaf_hits(const SceneView& S, const O& ob, f3 o, f3 d, float time, Emit&& emit) {
    double th[2];
    int nh = 0;
    f3 c = mk(0.0f, 0.0f, 0.0f), nb = mk(0.0f, 0.0f, 0.0f);
    if (ob.type == OBJ_SPHERE) {  // simple_geometry.py:20-46
        c = moved(ob, ob.a, time);
        double b, s, two_a;
        if (!sphere_roots(o, d, c, ob.r2, b, s, two_a)) return;
        const double t1 = (-b - s) / two_a, t2 = (-b + s) / two_a;
        if (t1 > 0.0) th[nh++] = t1;
        if (t2 > 0.0) th[nh++] = t2;
    } else if (ob.type == OBJ_PLANE) {  // :105-120
        nb = ld3(ob.b);
        const float den = dot(d, nb);
        if (!(fabsf(den) >= kEps4Up)) return;
        const double t = (double)dot(sub(moved(ob, ob.a, time), o), nb) / (double)den;
        if (!(t >= 0.0)) return;
        th[nh++] = t;
    } else if (ob.type == OBJ_BOX) {  // :188-249 (entry, then exit, both with the entry normal)
        double start, end;
        int label;
        if (!box_slabs(o, d, moved(ob, ob.a, time), moved(ob, ob.b, time), start, label, end)) return;
        if (start > end || start < 0.0) return;
        nb = box_normal(label, d);
        th[0] = start;
        th[1] = end;
        nh = 2;
    } else if (MESH && ob.type == OBJ_MESH) {  // mesh.py:72-119, faces in OBJ order
        if (!mesh_bv(ob, o, d)) return;
        for (int f = 0; f < ob.tri_count; ++f) {
            cref<DTri> T = S.tris[ob.tri_begin + f];
            const f3 n = ld3(T.n);
            const float den = dot(d, n);
            if (fabsf(den) < kEps4Up) continue;
            const f3 v0 = ld3(T.v0);
            const double t = (double)dot(sub(v0, o), n) / (double)den;
            if (t < 0.0) continue;
            const f3 p = get_point(o, d, t);
            if (dot(cross(ld3(T.e01), sub(p, v0)), n) >= 0.0f && dot(cross(ld3(T.e12), sub(p, ld3(T.v1))), n) >= 0.0f &&
                dot(cross(ld3(T.e20), sub(p, ld3(T.v2))), n) >= 0.0f)
                emit(t, p, !SURF ? n : ob.flat ? n : smooth_normal(T, (DTriN)S.trins[ob.tri_begin + f], p),
                     SURF ? ob.mat0 : -1);
        }
        return;
    }
#pragma unroll 1
    for (int k = 0; k < nh; ++k) {
        const double t = k ? th[1] : th[0];
        const f3 p = get_point(o, d, t);
        f3 nrm = nb;
        if (SURF && ob.type == OBJ_SPHERE) nrm = normalize(sub(p, c));
        emit(t, p, nrm, !SURF ? -1 : ob.type == OBJ_PLANE ? plane_material(ob, p, time) : ob.mat0);
    }
}

// Leaf shadow_intersect (simple_geometry.py:48-72, :122-131, :251-294; mesh.py:121-153).
template <bool MESH, class O>
RTX_HD bool leaf_shadow(const SceneView& S, const O& ob, f3 o, f3 d, double t_max, float time) {
    if (ob.type == OBJ_SPHERE) {
        double b, s, two_a;
        if (!sphere_roots(o, d, moved(ob, ob.a, time), ob.r2, b, s, two_a)) return false;
        const double t1 = (-b - s) / two_a;
        if (1e-3 < t1 && t1 < t_max) return true;
        const double t2 = (-b + s) / two_a;
        return 1e-3 < t2 && t2 < t_max;
    }
    if (ob.type == OBJ_PLANE) {
        const f3 n = ld3(ob.b);
        const float den = dot(d, n);
        if (!(fabsf(den) >= kEps4Up)) return false;  // None
        const double t = (double)dot(sub(moved(ob, ob.a, time), o), n) / (double)den;
        return 1e-4 < t && t < t_max;
    }
    if (ob.type == OBJ_BOX) return box_shadow(o, d, moved(ob, ob.a, time), moved(ob, ob.b, time), t_max);
    if (MESH && ob.type == OBJ_MESH) {
        if (!mesh_bv(ob, o, d)) return false;
        for (int f = 0; f < ob.tri_count; ++f) {
            cref<DTri> T = S.tris[ob.tri_begin + f];
            const f3 n = ld3(T.nu);
            const float den = dot(d, n);
            if (fabsf(den) < kEps4Up) continue;
            const f3 v0 = ld3(T.v0);
            const double t = (double)dot(sub(v0, o), n) / (double)den;
            if (t < 1e-4) continue;
            const f3 p = get_point(o, d, t);
            if (dot(cross(ld3(T.e01), sub(p, v0)), n) >= 0.0f && dot(cross(ld3(T.e12), sub(p, ld3(T.v1))), n) >= 0.0f &&
                dot(cross(ld3(T.e20), sub(p, ld3(T.v2))), n) >= 0.0f)
                return true;
        }
    }
    return false;
}

// Leaf is_inside: Sphere (simple_geometry.py:74-80, fp32 length vs the fp64 radius),
// AABB (:296-307); Plane and Mesh keep Geometry's False.
template <class O>
RTX_HD bool leaf_inside(const O& ob, f3 p, float time) {
    if (ob.type == OBJ_SPHERE) {
        const f3 q = sub(p, moved(ob, ob.a, time));
        return (double)sqrtf(dot(q, q)) < ob.radius;
    }
    if (ob.type == OBJ_BOX) {
        const f3 mn = moved(ob, ob.a, time), mx = moved(ob, ob.b, time);
        return mn.x < p.x && p.x < mx.x && mn.y < p.y && p.y < mx.y && mn.z < p.z && p.z < mx.z;
    }
    return false;
}

// Folds child `cidx`'s value v into the accumulator bit of its parent (kind pk, depth pd):
// union = any, intersection = all, difference = child 0 and not child 1.
RTX_HD uint32_t hfold(uint32_t acc, int32_t pk, int32_t pd, int32_t cidx, bool v) {
    const uint32_t bit = 1u << pd;
    const bool a = (acc & bit) != 0u;
    const bool r = pk == HN_UNION ? (a || v) : pk == HN_INTER ? (a && v) : (cidx == 0 ? v : (cidx == 1 ? (a && !v) : a));
    return r ? (acc | bit) : (acc & ~bit);
}
RTX_HD uint32_t hinit(uint32_t acc, int32_t kind, int32_t depth) {
    const uint32_t bit = 1u << depth;
    return kind == HN_INTER ? (acc | bit) : (acc & ~bit);
}
// The remaining children of an open node (kind k, depth dep) cannot change its value in
// any active lane: a union already true, an intersection already false, a difference
// false after child 0 (next child index nc). Wave-uniform.
RTX_HD bool hdecided(uint32_t acc, int32_t k, int32_t dep, int32_t nc) {
    const bool v = ((acc >> dep) & 1u) != 0u;
    if (k == HN_UNION) return RTX_ALL(v);
    if (k == HN_INTER || (k == HN_DIFF && nc >= 1)) return RTX_ALL(!v);
    return false;
}

// Culling tests against DBound boxes (conservative: a false answer is exact).
RTX_HD bool box_nonempty(const float RTX_CONST* lo, const float RTX_CONST* hi) {
    return lo[0] <= hi[0] && lo[1] <= hi[1] && lo[2] <= hi[2];
}
// The ray o + t d, t in [0, tcap], meets the box. The box is widened by
// 2^-8 (|o|_max + |box|_max): the reference's sphere test forms its discriminant from
// fp32 dot products of o - c, whose rounding (~2^-23 |o - c|^2 against a (dist^2 - r^2))
// lets it report hits up to ~2^-10.5 |o - c| outside the sphere; every other test is
// far tighter (plane/box/triangle points: ~2^-23 (|o| + |geometry|)).
#ifndef RTX_MEETS_RCP
#define RTX_MEETS_RCP 1
#endif
RTX_HD bool ray_meets(const float RTX_CONST* lo, const float RTX_CONST* hi, f3 o, f3 d, float tcap) {
#if defined(RTX_NO_CULL)
    return true;
#endif
    // lo[3]: the box's max |coordinate|, or -inf when it is empty (rtx_api.hip hb_store), so
    // no lane spends VALU on the wave-uniform emptiness test and maximum
    const float bm = lo[3];
    if (!(bm >= 0.0f)) return false;
    const float om = fmaxf(fabsf(o.x), fmaxf(fabsf(o.y), fabsf(o.z)));
    const float pad = 0x1p-8f * (om + bm);
    // v_rcp (1 ulp): its error moves an entry by ~2^-23 of (|box| + |o|) |1/d|, far
    // inside the pad's 2^-8 (|o| + |box|) |1/d|
    auto inv = [](float v) { return RTX_MEETS_RCP ? rcp_approx(fabsf(v) < 1e-30f ? copysignf(1e-30f, v) : v)
                                                  : 1.0f / (fabsf(v) < 1e-30f ? copysignf(1e-30f, v) : v); };
    const float ix = inv(d.x), iy = inv(d.y), iz = inv(d.z);
    const float tx1 = (lo[0] - pad - o.x) * ix, tx2 = (hi[0] + pad - o.x) * ix;
    const float ty1 = (lo[1] - pad - o.y) * iy, ty2 = (hi[1] + pad - o.y) * iy;
    const float tz1 = (lo[2] - pad - o.z) * iz, tz2 = (hi[2] + pad - o.z) * iz;
    const float tn = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fminf(tz1, tz2));
    const float tf = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fmaxf(tz1, tz2));
    return tn <= tf && tf >= 0.0f && tn <= tcap;
}
// Where the ray o + t d, t >= 0, enters the (unpadded) box: an ordering heuristic only.
RTX_HD float box_entry(const float RTX_CONST* lo, const float RTX_CONST* hi, f3 o, f3 d) {
    if (!box_nonempty(lo, hi)) return INFINITY;
    auto inv = [](float v) { return rcp_approx(fabsf(v) < 1e-30f ? copysignf(1e-30f, v) : v); };
    const float ix = inv(d.x), iy = inv(d.y), iz = inv(d.z);
    const float tx1 = (lo[0] - o.x) * ix, tx2 = (hi[0] - o.x) * ix;
    const float ty1 = (lo[1] - o.y) * iy, ty2 = (hi[1] - o.y) * iy;
    const float tz1 = (lo[2] - o.z) * iz, tz2 = (hi[2] - o.z) * iz;
    const float tn = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fminf(tz1, tz2));
    const float tf = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fmaxf(tz1, tz2));
    return (tn <= tf && tf >= 0.0f) ? fmaxf(tn, 0.0f) : INFINITY;
}
// The first active lane's value (wave-uniform); the host emulation's one lane.
RTX_HD float wave_first(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x)));
#else
    return x;
#endif
}
RTX_HD bool pt_in(const float RTX_CONST* lo, const float RTX_CONST* hi, f3 p) {
#if defined(RTX_NO_CULL)
    return true;
#endif
    return lo[0] <= p.x && p.x <= hi[0] && lo[1] <= p.y && p.y <= hi[1] && lo[2] <= p.z && p.z <= hi[2];
}

// Inlining of the CSG helpers. 2 (default): everything inlined; 1: is_inside /
// get_material / walk_up out of line; 0: also hier_closest / hier_shadow. Each helper has
// ONE call site per enumeration (leaf_hits emits through one site, diff_shadow enumerates
// both children through one hier_enum, hier_shadow reaches every difference node through
// one diff_shadow, walk_up tests siblings through one is_inside), so inlining no longer
// multiplies them: the NovelScene1 kernel went from 110 call sites (50 walk_up, 40
// is_inside), 230 VGPRs and 961 SGPR spills to 195 VGPRs and 262 SGPR spills with no
// hierarchy calls; NovelScene1 29.0 -> 27.9 ms, NovelScene2 155 -> 143 ms (same box,
// profiles/r03/csg_inline/). Out of line (1) the restructured code measured 30.3 ms, and
// occupancy bounds of 3 and 4 waves/SIMD spill (29.6, 36.9 ms).
#ifndef RTX_HIER_INLINE
#define RTX_HIER_INLINE 2
#endif
#if RTX_HIER_INLINE >= 2
#define RTX_HX RTX_HD
#else
#define RTX_HX __host__ __device__ __attribute__((noinline)) inline
#endif

// is_inside(x, p) for p in the frame of x's parent's children (hierarchy.py:111-129).
RTX_HX bool is_inside(const SceneView& S, const HStack& hs, int x, f3 p, float time) {
    if (!pt_in(S.ibox[x].lo, S.ibox[x].hi, p)) return false;
    cref<DNodeHot> X = S.nodes[x];
    if (X.kind == HN_LEAF) return leaf_inside(S.objs[X.obj], p, time);
    if (X.kind == HN_OTHER) return false;
    hs.put_pt(X.depth, xform(S.nmat[x].Minv, p, 1.0f));
    uint32_t acc = hinit(0u, X.kind, X.depth);
    int open = x;
    int32_t okind = X.kind, odepth = X.depth, oend = X.end, oparent = X.parent, ocidx = X.cidx;
    int i = x + 1;
    for (;;) {
        while (i >= oend) {  // close finished subtrees
            const bool v = ((acc >> odepth) & 1u) != 0u;
            if (open == x) return v;
            cref<DNodeHot> Pn = S.nodes[oparent];
            acc = hfold(acc, Pn.kind, Pn.depth, ocidx, v);
            open = oparent;
            okind = Pn.kind; odepth = Pn.depth; oend = Pn.end; oparent = Pn.parent; ocidx = Pn.cidx;
        }
        cref<DNodeHot> c = S.nodes[i];
        if ((okind == HN_DIFF && c.cidx >= 2) || hdecided(acc, okind, odepth, c.cidx)) { i = oend; continue; }
        if (c.kind == HN_LEAF) {
            acc = hfold(acc, okind, odepth, c.cidx, leaf_inside(S.objs[c.obj], hs.get_pt(odepth), time));
            ++i;
        } else if (c.kind == HN_OTHER) {
            acc = hfold(acc, okind, odepth, c.cidx, false);
            i = c.end;
        } else {
            hs.put_pt(c.depth, xform(S.nmat[i].Minv, hs.get_pt(odepth), 1.0f));
            acc = hinit(acc, c.kind, c.depth);
            open = i;
            okind = c.kind; odepth = c.depth; oend = c.end; oparent = c.parent; ocidx = c.cidx;
            ++i;
        }
    }
}

// get_material(x, p) (hierarchy.py:131-138, Plane.get_material, Geometry.get_material):
// the first child containing the point, recursively; -1 = None.
RTX_HX int32_t get_material(const SceneView& S, const HStack& hs, int x, f3 p, float time) {
    for (;;) {
        cref<DNodeHot> X = S.nodes[x];
        if (X.kind == HN_LEAF) {
            cref<DObj> ob = S.objs[X.obj];
            return ob.type == OBJ_PLANE ? plane_material(ob, p, time) : ob.mat0;
        }
        const f3 q = xform(S.nmat[x].Minv, p, 1.0f);
        int found = -1;
        for (int j = x + 1; j < X.end; j = S.nodes[j].end)
            if (is_inside(S, hs, j, q, time)) { found = j; break; }
        if (found < 0) return -1;
        x = found;
        p = q;
    }
}

// The filters and transforms a hit of leaf `cur` meets on its way up to node `stop`
// (inclusive): intersection keeps hits inside every sibling, difference keeps child-0
// hits outside child 1 and child-1 hits inside child 0 (material of child 0, normal
// negated), then None materials fall back to the node's and position/normal move to the
// parent frame (hierarchy.py:49-76). Returns false if a filter drops the hit.
template <bool SURF = true>
RTX_HX bool walk_up(const SceneView& S, const HStack& hs, int cur, int stop, float time, f3& pos, f3& n,
                    int32_t& mat) {
    while (cur != stop) {
        cur = wave_uniform(cur);  // (a leaf's ancestors: the same in every lane)
        cref<DNodeHot> c = S.nodes[cur];
        const int a = c.parent;
        cref<DNodeHot> A = S.nodes[a];
        if (A.kind == HN_INTER || A.kind == HN_DIFF) {
            // intersection: every other child must contain the hit; difference: child 1 must
            // not contain a child-0 hit, child 0 must contain a child-1 hit (one is_inside site)
            const bool inter = A.kind == HN_INTER;
            const int c0 = a + 1, c1 = S.nodes[c0].end;
            const bool keep = inter || c.cidx != 0;  // the is_inside answer that keeps the hit
            for (int j = inter ? c0 : (c.cidx == 0 ? c1 : c0); j < A.end; j = S.nodes[j].end) {
                if (j == cur) continue;
                if (is_inside(S, hs, wave_uniform(j), pos, time) != keep) return false;
                if (!inter) break;
            }
            if (SURF && !inter && c.cidx != 0) {
                mat = get_material(S, hs, c0, pos, time);
                n = neg(n);
            }
        }
        if (SURF && mat < 0) mat = A.mat0 < 0 ? 0 : A.mat0;  // the reference raises IndexError for A.mat0 < 0
        pos = xform(S.nmat[a].M, pos, 1.0f);
        if (SURF) n = normal_xform(S.nmat[a].Minv, n);
        cur = a;
    }
    return true;
}

// Enumerates s.intersect(R[depth(s)]) in the reference's list order: want(t64) is asked
// before a hit's filters run (t does not change on the way up), take(t64, position,
// normal, material, leaf DObj) receives every surviving hit in the frame of s's parent.
template <bool MESH, class Want, class Take, class Cap, bool SURF = true>
RTX_HD void hier_enum(const SceneView& S, const HStack& hs, int s, float time, Want& want, Take& take, Cap& cap) {
    // subtrees whose hit region the ray cannot meet before cap() are skipped (wave-uniform)
    auto culled = [&](int c, int32_t depth) {
        f3 ro, rd;
        hs.get_ray(depth, ro, rd);
        return !RTX_ANY(ray_meets(S.hbox[c].lo, S.hbox[c].hi, ro, rd, cap()));
    };
    s = wave_uniform(s);
    cref<DNodeHot> root = S.nodes[s];
    if (culled(s, root.depth)) return;
    if (root.kind == HN_OTHER) return;  // unknown hierarchy_type: no hits
    // preorder from s itself (a leaf root is visited once), one leaf visit site
    for (int i = s; i < root.end;) {
        i = wave_uniform(i);
        cref<DNodeHot> c = S.nodes[i];
        if (i != s) {
            if (c.pkind == HN_DIFF && c.cidx >= 2) { i = c.end; continue; }  // difference reads children 0, 1
            if (culled(i, c.depth)) { i = c.end; continue; }
            if (c.kind == HN_OTHER) { i = c.end; continue; }
        }
        f3 ro, rd;
        hs.get_ray(c.depth, ro, rd);
        if (c.kind == HN_LEAF) {
            const int32_t obj = c.obj, li = i;
            auto emit = [&](double t, f3 pos, f3 n, int32_t mat) {
                if (!want(t)) return;
                if (walk_up<SURF>(S, hs, li, s, time, pos, n, mat)) take(t, pos, n, mat, obj);
            };
            leaf_hits<MESH, cref<DObj>, decltype(emit)&, SURF>(S, S.objs[obj], ro, rd, time, emit);
        } else {
            hs.put_ray(c.depth + 1, xform(S.nmat[i].Minv, ro, 1.0f), xform(S.nmat[i].Minv, rd, 0.0f));
        }
        ++i;
    }
}

// Difference.shadow_intersect (hierarchy.py:95-107): every hit of child 0 / child 1 past
// the shadow epsilon that the other child does not veto; no t_max test.
template <bool MESH>
RTX_HD bool diff_shadow(const SceneView& S, const HStack& hs, int x, float time) {
    x = wave_uniform(x);
    cref<DNodeHot> X = S.nodes[x];
    {
        f3 ro, rd;
        hs.get_ray(X.depth, ro, rd);
        hs.put_ray(X.depth + 1, xform(S.nmat[x].Minv, ro, 1.0f), xform(S.nmat[x].Minv, rd, 0.0f));
    }
    const int c0 = x + 1, c1 = S.nodes[c0].end;
    bool found = false;
    auto want = [&](double t) { return !found && t > 1e-4; };
    auto cap = [&]() { return found ? -1.0f : INFINITY; };
    // child 0's hits count outside child 1, child 1's inside child 0 (one enumeration site)
#pragma unroll 1
    for (int k = 0; k < 2; ++k) {
        const int mine = k ? c1 : c0, other = k ? c0 : c1;
        auto take = [&](double, f3 pos, f3, int32_t, int32_t) {
            found = is_inside(S, hs, wave_uniform(other), pos, time) == (k != 0);
        };
        // (a shadow needs where the hit is, not its normal or material)
        hier_enum<MESH, decltype(want), decltype(take), decltype(cap), false>(S, hs, mine, time, want, take, cap);
    }
    return found;
}

// Best hierarchy hit: the surface the walk-up produced (world frame).
constexpr int32_t kHierHit = -2;  // Hit.obj of a hierarchy hit; Hit.sub then holds the root's oid
struct HHit {
    double t64;
    f3 pos, n;
    int32_t mat, gobj;  // gobj: the leaf DObj (Plane/AABB get_diffuse), -1 otherwise
};

// (library build knob of the CSG-specialized split passes, below; the host sizes their LDS
// from it)
#ifndef RTX_CSG_RAYREG
#define RTX_CSG_RAYREG 1
#endif
#if defined(RTX_CSG_STATIC)
// ---- Hierarchies with their shape as compile-time constants (the scene-specialized split
// passes, rtx_api.hip jit_csg_tables): the traversals above -- the same tests in the same
// order, the same wave votes, the same arithmetic -- unrolled over the scene's node table
// (rtx_csg::kNode, kM, kMinv in the kernel's source), so node fields and matrices are
// literals and no traversal step waits on a node record. Points and rays descend by value
// (RTX_CSG_RAYREG 0: rays through the LDS stack at constant levels, as the loop form). Only
// the boxes (per motion time) and the leaves' DObj records are read from memory, at
// constant offsets.
namespace csg {
using rtx_csg::kNode;
// The boxes of node I (hit, inside, shadow) and the leaves' object records: the uploaded
// arrays, or (RTX_CSG_BAKED 2: the boxes, 3: also the records; option jit_csg) the camera's
// values baked into the source with the tables -- the same bytes, reads at constant offsets
// folding to literals. (Measured slower: rtx_api.hip jit_csg_baked.)
#if defined(RTX_CSG_BAKED)
template <int I> RTX_HD cref<DBox> hbox(const SceneView&) { return ((cptr<DBox>)rtx_csg::kBoxes)[I]; }
template <int I> RTX_HD cref<DBox> ibox(const SceneView&) { return ((cptr<DBox>)rtx_csg::kBoxes)[rtx_csg::kCount + I]; }
template <int I> RTX_HD cref<DBox> sbox(const SceneView&) { return ((cptr<DBox>)rtx_csg::kBoxes)[2 * rtx_csg::kCount + I]; }
#else
template <int I> RTX_HD cref<DBox> hbox(const SceneView& S) { return S.hbox[I]; }
template <int I> RTX_HD cref<DBox> ibox(const SceneView& S) { return S.ibox[I]; }
template <int I> RTX_HD cref<DBox> sbox(const SceneView& S) { return S.sbox[I]; }
#endif
#if defined(RTX_CSG_BAKED) && RTX_CSG_BAKED >= 3
template <int O> RTX_HD cref<DObj> obj(const SceneView&) { return ((cptr<DObj>)rtx_csg::kObjs)[O]; }
#else
template <int O> RTX_HD cref<DObj> obj(const SceneView& S) { return S.objs[O]; }
#endif
RTX_HD bool fold(bool a, int32_t pk, int32_t cidx, bool v) {  // hfold for one node's value
    return pk == HN_UNION ? (a || v) : pk == HN_INTER ? (a && v) : (cidx == 0 ? v : (cidx == 1 ? (a && !v) : a));
}
RTX_HD bool decided(bool a, int32_t k, int32_t nc) {  // hdecided
    if (k == HN_UNION) return RTX_ALL(a);
    if (k == HN_INTER || (k == HN_DIFF && nc >= 1)) return RTX_ALL(!a);
    return false;
}

// is_inside: the value of X's children (X inner, q in their frame), no box test
// (is_inside's loop tests the box of the node it is called on only)
template <int X>
RTX_HD bool inside_body(const SceneView& S, f3 p, float time);
template <int X, int C>
RTX_HD bool inside_kids(const SceneView& S, f3 q, float time, bool acc) {
    constexpr rtx_csg::CNode x = kNode[X];
    if constexpr (C >= x.end) {
        return acc;
    } else {
        constexpr rtx_csg::CNode c = kNode[C];
        if constexpr (x.kind == HN_DIFF && c.cidx >= 2) {
            return acc;
        } else {
            if (decided(acc, x.kind, c.cidx)) return acc;
            bool v = false;
            if constexpr (c.kind == HN_LEAF) v = leaf_inside(obj<c.obj>(S), q, time);
            else if constexpr (c.kind != HN_OTHER) v = inside_body<C>(S, q, time);
            return inside_kids<X, c.end>(S, q, time, fold(acc, x.kind, c.cidx, v));
        }
    }
}
template <int X>
RTX_HD bool inside_body(const SceneView& S, f3 p, float time) {
    return inside_kids<X, X + 1>(S, xform(rtx_csg::kMinv[X], p, 1.0f), time, kNode[X].kind == HN_INTER);
}
// is_inside(X, p)
template <int X>
RTX_HD bool inside(const SceneView& S, f3 p, float time) {
    if (!pt_in(ibox<X>(S).lo, ibox<X>(S).hi, p)) return false;
    constexpr rtx_csg::CNode x = kNode[X];
    if constexpr (x.kind == HN_LEAF) return leaf_inside(obj<x.obj>(S), p, time);
    else if constexpr (x.kind == HN_OTHER) return false;
    else return inside_body<X>(S, p, time);
}

// get_material(X, p)
template <int X, int J>
RTX_HD int32_t material_kids(const SceneView& S, f3 q, float time);
template <int X>
RTX_HD int32_t material(const SceneView& S, f3 p, float time) {
    constexpr rtx_csg::CNode x = kNode[X];
    if constexpr (x.kind == HN_LEAF) {
        cref<DObj> ob = obj<x.obj>(S);
        return ob.type == OBJ_PLANE ? plane_material(ob, p, time) : ob.mat0;
    } else {
        return material_kids<X, X + 1>(S, xform(rtx_csg::kMinv[X], p, 1.0f), time);
    }
}
template <int X, int J>
RTX_HD int32_t material_kids(const SceneView& S, f3 q, float time) {
    if constexpr (J >= kNode[X].end) {
        return -1;
    } else {
        if (inside<J>(S, q, time)) return material<J>(S, q, time);
        return material_kids<X, kNode[J].end>(S, q, time);
    }
}

// walk_up's filter at parent A of CUR: the siblings from J on must contain the hit (KEEP)
// or not; a difference tests one
template <int A, int CUR, int J, bool INTER, bool KEEP>
RTX_HD bool walk_filter(const SceneView& S, float time, f3 pos) {
    if constexpr (J >= kNode[A].end) {
        return true;
    } else if constexpr (J == CUR) {
        return walk_filter<A, CUR, kNode[J].end, INTER, KEEP>(S, time, pos);
    } else {
        if (inside<J>(S, pos, time) != KEEP) return false;
        if constexpr (!INTER) return true;
        else return walk_filter<A, CUR, kNode[J].end, INTER, KEEP>(S, time, pos);
    }
}
// walk_up(CUR -> STOP)
template <int CUR, int STOP, bool SURF>
RTX_HD bool walk(const SceneView& S, float time, f3& pos, f3& n, int32_t& mat) {
    if constexpr (CUR == STOP) {
        return true;
    } else {
        constexpr rtx_csg::CNode c = kNode[CUR];
        constexpr int A = c.parent;
        constexpr rtx_csg::CNode a = kNode[A];
        if constexpr (a.kind == HN_INTER || a.kind == HN_DIFF) {
            constexpr bool inter = a.kind == HN_INTER;
            constexpr int c0 = A + 1;
            constexpr int j0 = inter ? c0 : (c.cidx == 0 ? kNode[c0].end : c0);
            if (!walk_filter<A, CUR, j0, inter, inter || c.cidx != 0>(S, time, pos)) return false;
            if constexpr (SURF && !inter && c.cidx != 0) {
                mat = material<c0>(S, pos, time);
                n = neg(n);
            }
        }
        if (SURF && mat < 0) mat = a.mat0 < 0 ? 0 : a.mat0;
        pos = xform(rtx_csg::kM[A], pos, 1.0f);
        if (SURF) n = normal_xform(rtx_csg::kMinv[A], n);
        return walk<A, STOP, SURF>(S, time, pos, n, mat);
    }
}

// Rays descend by value (RTX_CSG_RAYREG 1: registers) or, as the loop form, through the
// LDS stack at constant levels (0): at_depth / to_depth are the two forms' reads and writes.
template <int DEPTH>
RTX_HD void at_depth(const HStack& hs, f3& ro, f3& rd) {
#if !RTX_CSG_RAYREG
    hs.get_ray(DEPTH, ro, rd);
#else
    (void)hs, (void)ro, (void)rd;
#endif
}
template <int DEPTH>
RTX_HD void to_depth(const HStack& hs, f3 ro, f3 rd) {
#if !RTX_CSG_RAYREG
    hs.put_ray(DEPTH, ro, rd);
#else
    (void)hs, (void)ro, (void)rd;
#endif
}

// hier_enum(ROOT): node I of ROOT's subtree in preorder, (ro, rd) the ray of its depth
template <int X, int C, int ROOT, bool MESH, bool SURF, class Want, class Take, class Cap>
RTX_HD void enum_kids(const SceneView& S, const HStack& hs, f3 ro, f3 rd, float time, Want& want, Take& take, Cap& cap);
template <int I, int ROOT, bool MESH, bool SURF, class Want, class Take, class Cap>
RTX_HD void enum_node(const SceneView& S, const HStack& hs, f3 ro, f3 rd, float time, Want& want, Take& take, Cap& cap) {
    constexpr rtx_csg::CNode c = kNode[I];
    if constexpr (I != ROOT && c.pkind == HN_DIFF && c.cidx >= 2) {
        return;  // difference reads children 0, 1
    } else {
        at_depth<c.depth>(hs, ro, rd);
        if constexpr (I != ROOT)  // (the caller tested the root's box)
            if (!RTX_ANY(ray_meets(hbox<I>(S).lo, hbox<I>(S).hi, ro, rd, cap()))) return;
        if constexpr (c.kind == HN_LEAF) {
            auto emit = [&](double t, f3 pos, f3 n, int32_t mat) {
                if (!want(t)) return;
                if (walk<I, ROOT, SURF>(S, time, pos, n, mat)) take(t, pos, n, mat, c.obj);
            };
            leaf_hits<MESH, cref<DObj>, decltype(emit)&, SURF>(S, obj<c.obj>(S), ro, rd, time, emit);
        } else if constexpr (c.kind != HN_OTHER) {
            const f3 co = xform(rtx_csg::kMinv[I], ro, 1.0f), cd = xform(rtx_csg::kMinv[I], rd, 0.0f);
            to_depth<c.depth + 1>(hs, co, cd);
            enum_kids<I, I + 1, ROOT, MESH, SURF>(S, hs, co, cd, time, want, take, cap);
        }
    }
}
template <int X, int C, int ROOT, bool MESH, bool SURF, class Want, class Take, class Cap>
RTX_HD void enum_kids(const SceneView& S, const HStack& hs, f3 ro, f3 rd, float time, Want& want, Take& take, Cap& cap) {
    if constexpr (C < kNode[X].end) {
        enum_node<C, ROOT, MESH, SURF>(S, hs, ro, rd, time, want, take, cap);
        enum_kids<X, kNode[C].end, ROOT, MESH, SURF>(S, hs, ro, rd, time, want, take, cap);
    }
}
template <int ROOT, bool MESH, bool SURF, class Want, class Take, class Cap>
RTX_HD void enum_root(const SceneView& S, const HStack& hs, f3 ro, f3 rd, float time, Want& want, Take& take, Cap& cap) {
    at_depth<kNode[ROOT].depth>(hs, ro, rd);
    if (!RTX_ANY(ray_meets(hbox<ROOT>(S).lo, hbox<ROOT>(S).hi, ro, rd, cap()))) return;
    enum_node<ROOT, ROOT, MESH, SURF>(S, hs, ro, rd, time, want, take, cap);
}

// diff_shadow(X), (ro, rd) the ray of X's depth
template <int X, bool MESH>
RTX_HD bool diff_shadow(const SceneView& S, const HStack& hs, f3 ro, f3 rd, float time) {
    constexpr rtx_csg::CNode x = kNode[X];
    at_depth<x.depth>(hs, ro, rd);
    const f3 co = xform(rtx_csg::kMinv[X], ro, 1.0f), cd = xform(rtx_csg::kMinv[X], rd, 0.0f);
    to_depth<x.depth + 1>(hs, co, cd);
    constexpr int c0 = X + 1, c1 = kNode[c0].end;
    static_assert(c1 < x.end, "a difference has two children (rtx_api.hip jit_csg_tables)");
    bool found = false;
    auto want = [&](double t) { return !found && t > 1e-4; };
    auto cap = [&]() { return found ? -1.0f : INFINITY; };
    {
        auto take = [&](double, f3 pos, f3, int32_t, int32_t) { found = inside<c1>(S, pos, time) == false; };
        enum_root<c0, MESH, false>(S, hs, co, cd, time, want, take, cap);
    }
    {
        auto take = [&](double, f3 pos, f3, int32_t, int32_t) { found = inside<c0>(S, pos, time) == true; };
        enum_root<c1, MESH, false>(S, hs, co, cd, time, want, take, cap);
    }
    return found;
}

// hier_shadow: the children of the open node X (value acc so far), (ro, rd) their ray
template <int X, int C, bool MESH>
RTX_HD bool shadow_kids(const SceneView& S, const HStack& hs, f3 ro, f3 rd, double t_max, float time, bool acc) {
    constexpr rtx_csg::CNode x = kNode[X];
    if constexpr (C >= x.end) {
        return acc;
    } else {
        constexpr rtx_csg::CNode c = kNode[C];
        if (decided(acc, x.kind, c.cidx)) return acc;
        at_depth<c.depth>(hs, ro, rd);
        const bool live = ray_meets(sbox<C>(S).lo, sbox<C>(S).hi, ro, rd, INFINITY);
        bool v = false;
        if (RTX_ANY(live)) {
            if constexpr (c.kind == HN_LEAF) {
                v = live && leaf_shadow<MESH>(S, obj<c.obj>(S), ro, rd, t_max, time);
            } else if constexpr (c.kind == HN_DIFF) {
                if (live) v = diff_shadow<C, MESH>(S, hs, ro, rd, time);
            } else if constexpr (c.kind != HN_OTHER) {
                const f3 co = xform(rtx_csg::kMinv[C], ro, 1.0f), cd = xform(rtx_csg::kMinv[C], rd, 0.0f);
                to_depth<c.depth + 1>(hs, co, cd);
                v = shadow_kids<C, C + 1, MESH>(S, hs, co, cd, t_max, time, c.kind == HN_INTER);
            }
        }
        return shadow_kids<X, c.end, MESH>(S, hs, ro, rd, t_max, time, fold(acc, x.kind, c.cidx, v));
    }
}
// hier_shadow(R)
template <int R, bool MESH>
RTX_HD bool shadow_root(const SceneView& S, const HStack& hs, f3 o, f3 d, double t_max, float time) {
    to_depth<0>(hs, o, d);
    if (!RTX_ANY(ray_meets(sbox<R>(S).lo, sbox<R>(S).hi, o, d, INFINITY))) return false;
    constexpr rtx_csg::CNode r = kNode[R];
    if constexpr (r.kind == HN_OTHER) {
        return false;
    } else if constexpr (r.kind == HN_DIFF) {
        return diff_shadow<R, MESH>(S, hs, o, d, time);
    } else {
        const f3 co = xform(rtx_csg::kMinv[R], o, 1.0f), cd = xform(rtx_csg::kMinv[R], d, 0.0f);
        to_depth<1>(hs, co, cd);
        return shadow_kids<R, R + 1, MESH>(S, hs, co, cd, t_max, time, r.kind == HN_INTER);
    }
}
// hier_occluded: roots R, R' = end(R), ... (Q: R's ordinal)
template <bool MESH, int R, int Q>
RTX_HD bool occluded_roots(const SceneView& S, const HStack& hs, f3 o, f3 d, double t_max, float time, bool occ,
                           uint32_t rmask) {
    if constexpr (R >= rtx_csg::kCount) {
        return occ;
    } else {
        if (RTX_ALL(occ)) return occ;
        const bool live = !occ && (Q >= 32 || ((rmask >> Q) & 1u) != 0u);
        if (RTX_ANY(live)) {
            if (live) occ = shadow_root<R, MESH>(S, hs, o, d, t_max, time);
        }
        return occluded_roots<MESH, kNode[R].end, Q + 1>(S, hs, o, d, t_max, time, occ, rmask);
    }
}
// hier_closest: roots R, R' = end(R), ... (Q: R's ordinal)
template <bool MESH, int R, int Q>
RTX_HD void closest_roots(const SceneView& S, const HStack& hs, f3 o, f3 d, float time, Hit& h, HHit& hh,
                          uint32_t rmask) {
    if constexpr (R < rtx_csg::kCount) {
        if (!(Q < 32 && !((rmask >> Q) & 1u))) {  // (else the tile's rays miss its hit box)
            constexpr int32_t oid = kNode[R].oid;
            auto want = [&](double t) {
                const float t32 = (float)t;
                if (t32 < h.t32) return true;
                if (!(t32 == h.t32)) return false;
                if (h.obj == -1) return t < INFINITY;
                double bt;
                int32_t bo;
                if (h.obj == kHierHit) { bt = hh.t64; bo = h.sub; }
                else { bt = hit_t64(S, h.obj, h.sub, o, d, time); bo = S.objs[h.obj].oid; }
                return t < bt || (t == bt && oid < bo);
            };
            auto take = [&](double t, f3 pos, f3 n, int32_t mat, int32_t leaf) {
                const int32_t ty = S.objs[leaf].type;
                h.t32 = (float)t;
                h.obj = kHierHit;
                h.sub = oid;
                hh = HHit{t, pos, n, mat, (ty == OBJ_PLANE || ty == OBJ_BOX) ? leaf : -1};
            };
            auto cap = [&]() { return h.t32; };
            enum_root<R, MESH, true>(S, hs, o, d, time, want, take, cap);
        }
        closest_roots<MESH, kNode[R].end, Q + 1>(S, hs, o, d, time, h, hh, rmask);
    }
}
}  // namespace csg
#endif

// Hierarchy.shadow_intersect of root r for the world ray (o, d): union = any child,
// intersection = every child (each tested on its own), difference = diff_shadow.
#if RTX_HIER_INLINE >= 1
#define RTX_HY RTX_HD
#else
#define RTX_HY __host__ __device__ __attribute__((noinline))
#endif
template <bool MESH>
RTX_HY bool hier_shadow(const SceneView& S, const HStack& hs, int r, f3 o, f3 d, double t_max, float time) {
    // the traversal state is wave-uniform by construction (every branch on it is a wave
    // vote); readfirstlane says so to the compiler, which otherwise keeps node indices in
    // VGPRs and loads the node records per lane
    r = wave_uniform(r);
    hs.put_ray(0, o, d);
    if (!RTX_ANY(ray_meets(S.sbox[r].lo, S.sbox[r].hi, o, d, INFINITY))) return false;
    cref<DNodeHot> R = S.nodes[r];
    if (R.kind == HN_OTHER) return false;
    // difference nodes (the root or inner ones) are evaluated at ONE diff_shadow site: dx
    // is the pending node (wave-uniform), dlive whether this lane's ray meets its box
    const bool root_diff = R.kind == HN_DIFF;
    int dx = root_diff ? r : -1, dend = 0;
    int32_t dcidx = 0;
    bool dlive = true;
    uint32_t acc = 0u;
    if (!root_diff) {
        hs.put_ray(1, xform(S.nmat[r].Minv, o, 1.0f), xform(S.nmat[r].Minv, d, 0.0f));
        acc = hinit(0u, R.kind, 0);
    }
    int open = r;
    int32_t okind = R.kind, odepth = R.depth, oend = R.end, oparent = R.parent, ocidx = R.cidx;
    int i = r + 1;
    for (;;) {
        if (dx >= 0) {
            bool v = false;
            if (dlive) v = diff_shadow<MESH>(S, hs, dx, time);
            if (root_diff) return v;
            acc = hfold(acc, okind, odepth, dcidx, v);
            i = dend;
            dx = -1;
        }
        while (i >= oend) {
            const bool v = ((acc >> odepth) & 1u) != 0u;
            if (open == r) return v;
            cref<DNodeHot> Pn = S.nodes[oparent];
            acc = hfold(acc, Pn.kind, Pn.depth, ocidx, v);
            open = oparent;
            okind = Pn.kind; odepth = Pn.depth; oend = Pn.end; oparent = Pn.parent; ocidx = Pn.cidx;
        }
        i = wave_uniform(i);
        cref<DNodeHot> c = S.nodes[i];
        if (hdecided(acc, okind, odepth, c.cidx)) { i = oend; continue; }
        bool live;
        {
            f3 ro, rd;
            hs.get_ray(c.depth, ro, rd);
            live = ray_meets(S.sbox[i].lo, S.sbox[i].hi, ro, rd, INFINITY);
        }
        if (!RTX_ANY(live)) {  // shadow_intersect is False for every lane
            acc = hfold(acc, okind, odepth, c.cidx, false);
            i = c.end;
        } else if (c.kind == HN_LEAF) {
            f3 lo, ld;
            hs.get_ray(c.depth, lo, ld);
            acc = hfold(acc, okind, odepth, c.cidx, live && leaf_shadow<MESH>(S, S.objs[c.obj], lo, ld, t_max, time));
            ++i;
        } else if (c.kind == HN_OTHER) {
            acc = hfold(acc, okind, odepth, c.cidx, false);
            i = c.end;
        } else if (c.kind == HN_DIFF) {
            dx = i;
            dlive = live;
            dcidx = c.cidx;
            dend = c.end;
        } else {
            f3 ro, rd;
            hs.get_ray(c.depth, ro, rd);
            hs.put_ray(c.depth + 1, xform(S.nmat[i].Minv, ro, 1.0f), xform(S.nmat[i].Minv, rd, 0.0f));
            acc = hinit(acc, c.kind, c.depth);
            open = i;
            okind = c.kind; odepth = c.depth; oend = c.end; oparent = c.parent; ocidx = c.cidx;
            ++i;
        }
    }
}

// The shadow rays of every hierarchy root, for the lanes not yet occluded. (Out of line,
// with hier_closest too, the kernel measured 247 VGPRs against 195 inlined: the calls cost
// more registers than they isolate.)
// rmask: the roots (bit q: the q-th, q < 32) the lane's ray may meet (DSGrid).
template <bool MESH>
RTX_HD bool hier_occluded(const SceneView& S, const HStack& hs, f3 o, f3 d, double t_max, float time, bool occ,
                          uint32_t rmask = ~0u) {
#if defined(RTX_CSG_STATIC)
    return csg::occluded_roots<MESH, 0, 0>(S, hs, o, d, t_max, time, occ, rmask);
#endif
    int q = 0;
    for (int r = 0; r < S.n_nodes; r = S.nodes[r].end, ++q) {
        if (RTX_ALL(occ)) break;
        const bool live = !occ && (q >= 32 || ((rmask >> q) & 1u) != 0u);
        if (!RTX_ANY(live)) continue;
        if (live) occ = hier_shadow<MESH>(S, hs, r, o, d, t_max, time);
    }
    return occ;
}

// Closest hit over the hierarchies, merged into h (flat objects done): a candidate wins
// with a smaller t, or an equal t and an earlier top-level object (scene.py:94).
#ifndef RTX_HIER_FIRST
#define RTX_HIER_FIRST 0  // nearest root first: measured slower (NovelScene1 29.1 -> 31.5 ms): off
#endif
// rmask: the roots (bit q: the q-th, q < 32) the wave's rays may hit (primary-ray bins).
template <bool MESH>
RTX_HY void hier_closest(const SceneView& S, const HStack& hs, f3 o, f3 d, float time, Hit& h, HHit& hh,
                         uint32_t rmask = ~0u) {
#if defined(RTX_CSG_STATIC)
    csg::to_depth<0>(hs, o, d);
    csg::closest_roots<MESH, 0, 0>(S, hs, o, d, time, h, hh, rmask);
    return;
#endif
    hs.put_ray(0, o, d);
    // The root whose hit box the wave's first ray enters first goes first: its hit then
    // caps the others' culling. Candidates compare by (t, top-level position), so the
    // order of the roots does not change the result (the order inside a root does, on
    // exact ties, and is kept).
    int32_t first = -1;
#if RTX_HIER_FIRST
    if (S.n_nodes > 0 && S.nodes[0].end < S.n_nodes) {
        float best = INFINITY;
        for (int r = 0; r < S.n_nodes; r = S.nodes[r].end) {
            const float e = wave_first(box_entry(S.hbox[r].lo, S.hbox[r].hi, o, d));
            if (e < best) { best = e; first = r; }
        }
    }
#endif
    int q = -1;  // the root's ordinal (when no root goes first)
    for (int k = first >= 0 ? -1 : 0; k < S.n_nodes;) {
        int r;
        if (k < 0) {
            r = first;
            k = 0;
        } else {
            r = k;
            k = S.nodes[k].end;
            if (r == first) continue;  // visited first
        }
        ++q;
        if (first < 0 && q < 32 && !((rmask >> q) & 1u)) continue;  // the tile's rays miss its hit box
        const int32_t oid = S.nodes[r].oid;
        auto want = [&](double t) {
            const float t32 = (float)t;
            if (t32 < h.t32) return true;
            if (!(t32 == h.t32)) return false;
            if (h.obj == -1) return t < INFINITY;
            double bt;
            int32_t bo;
            if (h.obj == kHierHit) { bt = hh.t64; bo = h.sub; }
            else { bt = hit_t64(S, h.obj, h.sub, o, d, time); bo = S.objs[h.obj].oid; }
            return t < bt || (t == bt && oid < bo);
        };
        auto take = [&](double t, f3 pos, f3 n, int32_t mat, int32_t leaf) {
            const int32_t ty = S.objs[leaf].type;
            h.t32 = (float)t;
            h.obj = kHierHit;
            h.sub = oid;
            hh = HHit{t, pos, n, mat, (ty == OBJ_PLANE || ty == OBJ_BOX) ? leaf : -1};
        };
        // a hit can win only at t <= the current best (the box test pads far beyond rounding)
        auto cap = [&]() { return h.t32; };
        hier_enum<MESH>(S, hs, r, time, want, take, cap);
    }
}

// Object/light counts (an experiment can pin them at compile time: -DRTX_FIXED_COUNTS=...)
#ifdef RTX_FIXED_COUNTS
#define RTX_NPLANE(S) RTX_FIXED_NP
#define RTX_NSPHERE(S) RTX_FIXED_NS
#define RTX_NBOX(S) RTX_FIXED_NB
#define RTX_NMESH(S) RTX_FIXED_NM
#define RTX_NLIGHTS(S) RTX_FIXED_NL
#else
#define RTX_NPLANE(S) (S).n_plane
#define RTX_NSPHERE(S) (S).n_sphere
#define RTX_NBOX(S) (S).n_box
#define RTX_NMESH(S) (S).n_mesh
#define RTX_NLIGHTS(S) (S).n_lights
#endif

// ------------------------------------------------------------------ closest hit
// Mesh.intersect's test of one face (mesh.py:77-117): t32 and whether the hit counts
// (lanes with maybe unset never do).
RTX_HD bool tri_hit(const DTri T, f3 o, f3 d, bool maybe, float& t32) {
    const f3 n = ld3(T.n);
    const float denom = dot(d, n);
    const f3 v0 = ld3(T.v0);
    const float num = dot(sub(v0, o), n);
    t32 = num / denom;
    // abs(denom) < epsilon -> skip; time < 0 -> skip
    bool valid = maybe && !(fabsf(denom) < kEps4Up) && !quot_neg(t32, num, denom);
    const f3 p = add(o, scale(d, t32));  // getPoint(time)
    const float b0 = dot(cross(ld3(T.e01), sub(p, v0)), n);
    const float b1 = dot(cross(ld3(T.e12), sub(p, ld3(T.v1))), n);
    const float b2 = dot(cross(ld3(T.e20), sub(p, ld3(T.v2))), n);
    return valid && b0 >= 0.0f && b1 >= 0.0f && b2 >= 0.0f;
}

// Wave-cooperative closest hit on a large mesh (experiment, -DRTX_WCOOP=1; off by
// default): the active lanes take their rays one at a time; for ray r
// every lane walks the same BVH path and the faces of the leaves it reaches (or of the
// tile's bin list, for a binned primary ray) are spread across the lanes, each lane
// folding its faces with `offer` (the same total order as the lane-per-ray loop: t32,
// then t64, then OBJ face index), and the lanes holding the smallest t32 hand their
// candidates to lane r, whose own `offer` keeps the reference's first-minimum choice.
#ifndef RTX_WCOOP
#define RTX_WCOOP 0
#endif
#ifndef RTX_WCOOP_MIN
#define RTX_WCOOP_MIN 1024  // faces: smaller meshes keep one ray per lane
#endif
#if RTX_WCOOP && defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ float lane_f(float x, int r) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), r));
}
// The active lanes holding the smallest non-negative key (ballots from the top bit down;
// lanes outside `active` never vote, whatever their registers hold).
__device__ __forceinline__ uint64_t wave_argmin(float v, uint64_t active) {
    const uint32_t key = __float_as_uint(v) & 0x7fffffffu;  // -0 ranks with +0
    uint64_t cand = active;
    for (int b = 30; b >= 0; --b) {
        const uint64_t z = __ballot(((key >> b) & 1u) == 0u) & cand;
        if (z) cand = z;
    }
    return cand;
}
__device__ __forceinline__ void coop_mesh(const SceneView& S, const DObj& ob, int32_t oi, int32_t bin,
                                          f3 o, f3 d, float time, Hit& h) {
    const uint64_t active = __ballot(1);
    const int lane = __lane_id();
    const int rank = __popcll(active & ((1ull << lane) - 1ull));
    const int nact = __popcll(active);
    const bool cull = face_cull(ob);
    const int32_t ub = bin >= 0 ? wave_uniform(bin) : -1;
    for (uint64_t pending = active; pending; pending &= pending - 1ull) {
        const int r = __builtin_amdgcn_readfirstlane(__builtin_ctzll(pending));
        const f3 ro{lane_f(o.x, r), lane_f(o.y, r), lane_f(o.z, r)};
        const f3 rd{lane_f(d.x, r), lane_f(d.y, r), lane_f(d.z, r)};
        const RayInv rri = ray_inv(ro, rd);
        float cap = lane_f(h.t32, r);  // ray r's best so far: a face must reach it
        Hit hl{INFINITY, -1, 0};
        int32_t face = -1;  // this lane's face of the batch
        int nbuf = 0;
        auto flush = [&]() {
            if (face >= 0) {
                bool fmaybe = true;
                if (cull) fmaybe = leaf_maybe_hit(RTX_FBOX(S, ob.tri_begin + face), ro, rri, ob.cmax, cap);
                float t32;
                const bool valid = tri_hit(RTX_TRI(S, ob.tri_begin + face), ro, rd, fmaybe, t32);
                offer(S, hl, valid, t32, oi, face, ro, rd, time);
            }
            face = -1;
            nbuf = 0;
            cap = fminf(cap, lane_f(hl.t32, __builtin_ctzll(wave_argmin(hl.t32, active))));
        };
        if (ub >= 0) {  // the tile's candidate faces, nearest first (rtx_api.hip primary_bins)
            const int32_t q1 = S.bin_start[ub + 1];
            for (int32_t q0 = S.bin_start[ub]; q0 < q1; q0 += nact) {
                if (cap < S.bin_zmin[q0]) break;
                const int32_t q = q0 + rank;
                face = q < q1 ? S.bin_faces[q] : -1;
                flush();
            }
        } else {
            for (int li = 0; li < ob.leaf_count;) {  // ray r's walk, the same in every lane
                const auto& L = RTX_LEAF(S, ob.leaf_begin + li);
                if (!RTX_ANY(leaf_maybe_hit(L, ro, rri, ob.cmax, cap))) { li = L.skip; continue; }
                ++li;
                for (int f0 = 0; f0 < L.count;) {  // the leaf's faces onto the free lanes
                    const int take = min(L.count - f0, nact - nbuf);
                    if (rank >= nbuf && rank < nbuf + take) face = L.first + f0 + (rank - nbuf);
                    nbuf += take;
                    f0 += take;
                    if (nbuf == nact) flush();
                }
            }
            if (nbuf > 0) flush();
        }
        const uint64_t has = __ballot(hl.obj >= 0);
        if (!has) continue;
        for (uint64_t win = wave_argmin(hl.obj >= 0 ? hl.t32 : INFINITY, active) & has; win; win &= win - 1ull) {
            const int j = __builtin_amdgcn_readfirstlane(__builtin_ctzll(win));
            const float t32 = lane_f(hl.t32, j);
            const int32_t sb = __builtin_amdgcn_readlane(hl.sub, j);
            if (lane == r) offer(S, h, true, t32, oi, sb, o, d, time);
        }
    }
}
#endif

template <bool B>
struct BoolTag {
    static constexpr bool value = B;
};

// Origin-only terms of the plane and sphere shadow tests -- dot(p0 - o, n) per plane,
// oc = o - c and dot(oc, oc) per sphere -- computed once per shading point and shared by
// its lights (the same operations, once instead of per light). Scene-specialized kernels
// only (fixed counts size the arrays); the generic kernels compute them per light.
struct OriginTerms {
#ifdef RTX_FIXED_COUNTS
    float pnum[RTX_FIXED_NP > 0 ? RTX_FIXED_NP : 1];
    f3 soc[RTX_FIXED_NS > 0 ? RTX_FIXED_NS : 1];
    float sq[RTX_FIXED_NS > 0 ? RTX_FIXED_NS : 1];
#endif
};

template <bool MESH, bool X, bool COUNT>
// prim (primary rays of one-sample unjittered static cameras, RTX_PRIM_ORIGIN): the
// origin-only terms of the planes and spheres, computed once on the host (rtx_camera_set,
// the same fp32 operations) instead of in every wave.
// blane: with bin, the ray's pixel in the bin's 8x8 tile (row * 8 + column), or -1.
RTX_HD Hit closest_hit(const SceneView& S, f3 o, f3 d, float time, Tally& tl, const HStack& hs, HHit& hh,
                       int32_t bin = -1, const OriginTerms* prim = nullptr, int32_t blane = -1) {
    Hit h{INFINITY, -1, 0};
    int oi = 0;
    // The flat objects. RTX_DEFER_TIES (flat scene-specialized kernels with secondary rays:
    // MirrorRefraction 39.7 -> 38.8 us; TwoSpheresPlane measured 22.0 -> 27.7 us with it --
    // no wave of it meets a tie, and without the exact pass's code it ran 21.6 us, so the
    // cost is that code's presence; out of line (noinline) it spilled 400 B/lane --
    // DepthOfField and TorusMesh equal, profiles/r05/noslp/ab_defer_ties.log): the first pass
    // takes strictly nearer hits only and notes an equal t (a tie the reference breaks by
    // the fp64 t and scene order, offer()); a wave that saw one runs the exact pass again.
    // h.t32 evolves the same in both (a tie never changes it), so without ties the first
    // pass's result is offer()'s.
    RayInv ri{};
    bool tie = false;
    auto flat = [&](auto exact_tag) {
        constexpr bool EXACT = decltype(exact_tag)::value;
        auto offer_ = [&](bool valid, float t32, int32_t obj, int32_t sb) {
            if (EXACT) {
                offer(S, h, valid, t32, obj, sb, o, d, time);
            } else {
                tie = tie || (valid && t32 == h.t32);
                const bool take = valid && t32 < h.t32;
                h.t32 = take ? t32 : h.t32;
                h.obj = take ? obj : h.obj;
                h.sub = take ? sb : h.sub;
            }
        };
        for (int k = 0; k < RTX_NPLANE(S); ++k, ++oi) {  // simple_geometry.py:105-120
            if (RTX_PROBE(18)) continue;  // cost probe: no planes in closest_hit
            const DObj ob = S.objs[oi];
            const f3 n = ld3(ob.b);
            const float denom = dot(d, n);
#ifdef RTX_FIXED_COUNTS
            const float num = prim ? prim->pnum[k] : dot(sub(moved(ob, ob.a, time), o), n);
#else
            const float num = dot(sub(moved(ob, ob.a, time), o), n);
#endif
            const float t32 = num / denom;
            // abs(denom) > epsilon and t >= 0
            const bool valid = fabsf(denom) >= kEps4Up && quot_nonneg(t32, num, denom);
            offer_(valid, t32, oi, 0);
        }
        // primary rays of a binned tile skip the spheres and boxes whose screen footprint
        // misses the tile (rtx_api.hip primary_bins; wave-uniform)
#if defined(RTX_PRIMARY_BINS) && !RTX_PRIMARY_BINS
        constexpr uint32_t omask = ~0u;
#else
        const uint32_t omask = bin >= 0 ? S.bin_objmask[wave_uniform(bin)] : ~0u;
#endif
        for (int k = 0; k < RTX_NSPHERE(S); ++k, ++oi) {  // simple_geometry.py:20-46
            if (!((omask >> (k & 15)) & 1u)) continue;
            if (RTX_PROBE(7)) continue;  // cost probe: no spheres in the primary test
            const DObj ob = S.objs[oi];
            const f3 ctr = moved(ob, ob.a, time);
            bool valid = false;
            float t32 = INFINITY;
            int32_t root = 0;
#ifdef RTX_FIXED_COUNTS
            const f3 oc = prim ? prim->soc[k] : sub(o, ctr);
            const float q = prim ? prim->sq[k] : dot(oc, oc);
#else
            const f3 oc = sub(o, ctr);
            const float q = dot(oc, oc);
#endif
            if (sphere_disc_sign_oc(d, oc, q, ob.r2f) >= 0) {  // fp64 only where a hit is possible
                double b, s, two_a;
                if (RTX_PROBE(4) ? sphere_roots(o, d, ctr, ob.r2, b, s, two_a) : sphere_roots_oc(d, oc, q, ob.r2, b, s, two_a)) {
                    double t = (-b - s) / two_a;
                    const bool near = t > 0.0;
                    // the far root only where some lane needs it (a ray from inside the sphere)
                    if (RTX_ANY(!near)) {
                        unspeculated();
                        if (!near) { t = (-b + s) / two_a; root = 1; }
                    }
                    valid = t > 0.0;
                    t32 = (float)t;
                }
            }
            offer_(valid, t32, oi, root);
        }
        if (RTX_NBOX(S) > 0 || (MESH && RTX_NMESH(S) > 0)) ri = ray_inv(o, d);
        for (int k = 0; k < RTX_NBOX(S); ++k, ++oi) {  // simple_geometry.py:188-249 (entry precedes exit)
            if (!((omask >> (16 + (k & 15))) & 1u)) continue;
            if (RTX_PROBE(17)) continue;  // cost probe: no boxes in closest_hit
            const DObj ob = S.objs[oi];
            const f3 mn = moved(ob, ob.a, time), mx = moved(ob, ob.b, time);
            double start = 0.0;
            int label = 0;
            bool valid;
            if (RTX_BOX_IV_CULL) {  // the intervals decide which lanes may hit before their best t
                const SlabIv iv = box_slabs_iv(o, d, mn, mx, &ri);
                const bool maybe = !box_iv_out(iv, h.t32);
                if (!RTX_ANY(maybe)) continue;
                valid = box_entry_iv(o, d, mn, mx, iv, maybe, start, label);
            } else {
                // the fp64 slabs only where some lane's ray may hit the box before its best t
                const bool maybe = box_maybe_hit_obj(ob, mn, mx, o, ri, h.t32);
                if (!RTX_ANY(maybe)) continue;
                valid = box_entry(o, d, mn, mx, maybe, start, label, &ri);
            }
            offer_(valid, (float)start, oi, label);
        }
    };
#if !defined(RTX_DEFER_TIES)
#define RTX_DEFER_TIES 0  // (rtx_api.hip jit_spec sets it for the secondary-ray kernels)
#endif
#if defined(RTX_FIXED_COUNTS) && RTX_DEFER_TIES
    if (!MESH && !X && !COUNT) {
        flat(BoolTag<false>{});
#if defined(RTX_TOOLS_BUILD) && defined(RTX_DEFER_PROBE)
        if (RTX_DEFER_PROBE == 1) tie = false;  // cost probe: never redo (wrong at ties)
#endif
        if (RTX_ANY(tie)) {
            unspeculated();
            h = Hit{INFINITY, -1, 0};
            oi = 0;
            flat(BoolTag<true>{});
        }
    } else
#endif
    {
        flat(BoolTag<true>{});
    }
    if (MESH) {
        for (int k = 0; k < RTX_NMESH(S); ++k, ++oi) {  // mesh.py:72-119, faces in order
            const DObj ob = S.objs[oi];
            // padded fp32 pre-test of an AABB volume (conservative, bv_maybe): the exact
            // test only where some lane's ray may enter the box before its best t
            if (!RTX_ANY(bv_maybe(ob, o, ri, h.t32))) continue;
            if (!mesh_bv(ob, o, d)) continue;  // the reference's bounding volume, quirks included
            // mesh.py:77-117 for stored face f (lanes with maybe set may take it)
#if RTX_WCOOP && defined(__HIP_DEVICE_COMPILE__)
            if (ob.tri_count >= RTX_WCOOP_MIN) {  // experiment: one ray per wave, faces across lanes
                coop_mesh(S, ob, oi, (bin >= 0 && S.mesh_bins && k == 0) ? bin : -1, o, d, time, h);
                continue;
            }
#endif
            auto test_face = [&](int f, bool maybe, bool cull) {
                bool fmaybe = maybe;
                if (cull) {  // the face's own padded box (the cluster's bound)
                    fmaybe = maybe && leaf_maybe_hit(RTX_FBOX(S, ob.tri_begin + f), o, ri, ob.cmax, h.t32);
                    if (!RTX_ANY(fmaybe)) return;  // no lane's ray can pass its exact test
                }
                tally_inc<COUNT>(tl, &Tally::tri);
                float t32;
                const bool valid = tri_hit(RTX_TRI(S, ob.tri_begin + f), o, d, fmaybe, t32);
                offer(S, h, valid, t32, oi, f, o, d, time);
            };
            if (bin >= 0 && S.mesh_bins && k == 0) {  // a primary ray: its tile's candidate faces
                const int32_t ub = wave_uniform(bin);  // the same in every lane of the tile's wave
                const int32_t q1 = S.bin_start[ub + 1];
                // a heavy tile: its chunks' closest faces, found by k_mesh_chunks this frame
                // (the same tests; the closest over the chunks is the closest over the list)
                const int32_t slot = (S.bin_heavy != nullptr && blane >= 0) ? S.bin_heavy[ub] : -1;
                if (slot >= 0) {
                    const int32_t nch = (q1 - S.bin_start[ub] + kHeavyChunk - 1) / kHeavyChunk;
                    for (int32_t c = 0; c < nch; ++c) {
                        const uint2 e = S.mesh_hits[(int64_t)(slot + c) * 64 + blane];
                        offer(S, h, (int32_t)e.y >= 0, __builtin_bit_cast(float, e.x), oi, (int32_t)e.y, o, d, time);
                    }
                    continue;
                }
#if defined(RTX_BIN_LDS) && RTX_BIN_LDS && defined(__HIP_DEVICE_COMPILE__)
                {
                    BinLds& sh = g_bin_lds[threadIdx.x >> 6];
                    const uint64_t act = __builtin_amdgcn_ballot_w64(true);  // (the lanes tracing here)
                    const int na = __builtin_popcountll(act);
                    const int rk = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
                    constexpr int kTriW = (int)(sizeof(DTri) / 16), kW = kTriW + (int)(sizeof(DFaceBox) / 16);
                    bool done = false;
                    for (int32_t qb = S.bin_start[ub]; qb < q1 && !done; qb += kHeavyChunk) {
                        if (RTX_ALL(h.t32 < S.bin_zmin[qb])) break;  // (the loop below's first exit test)
                        const int n = min(q1 - qb, kHeavyChunk);
                        wave_lds_sync();  // (the previous block's reads are done)
                        for (int i = rk; i < n; i += na) {
                            sh.face[i] = S.bin_faces[qb + i];
                            sh.zmin[i] = S.bin_zmin[qb + i];
                        }
                        wave_lds_sync();
                        for (int w = rk; w < n * kW; w += na) {
                            const int i = w / kW, k = w - i * kW;
                            const int64_t f = ob.tri_begin + sh.face[i];
                            if (k < kTriW)
                                reinterpret_cast<uint4*>(&sh.tri[i])[k] = reinterpret_cast<const uint4 RTX_CONST*>(&S.tris[f])[k];
                            else
                                reinterpret_cast<uint4*>(&sh.box[i])[k - kTriW] =
                                    reinterpret_cast<const uint4 RTX_CONST*>(&S.fboxes[f])[k - kTriW];
                        }
                        wave_lds_sync();
                        for (int i = 0; i < n; ++i) {
                            // faces come nearest first: once every lane's best hit precedes a
                            // face's nearest possible t, no later face can win (or tie)
                            if (RTX_ALL(h.t32 < sh.zmin[i])) { done = true; break; }
                            const DFaceBox B = sh.box[i];
                            const bool fmaybe = leaf_maybe_hit(B, o, ri, ob.cmax, h.t32);
                            if (!RTX_ANY(fmaybe)) continue;
                            tally_inc<COUNT>(tl, &Tally::tri);
                            float t32;
                            const bool valid = tri_hit(sh.tri[i], o, d, fmaybe, t32);
                            offer(S, h, valid, t32, oi, sh.face[i], o, d, time);
                        }
                    }
                }
#else
                for (int32_t q = S.bin_start[ub]; q < q1; ++q) {
                    // faces come nearest first: once every lane's best hit precedes a
                    // face's nearest possible t, no later face can win (or tie)
                    if (RTX_ALL(h.t32 < S.bin_zmin[q])) break;
                    test_face(S.bin_faces[q], true, true);
                }
#endif
                continue;
            }
            for (int li = 0; li < ob.leaf_count;) {  // stackless wave-uniform BVH walk
                const auto& L = RTX_LEAF(S, ob.leaf_begin + li);
                const bool maybe = leaf_maybe_hit(L, o, ri, ob.cmax, h.t32);
                if (!RTX_ANY(maybe)) { li = L.skip; continue; }
                ++li;
                for (int f = L.first; f < L.first + L.count; ++f) test_face(f, maybe, face_cull(ob));
            }
        }
    }
    if (X && !RTX_PROBE(9)) {  // hierarchies (hierarchy.py:42-78)
#if defined(RTX_PRIMARY_BINS) && !RTX_PRIMARY_BINS
        hier_closest<MESH>(S, hs, o, d, time, h, hh);
#else
        hier_closest<MESH>(S, hs, o, d, time, h, hh, bin >= 0 ? S.bin_rootmask[wave_uniform(bin)] : ~0u);
#endif
    }
    return h;
}

// ------------------------------------------------------------------ shadow any-hit
RTX_HD void origin_terms(const SceneView& S, f3 o, float time, OriginTerms& T) {
#ifdef RTX_FIXED_COUNTS
    int oi = 0;
    for (int k = 0; k < RTX_NPLANE(S); ++k, ++oi) {
        const DObj ob = S.objs[oi];
        T.pnum[k] = dot(sub(moved(ob, ob.a, time), o), ld3(ob.b));
    }
    for (int k = 0; k < RTX_NSPHERE(S); ++k, ++oi) {
        const DObj ob = S.objs[oi];
        T.soc[k] = sub(o, moved(ob, ob.a, time));
        T.sq[k] = dot(T.soc[k], T.soc[k]);
    }
#else
    (void)S; (void)o; (void)time; (void)T;
#endif
}

// Mesh.shadow_intersect's test of one face for the ray (o, d) (mesh.py:125-151: the
// unnormalized normal, no t_max).
template <class Tri>
RTX_HD bool shadow_tri(const Tri& T, f3 o, f3 d) {
    const f3 n = ld3(T.nu);
    const float denom = dot(d, n);
    const f3 v0 = ld3(T.v0);
    const float num = dot(sub(v0, o), n);
    const float t32 = num / denom;
    // abs(denom) < epsilon -> skip; time < shadow_epsilon -> skip
    bool hit = !(fabsf(denom) < kEps4Up) && !quot_lt(t32, num, denom, 1e-4, kEps4Near);
    const f3 p = add(o, scale(d, t32));
    return hit && dot(cross(ld3(T.e01), sub(p, v0)), n) >= 0.0f &&
           dot(cross(ld3(T.e12), sub(p, ld3(T.v1))), n) >= 0.0f &&
           dot(cross(ld3(T.e20), sub(p, ld3(T.v2))), n) >= 0.0f;
}
#ifndef RTX_LGRID_LANE
#define RTX_LGRID_LANE 1  // light-grid lists: 1 per lane, 0 one distinct cell of the wave at a time
#endif
// Per-lane light-grid lists two faces per step: the 81,920-face mesh at 1080p 0.263-0.277 ->
// 0.200 ms (its lit points near the shadow's edge run lists of up to ~200 faces, and the
// frame waited on those waves); TorusMesh (small mesh, short lists) 48.9 -> 53.4 us, so
// only kernels of scenes whose meshes have no face boxes (RTX_FACE_CULL_MODE 0) pair them.
#ifndef RTX_LGRID_PAIRS
#define RTX_LGRID_PAIRS (RTX_FACE_CULL_MODE == 0)
#endif

// The light-grid cell of a shadow ray from o toward a point light, d = L - o as the
// shader computes it (so -d = fl(o - L) exactly): >= 0 a cell, -1 the line through o and
// the light misses the mesh's cone (no face can occlude), -2 no grid answer (|w| out of
// the grid's range, NaN): walk the BVH.
RTX_HD int32_t lgrid_cell(cref<DLGrid> g, f3 d) {
    const f3 w = neg(d);
    const float w2 = dot(w, w);
    if (!(w2 >= g.r2min && w2 <= g.r2max)) return -2;
    const float wa = dot(w, ld3(g.a));
    if (wa * wa <= g.cos2 * w2) return -1;
    const float x = dot(w, ld3(g.u)) / wa, y = dot(w, ld3(g.v)) / wa;
    const int32_t G = g.G;
    auto clampi = [G](float t) {
        const int32_t i = (int32_t)floorf(t);
        return i < 0 ? 0 : (i > G - 1 ? G - 1 : i);
    };
    return clampi((y + g.tmax) * g.scale) * G + clampi((x + g.tmax) * g.scale);
}

// v of the first lane where pred holds (pred must hold somewhere), as a wave-uniform value.
RTX_HD int32_t first_where(int32_t v, bool pred) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_readlane(v, __builtin_ctzll(__ballot((int)pred)));
#else
    (void)pred;
    return v;
#endif
}

// The spheres, boxes and hierarchy roots directional light `light`'s shadow ray from p may
// meet (DSGrid); all bits: everything.
RTX_HD DSCell dir_shadow_mask(const SceneView& S, int light, f3 p) {
    cref<DSGrid> g = S.dsgrid[light];
    const int32_t G = g.G;
    if (G == 0) return DSCell{~0u, ~0u};
    const float m = fmaxf(fabsf(p.x), fmaxf(fabsf(p.y), fabsf(p.z)));
    if (!(m <= g.pmax)) return DSCell{~0u, ~0u};  // (NaN too)
    const float fx = (dot(p, mk(g.e1[0], g.e1[1], g.e1[2])) - g.u0) * g.su;
    const float fy = (dot(p, mk(g.e2[0], g.e2[1], g.e2[2])) - g.v0) * g.sv;
    DSCell c{g.always, g.always_root};
    if (fx >= 0.0f && fx < (float)G && fy >= 0.0f && fy < (float)G) {
        const DSCell q = S.dsg_cells[g.off + (int32_t)fy * G + (int32_t)fx];
        c.obj |= q.obj;
        c.root |= q.root;
    }
    return c;
}

#ifndef RTX_PLANE_SHADOW_RCP
#define RTX_PLANE_SHADOW_RCP 1
#endif
// Any order gives the same answer; cheap objects first, and the wave leaves as soon as
// every active lane is occluded. `light` >= 0: the ray goes to point light `light` (its
// light grid, if any, may stand in for the mesh's BVH walk).
template <bool MESH, bool X, bool COUNT>
RTX_HD bool occluded(const SceneView& S, f3 o, f3 d, double t_max, float time, Tally& tl, const HStack& hs,
                     const OriginTerms* ot = nullptr, int light = -1, int32_t self_obj = -1) {
    const float tmax32 = (float)t_max;
    // the floats around t_max (both tmax32 for the shader's 1.0 and inf)
    const float tmax_dn = (double)tmax32 > t_max ? nextafterf(tmax32, -INFINITY) : tmax32;
    const float tmax_up = (double)tmax32 < t_max ? nextafterf(tmax32, INFINITY) : tmax32;
    const float tmax_lim = nextafterf(tmax_dn, -INFINITY);  // a float strictly below t_max
    bool occ = false;
    int oi = 0;
    // self tests of planes (SceneView::plane_self) for a lane that hit plane self_obj
    cptr<float> pself = nullptr;
    float pm = INFINITY;
    if (light >= 0 && S.plane_self != nullptr && RTX_NPLANE(S) > 0) {  // (wave-uniform)
        pself = S.plane_self + 4 * light;
        pm = fmaxf(fabsf(o.x), fmaxf(fabsf(o.y), fabsf(o.z)));
    }
    for (int k = 0; k < RTX_NPLANE(S); ++k, ++oi) {  // simple_geometry.py:122-131
        if (RTX_PROBE(21)) continue;  // cost probe: planes never occlude
        // a camera hit on this plane, close enough to the origin: its own test cannot pass
        if (pself != nullptr && k < 4 && RTX_ALL(occ || (oi == self_obj && pm <= pself[k]))) continue;
        const DObj ob = S.objs[oi];
        const f3 n = ld3(ob.b);
        const float denom = dot(d, n);
#ifdef RTX_FIXED_COUNTS
        const float num = ot ? ot->pnum[k] : dot(sub(moved(ob, ob.a, time), o), n);
#else
        const float num = dot(sub(moved(ob, ob.a, time), o), n);
#endif
#if RTX_PLANE_SHADOW_RCP
        // num * v_rcp(denom) is within 2^-21 of num / denom: far from both thresholds it
        // decides alone, the correctly rounded quotient only near them (experiment)
        bool hit = false;
        if (fabsf(denom) >= kEps4Up) {
            const float ta = num * rcp_approx(denom), lo = ta * (1.0f - 0x1p-19f), hi = ta * (1.0f + 0x1p-19f);
            const float tlo = fminf(lo, hi), thi = fmaxf(lo, hi);
            // q > tlo >= kEps4Up > 1e-4; q < thi < fl32(1e-4) < 1e-4; q < thi < tmax_lim <
            // t_max keeps fl64(q) < t_max; q > tlo >= tmax_up >= t_max; an infinite t_max
            // holds every finite quotient (|denom| >= 1e-4)
            const int above = tlo >= kEps4Up ? 1 : (thi < kEps4Near ? 0 : -1);
            const int below = tmax_dn == INFINITY ? (fabsf(num) < INFINITY ? 1 : -1)
                              : (thi < tmax_lim ? 1 : (tlo >= tmax_up && tlo < INFINITY ? 0 : -1));
            if (above >= 0 && below >= 0) {
                hit = above == 1 && below == 1;
            } else {
                unspeculated();  // (the correctly rounded quotient only near a threshold)
                const float t32 = num / denom;
                hit = quot_gt(t32, num, denom, 1e-4, kEps4Near) && quot_lt(t32, num, denom, t_max, tmax32);
            }
        }
#else
        const float t32 = num / denom;
        const bool hit = fabsf(denom) >= kEps4Up && quot_gt(t32, num, denom, 1e-4, kEps4Near) &&
                         quot_lt(t32, num, denom, t_max, tmax32);
#endif
        occ = occ || hit;
    }
    if (RTX_ALL(occ)) return true;
    // the spheres and boxes this lane's ray may meet: a directional light's shadow grid
    DSCell sc{~0u, ~0u};
    uint32_t self_boxes = 0u;  // (self_obj: the flat object a camera ray hit at o, or -1)
#if !(defined(RTX_DIR_GRIDS) && !RTX_DIR_GRIDS)
    if (light >= 0 && S.dsg_on) {
        sc = dir_shadow_mask(S, light, o);
        self_boxes = S.dsgrid[light].self_boxes;
    }
#endif
    const uint32_t smask = sc.obj;
    for (int k = 0; k < RTX_NSPHERE(S); ++k, ++oi) {  // simple_geometry.py:48-72 (shadow_epsilon 1e-3)
        if (RTX_PROBE(19)) continue;  // cost probe: spheres never occlude
        const bool sl = ((smask >> (k & 15)) & 1u) != 0u;
        if (!RTX_ANY(sl && !occ)) continue;
        const DObj ob = S.objs[oi];
        const f3 ctr = moved(ob, ob.a, time);
#ifdef RTX_FIXED_COUNTS
        const f3 oc = ot ? ot->soc[k] : sub(o, ctr);
        const float q = ot ? ot->sq[k] : dot(oc, oc);
#else
        const f3 oc = sub(o, ctr);
        const float q = dot(oc, oc);
#endif
        int dec = -1;
        if (RTX_SHADOW_F32 && !RTX_PROBE(4)) {
            dec = sphere_shadow_f32(d, oc, q, ob.r2f, tmax_dn, tmax_up);
            if (!occ && sl && dec >= 0) occ = dec == 1;
        }
        if (!occ && sl && dec < 0 && sphere_disc_sign_oc(d, oc, q, ob.r2f) >= 0) {
            double b, s, two_a;
            if (RTX_PROBE(4) ? sphere_roots(o, d, ctr, ob.r2, b, s, two_a)
                                : sphere_roots_oc(d, oc, q, ob.r2, b, s, two_a)) {
                const double t1 = (-b - s) / two_a;
                bool hit = 1e-3 < t1 && t1 < t_max;
                if (RTX_ANY(!hit)) {  // the second root only where some lane needs it
                    unspeculated();
                    if (!hit) {
                        const double t2 = (-b + s) / two_a;
                        hit = 1e-3 < t2 && t2 < t_max;
                    }
                }
                occ = hit;
            }
        }
    }
    if (RTX_ALL(occ)) return true;
    RayInv ri{};
    // the reciprocals once some lane's ray may meet a box (meshes: once a lane passes a
    // bounding volume)
    bool have_ri = false;
    if (RTX_NBOX(S) > 0 && RTX_ANY(!occ && (smask >> 16) != 0u)) {
        ri = ray_inv(o, d);
        have_ri = true;
    }
    for (int k = 0; k < RTX_NBOX(S); ++k, ++oi) {  // simple_geometry.py:251-294
        if (RTX_PROBE(20)) continue;  // cost probe: boxes never occlude
        const bool sl = ((smask >> (16 + (k & 15))) & 1u) != 0u && !(oi == self_obj && k < 16 && ((self_boxes >> (16 + k)) & 1u));
        if (!RTX_ANY(sl && !occ)) continue;
        const DObj ob = S.objs[oi];
        const f3 mn = moved(ob, ob.a, time), mx = moved(ob, ob.b, time);
        if (RTX_BOX_IV_CULL) {
            if (RTX_ALL(occ)) break;
            const SlabIv iv = box_slabs_iv(o, d, mn, mx, &ri);
            const bool maybe = !occ && sl && !box_iv_out(iv, INFINITY);
            if (!RTX_ANY(maybe)) continue;
            if (maybe) occ = box_shadow_iv(o, d, mn, mx, iv, t_max);
        } else {
            const bool maybe = !occ && sl && box_maybe_hit_obj(ob, mn, mx, o, ri, INFINITY);
            if (!RTX_ANY(maybe)) continue;
            if (maybe) occ = box_shadow(o, d, mn, mx, t_max, &ri);
        }
    }
    if (MESH) {
        for (int k = 0; k < RTX_NMESH(S); ++k, ++oi) {  // mesh.py:121-153 (no t_max test)
            const DObj ob = S.objs[oi];
            if (RTX_ALL(occ) || RTX_PROBE(16)) break;  // 16: cost probe, meshes never occlude
            if (!have_ri) {
                ri = ray_inv(o, d);
                have_ri = true;
            }
            bool live = !occ && bv_maybe(ob, o, ri, INFINITY);  // conservative pre-test
            if (!RTX_ANY(live)) continue;
            if (RTX_PROBE(13)) continue;  // cost probe: the padded box pre-test only
            live = live && mesh_bv(ob, o, d);
            if (!RTX_ANY(live) || RTX_PROBE(12)) continue;  // 12: cost probe, bounding volumes only
            // mesh.py:125-151 for stored face f (lanes with maybe set may take it)
            auto shadow_face = [&](int f, bool maybe) {
                bool fmaybe = maybe;
                if (face_cull(ob)) {
                    fmaybe = maybe && leaf_maybe_hit(RTX_FBOX(S, ob.tri_begin + f), o, ri, ob.cmax);
                    if (!RTX_ANY(fmaybe)) return;
                }
                tally_inc<COUNT>(tl, &Tally::tri);
                occ = occ || (fmaybe && shadow_tri(RTX_TRI(S, ob.tri_begin + f), o, d));
            };
#if !(defined(RTX_LIGHT_GRIDS) && !RTX_LIGHT_GRIDS)
            if (light >= 0 && k == 0 && S.lgrid_on) {
                cref<DLGrid> g = S.lgrid[light];
                if (g.G > 0) {
                    // lanes with a cell test only its faces, one distinct cell of the wave at
                    // a time (the faces' loads stay wave-uniform); -1: nothing to test
                    const int32_t cell = lgrid_cell(g, d);
                    bool todo = live && cell >= 0;
                    live = live && cell == -2;
#if RTX_LGRID_LANE
                    // each lane runs its own cell's list (per-lane loads of the faces)
                    if (todo && !occ) {
                        const int32_t q1 = S.lg_start[g.start_off + cell + 1];
                        const f3 w = neg(d);
                        // the mesh side of the light: faces farther along a than |w| are out
                        const float wcap = dot(w, ld3(g.a)) > 0.0f ? dot(w, w) : INFINITY;
#if RTX_LGRID_PAIRS
                        // two faces per step (their loads and tests overlap): any face before
                        // the cut that the ray meets occludes, in whatever order they are tested
                        for (int32_t q = S.lg_start[g.start_off + cell]; q < q1; q += 2) {
                            const bool two = q + 1 < q1;
                            const float da = S.lg_d2[q], db = two ? S.lg_d2[q + 1] : INFINITY;
                            if (da > wcap) break;
                            const int32_t fa = S.lg_faces[q], fb = S.lg_faces[two ? q + 1 : q];
                            const DTri Ta = S.tris[ob.tri_begin + fa], Tb = S.tris[ob.tri_begin + fb];
                            const bool ha = shadow_tri(Ta, o, d);
                            const bool hb = shadow_tri(Tb, o, d) && db <= wcap;
                            tally_inc<COUNT>(tl, &Tally::tri);
                            if (db <= wcap) tally_inc<COUNT>(tl, &Tally::tri);
                            if (ha || hb) { occ = true; break; }
                            if (db > wcap) break;
                        }
#else
                        for (int32_t q = S.lg_start[g.start_off + cell]; q < q1; ++q) {
                            if (S.lg_d2[q] > wcap) break;
                            tally_inc<COUNT>(tl, &Tally::tri);
                            if (shadow_tri(S.tris[ob.tri_begin + S.lg_faces[q]], o, d)) { occ = true; break; }
                        }
#endif
                    }
                    todo = false;
#endif
                    while (RTX_ANY(todo)) {
                        const int32_t c = first_where(cell, todo);
                        const bool mine = todo && cell == c;
                        if (mine) {
                            const int32_t q1 = S.lg_start[g.start_off + c + 1];
                            for (int32_t q = S.lg_start[g.start_off + c]; q < q1; ++q) {
                                if (RTX_ALL(occ)) break;
                                shadow_face(S.lg_faces[q], !occ);
                            }
                        }
                        todo = todo && !mine;
                    }
                    if (!RTX_ANY(live)) continue;
                }
            }
#endif
            for (int li = 0; li < ob.leaf_count;) {  // stackless wave-uniform BVH walk
              const auto& L = RTX_LEAF(S, ob.leaf_begin + li);
              const bool maybe = live && !occ && leaf_maybe_hit(L, o, ri, ob.cmax);
              if (!RTX_ANY(maybe)) { li = L.skip; continue; }
              ++li;
              for (int f = L.first; f < L.first + L.count; ++f) shadow_face(f, maybe);
            }
        }
    }
    if (X && !RTX_PROBE(10)) occ = hier_occluded<MESH>(S, hs, o, d, t_max, time, occ, sc.root);  // hierarchy.py:80-109
    return occ;
}

// The shadow rays of every light at once, for scene-specialized kernels of flat scenes of
// planes and spheres whose lights are all point lights (RTX_LIGHTS_TOGETHER): objects in
// the outer loop, lights in the inner one, so the lights' tests of one object are
// independent chains of one block instead of one light's whole occluded() after another.
// Every light's test is occluded()'s, operation for operation (t_max = 1: a point light,
// scene.py:155-158); returns bit li = light li's ray is occluded.
#if defined(RTX_FIXED_COUNTS) && !defined(RTX_LIGHTS_TOGETHER)
#define RTX_LIGHTS_TOGETHER (RTX_FIXED_NB == 0 && RTX_FIXED_NM == 0 && RTX_FIXED_LDIR == 0u && RTX_FIXED_NL >= 2 && \
                             RTX_FIXED_NL <= 8 && RTX_PLANE_SHADOW_RCP && !RTX_SHADOW_F32)
#endif
#if defined(RTX_LIGHTS_TOGETHER) && RTX_LIGHTS_TOGETHER
RTX_HD uint32_t occluded_points(const SceneView& S, f3 o, const f3* sd, const OriginTerms& ot, int32_t self_obj) {
    constexpr int NL = RTX_FIXED_NL;
    const double t_max = 1.0;
    const float tmax32 = 1.0f, tmax_up = 1.0f, tmax_lim = nextafterf(1.0f, -INFINITY);
    bool occ[NL];
#pragma unroll
    for (int li = 0; li < NL; ++li) occ[li] = false;
    int oi = 0;
    const float pm = fmaxf(fabsf(o.x), fmaxf(fabsf(o.y), fabsf(o.z)));
    for (int k = 0; k < RTX_NPLANE(S); ++k, ++oi) {  // simple_geometry.py:122-131
        // a camera hit on this plane, close enough to the origin: its own test cannot pass
        bool skip[NL];
        bool all_skip = true;
#pragma unroll
        for (int li = 0; li < NL; ++li) {
            skip[li] = S.plane_self != nullptr && k < 4 &&
                       RTX_ALL(occ[li] || (oi == self_obj && pm <= S.plane_self[4 * li + k]));
            all_skip = all_skip && skip[li];
        }
        if (all_skip) continue;
        const DObj ob = S.objs[oi];
        const f3 n = ld3(ob.b);
        const float num = ot.pnum[k];
        float den[NL];
        bool hit[NL], slow[NL];
        bool any_slow = false;
#pragma unroll
        for (int li = 0; li < NL; ++li) {  // occluded()'s quotient filter (RTX_PLANE_SHADOW_RCP)
            den[li] = dot(sd[li], n);
            hit[li] = slow[li] = false;
            if (fabsf(den[li]) >= kEps4Up) {
                const float ta = num * rcp_approx(den[li]), lo = ta * (1.0f - 0x1p-19f), hi = ta * (1.0f + 0x1p-19f);
                const float tlo = fminf(lo, hi), thi = fmaxf(lo, hi);
                const int above = tlo >= kEps4Up ? 1 : (thi < kEps4Near ? 0 : -1);
                const int below = thi < tmax_lim ? 1 : (tlo >= tmax_up && tlo < INFINITY ? 0 : -1);
                if (above >= 0 && below >= 0) hit[li] = above == 1 && below == 1;
                else slow[li] = !skip[li];
            }
            any_slow = any_slow || slow[li];
        }
        if (RTX_ANY(any_slow)) {
            unspeculated();  // (the correctly rounded quotient only near a threshold)
#pragma unroll
            for (int li = 0; li < NL; ++li)
                if (slow[li]) {
                    const float t32 = num / den[li];
                    hit[li] = quot_gt(t32, num, den[li], 1e-4, kEps4Near) && quot_lt(t32, num, den[li], t_max, tmax32);
                }
        }
#pragma unroll
        for (int li = 0; li < NL; ++li) occ[li] = occ[li] || (!skip[li] && hit[li]);
    }
    for (int k = 0; k < RTX_NSPHERE(S); ++k, ++oi) {  // simple_geometry.py:48-72 (shadow_epsilon 1e-3)
        bool need[NL];
        bool any_need = false;
        const DObj ob = S.objs[oi];
#pragma unroll
        for (int li = 0; li < NL; ++li) {
            need[li] = !occ[li] && sphere_disc_sign_oc(sd[li], ot.soc[k], ot.sq[k], ob.r2f) >= 0;
            any_need = any_need || need[li];
        }
        if (!RTX_ANY(any_need)) continue;
        double b[NL], sq[NL], two_a[NL];
        bool roots[NL], hit[NL];
        bool any_far = false;
#pragma unroll
        for (int li = 0; li < NL; ++li) {
            roots[li] = need[li] && sphere_roots_oc(sd[li], ot.soc[k], ot.sq[k], ob.r2, b[li], sq[li], two_a[li]);
            hit[li] = false;
            if (roots[li]) {
                const double t1 = (-b[li] - sq[li]) / two_a[li];
                hit[li] = 1e-3 < t1 && t1 < t_max;
            }
            any_far = any_far || (roots[li] && !hit[li]);
        }
        if (RTX_ANY(any_far)) {  // the second root only where some lane needs it
            unspeculated();
#pragma unroll
            for (int li = 0; li < NL; ++li)
                if (roots[li] && !hit[li]) {
                    const double t2 = (-b[li] + sq[li]) / two_a[li];
                    hit[li] = 1e-3 < t2 && t2 < t_max;
                }
        }
#pragma unroll
        for (int li = 0; li < NL; ++li) occ[li] = occ[li] || (roots[li] && hit[li]);
    }
    uint32_t m = 0u;
#pragma unroll
    for (int li = 0; li < NL; ++li) m |= occ[li] ? 1u << li : 0u;
    return m;
}
#endif

struct Surface {
    f3 position, normal;
    int32_t mat;
    int32_t gobj;  // DObj whose get_diffuse shades the hit (textured or hierarchy Plane/AABB), or -1
};

template <bool MESH, bool X>
RTX_HD Surface resolve_hit(const SceneView& S, const Hit& h, const HHit& hh, f3 o, f3 d, float time) {
    Surface sf;
    if (X && h.obj == kHierHit) {
        sf.position = hh.pos;
        sf.normal = hh.n;
        sf.mat = hh.mat;
        sf.gobj = hh.gobj;
        return sf;
    }
    const DObj ob = RTX_OBJ(S, h.obj);
    sf.gobj = (X && ob.has_tex) ? h.obj : -1;
    sf.position = add(o, scale(d, h.t32));  // getPoint(t): fl32(t64) == t32
    sf.mat = ob.mat0;
    const int32_t type = ob.type;
    if (type == OBJ_SPHERE) {
        sf.normal = normalize(sub(sf.position, moved(ob, ob.a, time)));
    } else if (type == OBJ_PLANE) {
        sf.normal = ld3(ob.b);
        sf.mat = plane_material(ob, sf.position, time);
    } else if (type == OBJ_BOX) {
        sf.normal = box_normal(h.sub, d);  // entry-slab label and the direction's sign
    } else if (MESH) {
        const DTri T = S.tris[ob.tri_begin + h.sub];
        if (ob.flat)
            sf.normal = ld3(T.n);
        else
            sf.normal = smooth_normal(T, (DTriN)S.trins[ob.tri_begin + h.sub], sf.position);
    }
    return sf;
}

// ------------------------------------------------------------------ shading
// General fp64 pow for non-integer exponents, kept out of line: the inlined libm path
// would raise the kernel's register allocation (occupancy) for a case the reference
// scenes never use.
__host__ __device__ __attribute__((noinline)) inline double pow_general(double x, double y) { return pow(x, y); }

// x ** n for an integer n >= 0 in double-double arithmetic (Dekker products through fma,
// relative error below 2^-98 for n < 2^16), rounded once to fp64: fl64 of the exact power,
// which is what a correctly rounded libm pow returns. The rare path of spec_pow.
RTX_HD void dd_mul(double& ah, double& al, double bh, double bl) {
    const double p = ah * bh;
    double e = __builtin_fma(ah, bh, -p);  // exact: ah * bh = p + e
    e = e + (ah * bl + al * bh);
    const double s = p + e;
    al = e - (s - p);
    ah = s;
}
__host__ __device__ __attribute__((noinline)) inline double pow_int_dd(double x, int n) {
    double rh = 1.0, rl = 0.0, bh = x, bl = 0.0;
    while (n) {
        if (n & 1) dd_mul(rh, rl, bh, bl);
        n >>= 1;
        if (n) dd_mul(bh, bl, bh, bl);
    }
    return rh + rl;
}

// `x ** hardness` (CPython float_pow -> libm pow) in fp64, cast to fp32 by the caller.
// Integer exponents use binary exponentiation: at most 2 * pow_bits roundings, so the
// result is within 2^-48 (relative; hardness <= 4096, so pow_bits <= 13) of the exact power. Its fp32 cast
// therefore equals that of libm's correctly rounded pow unless the exact value lies that
// close to an fp32 rounding boundary: r * (1 -/+ 2^-47) then round to different floats,
// and only those lanes (about 2^-22 of the evaluations; tests/test_pow.py finds 2 of
// 1.29e8 that the fast value would get wrong) recompute the power in double-double. The
// loop runs a scene-uniform number of steps (bits of the largest integer hardness) with
// selects, so lanes shading different materials do not diverge; each lane performs
// exactly the multiplications of `while (n) { if (n & 1) r *= b; b *= b; n >>= 1; }`.
RTX_HD double spec_pow(double x, const DMat& m, int pow_bits) {
    if (RTX_PROBE(5)) return (double)__builtin_powf((float)x, (float)m.hardness);  // cost probe only
#ifdef RTX_FIXED_HARD  // scene-specialized: every specular lobe has this integer hardness
    if (true) {
        const int n = RTX_FIXED_HARD;
#else
    if (m.hard_is_int) {
        const int n = m.hard_int;
#endif
        double r = 1.0, b = x;
        for (int k = 0; k < pow_bits; ++k) {
#if defined(__HIP_DEVICE_COMPILE__)
            if (!RTX_ANY(n >> k)) break;  // wave-uniform exit once no lane has bits left
#endif
            const double rb = r * b;
            r = ((n >> k) & 1) ? rb : r;
            b = b * b;
        }
        // fp32 rounding boundary within the error bound: the double-double power decides
        const bool near = (float)(r * (1.0 - 0x1p-47)) != (float)(r * (1.0 + 0x1p-47));
        if (RTX_ANY(near)) {
            unspeculated();
            if (near) r = pow_int_dd(x, n);
        }
        return r;
    }
    return pow_general(x, m.hardness);
}

// _compute_regular_lighting (scene.py:140-187)
// occ_mask >= 0 (the split hierarchy passes, rtx_split.h): bit li says whether light li's
// shadow ray is occluded, as a separate pass found it; no shadow ray is traced here.
template <bool MESH, bool X, bool COUNT>
RTX_HD f3 regular_lighting(const SceneView& S, f3 dir, f3 pos, f3 normal, const DMat& m, f3 diffuse, float time,
                           Tally& tl, const HStack& hs, int64_t occ_mask = -1, int32_t self_obj = -1) {
    f3 colour = mk(0.0f, 0.0f, 0.0f);
    tally_inc<COUNT>(tl, &Tally::shade);
    OriginTerms ot;
    origin_terms(S, pos, time, ot);
#ifdef RTX_FIXED_COUNTS
    const OriginTerms* otp = RTX_NLIGHTS(S) > 1 ? &ot : nullptr;
#else
    const OriginTerms* otp = nullptr;
#endif
#if defined(RTX_LIGHTS_TOGETHER) && RTX_LIGHTS_TOGETHER
    if (!MESH && !X && occ_mask < 0 && !RTX_PROBE(1)) {  // every light's shadow ray at once
        f3 sd[RTX_FIXED_NL];
#pragma unroll
        for (int li = 0; li < RTX_FIXED_NL; ++li) sd[li] = sub(ld3(S.lights[li].vec), pos);
        occ_mask = (int64_t)occluded_points(S, pos, sd, ot, self_obj);
    }
#endif
    for (int li = 0; li < RTX_NLIGHTS(S); ++li) {
        const DLight L = S.lights[li];
#ifdef RTX_FIXED_LDIR  // scene-specialized: bit li set = directional
        const bool point = ((RTX_FIXED_LDIR >> li) & 1u) == 0u;
#else
        const bool point = L.type == LIGHT_POINT;
#endif
        f3 sdir;
        double t_max;
        if (point) {
            sdir = sub(ld3(L.vec), pos);
            t_max = 1.0;
        } else {
            sdir = ld3(L.negvec);
            t_max = INFINITY;
        }
        tally_inc<COUNT>(tl, &Tally::shadow);
        if (occ_mask >= 0) {
            if ((occ_mask >> li) & 1) continue;
        } else if (!RTX_PROBE(1) && occluded<MESH, X, COUNT>(S, pos, sdir, t_max, time, tl, hs, otp, li, self_obj)) {
            continue;
        }
        if (RTX_PROBE(3)) { colour = add(colour, mul(ld3(L.cp), diffuse)); continue; }
        f3 light_dir = point ? normalize(sdir) : ld3(L.ndir);
        f3 lambert = scale(diffuse, pos_part(dot(normal, light_dir)));
        f3 ls = lambert;
        if (!m.spec_zero) {
            f3 half_vect = normalize(sub(light_dir, dir));
            float nh = dot(normal, half_vect);
            double base = nh > 0.0f ? (double)nh : 0.0;
#ifdef RTX_FIXED_POWBITS
            f3 specular = scale(ld3(m.specular), (float)spec_pow(base, m, RTX_FIXED_POWBITS));
#else
            f3 specular = scale(ld3(m.specular), (float)spec_pow(base, m, S.pow_bits));
#endif
            ls = add(lambert, specular);
        }
        // spec_zero: specular == +0 and diffuse >= +0, so lambert + specular == lambert exactly
        colour = add(colour, mul(ld3(L.cp), ls));
    }
    colour = add(colour, mul(ld3(S.ambient), diffuse));
    return colour;
}

// ------------------------------------------------------------------ cast_ray, iteratively
// scene.py:81-116 + _compute_refraction (:189-209). Secondary rays form a chain (one
// reflect or refract child per level), so the recursion becomes a loop that records one
// frame (lighting RGB, material) per mirror/refractive level and unwinds bottom-up with
// the per-level clamp: colour = clamp(L * tint + child * (1 - tint)). Frames live in a
// caller-provided store: LDS on the device ([frame][word][thread], conflict-free), a
// local array in the host emulation.
// RTX_FRAME_MATBITS > 0 (scene-specialized kernels of scenes with at most
// 2^RTX_FRAME_MATBITS materials): a frame's material index lives in a register instead,
// RTX_FRAME_MATBITS bits per level of one 64-bit word, and LDS holds 3 words per frame --
// 30 instead of 40 KB per 256-thread block, so 5 blocks (20 waves) fit a CU's 160 KB
// instead of 4.
#ifndef RTX_FRAME_MATBITS
#define RTX_FRAME_MATBITS 0
#endif
static_assert(RTX_FRAME_MATBITS * kMaxDepth <= 64, "frame materials must fit one 64-bit word");
constexpr int kFrameWords = RTX_FRAME_MATBITS ? 3 : 4;
// Frames kept in LDS; deeper levels of a chain (rare) go to a per-lane private array
// (scratch), so a smaller LDS stack lets more blocks share a CU. The scene-specialized
// kernels of flat scenes with secondary rays keep 6 levels in LDS (rtx_api.hip jit_spec:
// MirrorRefraction 38.7 -> 36.4 us); the precompiled kernels keep every level.
#ifndef RTX_FRAME_LDS_LEVELS
#define RTX_FRAME_LDS_LEVELS kMaxDepth
#endif
constexpr int kFrameLds = RTX_FRAME_LDS_LEVELS;
static_assert(kFrameLds >= 1 && kFrameLds <= kMaxDepth, "RTX_FRAME_LDS_LEVELS out of range");
struct FrameStack {
    float* base;
    int stride;
    RTX_HD void put(int k, f3 L, int32_t mat) const {
        float* p = base + k * kFrameWords * stride;
        p[0] = L.x;
        p[stride] = L.y;
        p[2 * stride] = L.z;
        if (!RTX_FRAME_MATBITS) p[3 * stride] = __builtin_bit_cast(float, mat);
    }
    RTX_HD f3 get(int k, int32_t& mat) const {
        const float* p = base + k * kFrameWords * stride;
        if (!RTX_FRAME_MATBITS) mat = __builtin_bit_cast(int32_t, p[3 * stride]);
        return f3{p[0], p[stride], p[2 * stride]};
    }
};

template <bool MESH, bool SEC, bool X, bool COUNT>
RTX_HD f3 cast_ray(const SceneView& S, f3 o, f3 d, float time, Tally& tl, const FrameStack& fs, const HStack& hs,
                   int32_t bin = -1, const OriginTerms* prim = nullptr, int32_t blane = -1) {
    int nfr = 0;
    uint64_t fmats = 0;  // RTX_FRAME_MATBITS: the frames' material indices
    f3 deep[kMaxDepth - kFrameLds > 0 ? kMaxDepth - kFrameLds : 1];  // frames kFrameLds.. (private)
    int32_t deep_mat[kMaxDepth - kFrameLds > 0 ? kMaxDepth - kFrameLds : 1];
    f3 tail = mk(0.0f, 0.0f, 0.0f);
    bool in_shape = false;
    for (int level = 0; level < (SEC ? kMaxDepth : 1); ++level) {
        if (COUNT) tl.cast[level]++;
        if (RTX_PROBE(8)) { tail = d; break; }  // cost probe: camera + store only
        HHit hh;
        const Hit h = closest_hit<MESH, X, COUNT>(S, o, d, time, tl, hs, hh, level == 0 ? bin : -1,
                                                  level == 0 ? prim : nullptr, blane);
        if (h.obj == -1) break;  // miss -> black
        const Surface sf = resolve_hit<MESH, X>(S, h, hh, o, d, time);
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
            tir = is_zero(rdir);  // total internal reflection -> black child
            next_o = add(sf.position, scale(rdir, 0.0001f));
            next_d = rdir;
            chain = true;
        }
        if ((RTX_PROBE(2) || RTX_PROBE(7)) && !chain) { tail = ld3(m.diffuse); break; }
        // scene.py:143-146: Plane/AABB hits shade with get_diffuse(position)
        const f3 diffuse = (X && sf.gobj >= 0) ? get_diffuse(S, S.objs[sf.gobj], sf.position, time) : ld3(m.diffuse);
        // a camera ray's hit (level 0) tells occluded which flat object it lies on
        const f3 L = regular_lighting<MESH, X, COUNT>(S, d, sf.position, n, m, diffuse, time, tl, hs, -1,
                                                      level == 0 ? h.obj : -1);
        if (!SEC || !chain) {
            tail = clamp01(L);
            break;
        }
        if (kFrameLds == kMaxDepth || nfr < kFrameLds) {
            fs.put(nfr, L, sf.mat);
        } else {
            deep[nfr - kFrameLds] = L;
            deep_mat[nfr - kFrameLds] = sf.mat;
        }
        if (RTX_FRAME_MATBITS) fmats |= (uint64_t)(uint32_t)sf.mat << (nfr * RTX_FRAME_MATBITS);
        ++nfr;
        if (tir) break;
        in_shape = m.type == MAT_REFRACTIVE ? !in_shape : false;
        o = next_o;
        d = next_d;
    }
    if (SEC) {
        for (int k = nfr - 1; k >= 0; --k) {
            int32_t mi;
            f3 L;
            if (kFrameLds == kMaxDepth || k < kFrameLds) {
                L = fs.get(k, mi);
            } else {
                L = deep[k - kFrameLds];
                mi = deep_mat[k - kFrameLds];
            }
            if (RTX_FRAME_MATBITS)
                mi = (int32_t)((fmats >> (k * RTX_FRAME_MATBITS)) & ((1ull << (RTX_FRAME_MATBITS % 64)) - 1));
            const DMat m = RTX_MAT(S, mi);
            tail = clamp01(add(scale(L, m.tint), scale(tail, m.omt)));
        }
    }
    return tail;
}

// ------------------------------------------------------------------ Philox4x32-10
RTX_HD void philox4x32(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

}  // namespace rtx
