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
//   k_to_rgb8     (v * 255.0) truncated to uint8 (main.py:33)
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <dirent.h>
#include <fstream>
#include <functional>
#include <future>
#include <list>
#include <map>
#include <numeric>
#include <mutex>
#include <sstream>
#include <string>
#include <sys/stat.h>
#include <unistd.h>
#include <vector>

#include "../../include/rtx.h"
#include "rtx_kernels.h"
#include "rtx_bins.h"
#include "rtx_launch.h"
#include "rtx_split.h"

// faces per mesh BVH leaf (cluster); meshes of at most kFaceCullMaxFaces faces also
// test each face's box before its exact test (DObj::face_cull)
#ifndef RTX_LEAF_FACES
#define RTX_LEAF_FACES 8
#endif
#ifndef RTX_FACE_CULL_MAX
#define RTX_FACE_CULL_MAX 4096
#endif
constexpr int32_t kFaceCullMaxFaces = RTX_FACE_CULL_MAX;

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

// ------------------------------------------------------------------ library options
// Process-wide switches of librtx.so (rtx_set_option / rtx_get_option; INTEGRATION.md
// "Options"): each starts from $RTX_<NAME> when that is set, else from its default, and is
// read where the library decides (per render or per camera upload). Set them before
// rendering; they are not synchronised with renders running on other threads.
enum Opt {
    OPT_SPLIT, OPT_SPLIT_BYTES, OPT_SPLIT_RATIO, OPT_BINS, OPT_HEAVY_TILES, OPT_LENS_BINS, OPT_LGRID, OPT_DSGRID, OPT_DSGRID_MIN,
    OPT_SELF_SKIP, OPT_TILE_SCHED, OPT_XCD_MAP, OPT_TILE_BLOCK, OPT_PRIM_ORIGIN, OPT_SPP, OPT_SPP_MIN, OPT_JIT, OPT_JIT_BAKE, OPT_JIT_EXT,
    OPT_JIT_DUMP, OPT_JIT_IDLE_BAKED, OPT_JIT_DISK_BAKED, OPT_JIT_CACHE, OPT_JIT_FLAGS, OPT_JIT_ILP, OPT_JIT_ASYNC,
    OPT_DEV_BINS, OPT_CHUNK_MODE, OPT_BIN_LDS, OPT_JIT_CSG, OPT_CSG_RAYS, OPT_CSG_SHADE, OPT_SETUP_LOG, OPT_COUNT
};
struct OptDef {
    const char* name;
    double dflt;
    bool str;  // a string value (kept in OptVal::s)
};
constexpr OptDef kOpts[OPT_COUNT] = {
    {"split", 1, false},                      // hierarchy/texture scenes in three passes (0: one kernel)
    {"split_bytes", 2147483648.0, false},     // record bytes of one split chunk
    {"split_ratio", -1, false},               // >= 0: fixed deeper records per sample (else learned)
    {"bins", 1, false},                       // primary-ray bins (0: every primary ray walks everything)
    {"heavy_tiles", 1, false},                // long bin face lists tested in chunks by a pass of their own
    {"lens_bins", 1, false},                  // bins for lens cameras too
    {"lgrid", 1, false},                      // light grids of point lights (mesh shadow rays)
    {"dsgrid", 1, false},                     // shadow grids of directional lights
    {"dsgrid_min", 8, false},                 // the fewest spheres (and nothing else) that get one
    {"self_skip", 1, false},                  // plane / box self tests skipped where provably passing
    {"tile_sched", 1, false},                 // measured longest-first tile order
    {"xcd_map", 0, false},                    // XCD-aware block order of tile-mapped launches
    {"tile_block", 64, false},                // threads per block of the secondary-ray / mesh tile kernels
    {"prim_origin", 1, false},                // host-computed origin terms of pinhole primary rays
    {"spp", -1, false},                       // sample-parallel mapping: -1 auto, 0 never, 1 always
    {"spp_min", 16, false},                   // auto: from this many samples per pixel (X scenes)
    {"jit", 1, false},                        // scene-specialized kernels (hiprtc)
    {"jit_bake", 1, false},                   // scene records as literals in one-sample kernels
    {"jit_ext", 0, false},                    // specialize hierarchy/texture kernels too
    {"jit_dump", 0, false},                   // print each specialized kernel's source and options
    {"jit_idle_baked", 8, false},             // idle baked kernel modules kept loaded
    {"jit_disk_baked", 64, false},            // baked code objects kept in the disk cache
    {"jit_cache", 0, true},                   // code-object cache directory ("" = /tmp/rtx_jit_<uid>)
    {"jit_flags", 0, true},                   // extra hiprtc options (part of the cache key)
    {"jit_ilp", 1, false},                    // max-ILP scheduling of one-sample primary+shadow kernels
    {"jit_async", 1, false},                  // compile on a host thread; the generic kernel renders meanwhile
    {"dev_bins", 1, false},                   // a mesh's primary-ray face bins built on the device
    {"chunk_mode", 3, false},                 // heavy-tile pass: bit 0 LDS-staged faces, bit 1 XCD-aware order
    {"bin_lds", 0, false},                    // primary-ray face lists staged in LDS (specialized mesh kernels)
    {"jit_csg", 1, false},                    // split hierarchy passes specialized on the CSG trees (2: + boxes, 3: + objects)
    {"csg_rays", 3, false},                   // their rays in registers (bit 0: trace, bit 1: shadow), else the LDS stack
    {"csg_shade", 0, false},                  // the shade pass compiled with them (measured no faster)
    {"setup_log", 0, false},                  // print the host time of each rtx_camera_set step
};
struct OptVal {
    double v;
    std::string s;
};
std::mutex g_opt_mu;
OptVal* opt_table() {
    static OptVal* t = [] {
        static OptVal vals[OPT_COUNT];
        for (int i = 0; i < OPT_COUNT; ++i) {
            vals[i].v = kOpts[i].dflt;
            std::string env = "RTX_";
            for (const char* c = kOpts[i].name; *c; ++c) env += (char)toupper((unsigned char)*c);
            if (const char* e = getenv(env.c_str())) {
                if (kOpts[i].str) vals[i].s = e;
                else if (*e) vals[i].v = atof(e);
            }
        }
        return vals;
    }();
    return t;
}
double opt(Opt o) { return opt_table()[o].v; }
bool opt_on(Opt o) { return opt_table()[o].v != 0.0; }
std::string opt_str(Opt o) {
    std::lock_guard<std::mutex> lock(g_opt_mu);
    return opt_table()[o].s;
}

}  // namespace

// ------------------------------------------------------------------ host-side conversion
// rtx_*_desc (ABI) -> device records. Pure host code with no HIP calls, shared with the
// tests-only host emulation build (tests/native/rtx_hostemu.hip).
namespace {

void set3(float* dst, const float* s) { dst[0] = s[0]; dst[1] = s[1]; dst[2] = s[2]; dst[3] = 0.0f; }
void set3(float* dst, f3 s) { dst[0] = s.x; dst[1] = s.y; dst[2] = s.z; dst[3] = 0.0f; }
bool finite3(const float* v) { return std::isfinite(v[0]) && std::isfinite(v[1]) && std::isfinite(v[2]); }

// Hierarchy.make_matrices (hierarchy.py:30-40) with GLM's float mat4 code (PyGLM):
// translate, rotate about x, y, z (glm.radians of a Python float is fp64, the angle is
// then a float; cosf/sinf), scale, and the cofactor inverse. m[col * 4 + row].
struct Mat4 {
    float m[16];
};
Mat4 m4_identity() {
    Mat4 r{};
    r.m[0] = r.m[5] = r.m[10] = r.m[15] = 1.0f;
    return r;
}
Mat4 m4_translate(const Mat4& m, f3 v) {  // Result[3] = m[0] v0 + m[1] v1 + m[2] v2 + m[3]
    Mat4 r = m;
    for (int k = 0; k < 4; ++k) r.m[12 + k] = ((m.m[k] * v.x + m.m[4 + k] * v.y) + m.m[8 + k] * v.z) + m.m[12 + k];
    return r;
}
Mat4 m4_rotate(const Mat4& m, float angle, f3 v) {
    const float c = cosf(angle), s = sinf(angle);
    const f3 axis = normalize(v);
    const f3 temp = scale(axis, 1.0f - c);
    const float ax[3] = {axis.x, axis.y, axis.z}, tp[3] = {temp.x, temp.y, temp.z};
    float R[3][3];
    R[0][0] = c + tp[0] * ax[0];
    R[0][1] = tp[0] * ax[1] + s * ax[2];
    R[0][2] = tp[0] * ax[2] - s * ax[1];
    R[1][0] = tp[1] * ax[0] - s * ax[2];
    R[1][1] = c + tp[1] * ax[1];
    R[1][2] = tp[1] * ax[2] + s * ax[0];
    R[2][0] = tp[2] * ax[0] + s * ax[1];
    R[2][1] = tp[2] * ax[1] - s * ax[0];
    R[2][2] = c + tp[2] * ax[2];
    Mat4 r = m;
    for (int col = 0; col < 3; ++col)
        for (int k = 0; k < 4; ++k)
            r.m[4 * col + k] = (m.m[k] * R[col][0] + m.m[4 + k] * R[col][1]) + m.m[8 + k] * R[col][2];
    return r;
}
Mat4 m4_scale(const Mat4& m, f3 v) {
    Mat4 r = m;
    const float sv[3] = {v.x, v.y, v.z};
    for (int col = 0; col < 3; ++col)
        for (int k = 0; k < 4; ++k) r.m[4 * col + k] = m.m[4 * col + k] * sv[col];
    return r;
}
Mat4 m4_inverse(const Mat4& M) {  // glm compute_inverse<4, 4>
    auto m = [&](int c, int r) { return M.m[4 * c + r]; };
    const float C00 = m(2, 2) * m(3, 3) - m(3, 2) * m(2, 3), C02 = m(1, 2) * m(3, 3) - m(3, 2) * m(1, 3);
    const float C03 = m(1, 2) * m(2, 3) - m(2, 2) * m(1, 3), C04 = m(2, 1) * m(3, 3) - m(3, 1) * m(2, 3);
    const float C06 = m(1, 1) * m(3, 3) - m(3, 1) * m(1, 3), C07 = m(1, 1) * m(2, 3) - m(2, 1) * m(1, 3);
    const float C08 = m(2, 1) * m(3, 2) - m(3, 1) * m(2, 2), C10 = m(1, 1) * m(3, 2) - m(3, 1) * m(1, 2);
    const float C11 = m(1, 1) * m(2, 2) - m(2, 1) * m(1, 2), C12 = m(2, 0) * m(3, 3) - m(3, 0) * m(2, 3);
    const float C14 = m(1, 0) * m(3, 3) - m(3, 0) * m(1, 3), C15 = m(1, 0) * m(2, 3) - m(2, 0) * m(1, 3);
    const float C16 = m(2, 0) * m(3, 2) - m(3, 0) * m(2, 2), C18 = m(1, 0) * m(3, 2) - m(3, 0) * m(1, 2);
    const float C19 = m(1, 0) * m(2, 2) - m(2, 0) * m(1, 2), C20 = m(2, 0) * m(3, 1) - m(3, 0) * m(2, 1);
    const float C22 = m(1, 0) * m(3, 1) - m(3, 0) * m(1, 1), C23 = m(1, 0) * m(2, 1) - m(2, 0) * m(1, 1);
    const float F0[4] = {C00, C00, C02, C03}, F1[4] = {C04, C04, C06, C07}, F2[4] = {C08, C08, C10, C11};
    const float F3[4] = {C12, C12, C14, C15}, F4[4] = {C16, C16, C18, C19}, F5[4] = {C20, C20, C22, C23};
    const float V0[4] = {m(1, 0), m(0, 0), m(0, 0), m(0, 0)}, V1[4] = {m(1, 1), m(0, 1), m(0, 1), m(0, 1)};
    const float V2[4] = {m(1, 2), m(0, 2), m(0, 2), m(0, 2)}, V3[4] = {m(1, 3), m(0, 3), m(0, 3), m(0, 3)};
    const float SA[4] = {+1, -1, +1, -1}, SB[4] = {-1, +1, -1, +1};
    Mat4 inv;
    for (int k = 0; k < 4; ++k) {
        inv.m[k] = ((V1[k] * F0[k] - V2[k] * F1[k]) + V3[k] * F2[k]) * SA[k];
        inv.m[4 + k] = ((V0[k] * F0[k] - V2[k] * F3[k]) + V3[k] * F4[k]) * SB[k];
        inv.m[8 + k] = ((V0[k] * F1[k] - V1[k] * F3[k]) + V3[k] * F5[k]) * SA[k];
        inv.m[12 + k] = ((V0[k] * F2[k] - V1[k] * F4[k]) + V2[k] * F5[k]) * SB[k];
    }
    float dot0[4];
    for (int k = 0; k < 4; ++k) dot0[k] = M.m[k] * inv.m[4 * k];  // m[0] * Row0
    const float det = (dot0[0] + dot0[1]) + (dot0[2] + dot0[3]);
    const float one_over = 1.0f / det;
    for (int k = 0; k < 16; ++k) inv.m[k] = inv.m[k] * one_over;
    return inv;
}
void make_matrices(const float* trs, Mat4& M, Mat4& Minv) {
    const double k = 0.017453292519943295;  // glm::radians
    Mat4 m = m4_identity();
    m = m4_translate(m, ld3(trs));
    m = m4_rotate(m, (float)((double)trs[3] * k), mk(1, 0, 0));
    m = m4_rotate(m, (float)((double)trs[4] * k), mk(0, 1, 0));
    m = m4_rotate(m, (float)((double)trs[5] * k), mk(0, 0, 1));
    m = m4_scale(m, ld3(trs + 6));
    M = m;
    Minv = m4_inverse(m);
}

// ------------------------------------------------------------------ hierarchy bounds
// Conservative boxes per hierarchy node (DBound, rtx_trace.h), in double precision, for
// the motion-time range [tlo, thi]; each box is padded by 1e-4 of its coordinate scale,
// orders of magnitude above the fp32 rounding of the device's transforms and hit points.
struct HBox {
    double lo[3], hi[3];
};
HBox hb_all() { return HBox{{-INFINITY, -INFINITY, -INFINITY}, {INFINITY, INFINITY, INFINITY}}; }
HBox hb_none() { return HBox{{INFINITY, INFINITY, INFINITY}, {-INFINITY, -INFINITY, -INFINITY}}; }
bool hb_empty(const HBox& b) { return !(b.lo[0] <= b.hi[0] && b.lo[1] <= b.hi[1] && b.lo[2] <= b.hi[2]); }
bool hb_finite(const HBox& b) {
    for (int k = 0; k < 3; ++k)
        if (!std::isfinite(b.lo[k]) || !std::isfinite(b.hi[k])) return false;
    return true;
}
HBox hb_union(const HBox& a, const HBox& b) {
    if (hb_empty(a)) return b;
    if (hb_empty(b)) return a;
    HBox r;
    for (int k = 0; k < 3; ++k) { r.lo[k] = std::min(a.lo[k], b.lo[k]); r.hi[k] = std::max(a.hi[k], b.hi[k]); }
    return r;
}
HBox hb_inter(const HBox& a, const HBox& b) {
    HBox r;
    for (int k = 0; k < 3; ++k) { r.lo[k] = std::max(a.lo[k], b.lo[k]); r.hi[k] = std::min(a.hi[k], b.hi[k]); }
    return hb_empty(r) ? hb_none() : r;
}
HBox hb_point(const float* p) { return HBox{{p[0], p[1], p[2]}, {p[0], p[1], p[2]}}; }
HBox hb_pad(HBox b) {
    if (hb_empty(b) || !hb_finite(b)) return b;
    double m = 0.0;
    for (int k = 0; k < 3; ++k) m = std::max({m, std::fabs(b.lo[k]), std::fabs(b.hi[k]), b.hi[k] - b.lo[k]});
    const double pad = 1e-4 * m + 1e-6;
    for (int k = 0; k < 3; ++k) { b.lo[k] -= pad; b.hi[k] += pad; }
    return b;
}
double hb_volume(const HBox& b) {
    if (hb_empty(b)) return 0.0;
    return (b.hi[0] - b.lo[0]) * (b.hi[1] - b.lo[1]) * (b.hi[2] - b.lo[2]);
}
// M * (x, y, z, 1) of the eight corners (node frame -> parent frame)
HBox hb_xform(const float* M, const HBox& b) {
    if (hb_empty(b)) return b;
    if (!hb_finite(b)) return hb_all();
    HBox r = hb_none();
    for (int c = 0; c < 8; ++c) {
        const double x = (c & 1) ? b.hi[0] : b.lo[0], y = (c & 2) ? b.hi[1] : b.lo[1], z = (c & 4) ? b.hi[2] : b.lo[2];
        double q[3];
        for (int k = 0; k < 3; ++k) q[k] = (double)M[k] * x + (double)M[4 + k] * y + (double)M[8 + k] * z + (double)M[12 + k];
        r = hb_union(r, HBox{{q[0], q[1], q[2]}, {q[0], q[1], q[2]}});
    }
    return hb_pad(r);
}
void hb_store(const HBox& b, float* lo, float* hi) {
    for (int k = 0; k < 3; ++k) {  // round outwards
        lo[k] = (float)b.lo[k];
        hi[k] = (float)b.hi[k];
        if ((double)lo[k] > b.lo[k]) lo[k] = std::nextafter(lo[k], -INFINITY);
        if ((double)hi[k] < b.hi[k]) hi[k] = std::nextafter(hi[k], INFINITY);
    }
    // lo[3]: the culling test's max |coordinate| (rtx_trace.h ray_meets), -inf for an empty
    // box (lo > hi on some axis, or NaN)
    const bool nonempty = lo[0] <= hi[0] && lo[1] <= hi[1] && lo[2] <= hi[2];
    lo[3] = nonempty ? std::fmax(std::fmax(std::fmax(std::fabs(lo[0]), std::fabs(lo[1])), std::fmax(std::fabs(lo[2]), std::fabs(hi[0]))),
                                 std::fmax(std::fabs(hi[1]), std::fabs(hi[2])))
                     : -INFINITY;
    hi[3] = 0.0f;
}

struct NodeBoxes {
    HBox h, i, s;
};

NodeBoxes leaf_boxes(const DObj& o, const std::vector<DTri>& tris, double tlo, double thi) {
    auto moved_box = [&](const float* p) {
        HBox b = hb_point(p);
        if (o.has_speed)
            for (double t : {tlo, thi}) {
                float q[3];
                for (int k = 0; k < 3; ++k) q[k] = p[k] + o.speed[k] * (float)t;
                b = hb_union(b, hb_point(q));
            }
        return b;
    };
    NodeBoxes nb;
    if (o.type == OBJ_SPHERE) {
        HBox b = moved_box(o.a);
        for (int k = 0; k < 3; ++k) { b.lo[k] -= o.radius; b.hi[k] += o.radius; }
        nb.h = nb.i = nb.s = hb_pad(b);
    } else if (o.type == OBJ_BOX) {
        const HBox b = hb_pad(hb_union(moved_box(o.a), moved_box(o.b)));
        nb.h = nb.i = nb.s = b;
    } else if (o.type == OBJ_PLANE) {
        nb.h = nb.s = hb_all();
        nb.i = hb_none();
    } else {  // mesh (no motion: mesh.py never reads speed)
        HBox b = hb_none();
        for (int f = 0; f < o.tri_count; ++f) {
            const DTri& T = tris[o.tri_begin + f];
            b = hb_union(b, hb_union(hb_point(T.v0), hb_union(hb_point(T.v1), hb_point(T.v2))));
        }
        nb.h = nb.s = hb_pad(b);
        nb.i = hb_none();
    }
    return nb;
}

// The device forms of the node and box records (rtx_trace.h DNodeHot / DNodeMat / DBox).
void split_nodes(const std::vector<DNode>& nodes, std::vector<DNodeHot>& hot, std::vector<DNodeMat>& mat) {
    hot.resize(nodes.size());
    mat.resize(nodes.size());
    for (size_t i = 0; i < nodes.size(); ++i) {
        const DNode& n = nodes[i];
        hot[i] = DNodeHot{n.kind, n.parent, n.cidx, n.depth, n.end, n.pkind, n.obj, n.mat0, n.oid, 0, 0, 0};
        std::memcpy(mat[i].M, n.M, sizeof(n.M));
        std::memcpy(mat[i].Minv, n.Minv, sizeof(n.Minv));
    }
}
// [hit boxes | inside boxes | shadow boxes], n each
std::vector<DBox> split_bounds(const std::vector<DBound>& b) {
    const size_t n = b.size();
    std::vector<DBox> out(3 * n);
    for (size_t i = 0; i < n; ++i) {
        std::memcpy(out[i].lo, b[i].hlo, 16); std::memcpy(out[i].hi, b[i].hhi, 16);
        std::memcpy(out[n + i].lo, b[i].ilo, 16); std::memcpy(out[n + i].hi, b[i].ihi, 16);
        std::memcpy(out[2 * n + i].lo, b[i].slo, 16); std::memcpy(out[2 * n + i].hi, b[i].shi, 16);
    }
    return out;
}
void bind_boxes(SceneView& v, const DBox* base, size_t n) {
    v.hbox = (cptr<DBox>)base;
    v.ibox = (cptr<DBox>)(base + n);
    v.sbox = (cptr<DBox>)(base + 2 * n);
}

std::vector<DBound> compute_bounds(const std::vector<DNode>& nodes, const std::vector<DObj>& objs,
                                   const std::vector<DTri>& tris, double tlo, double thi) {
    const int n = (int)nodes.size();
    std::vector<NodeBoxes> nb(n);
    for (int x = n - 1; x >= 0; --x) {  // children before parents
        const DNode& X = nodes[x];
        if (X.kind == HN_LEAF) { nb[x] = leaf_boxes(objs[X.obj], tris, tlo, thi); continue; }
        std::vector<int> ch;
        for (int j = x + 1; j < X.end; j = nodes[j].end) ch.push_back(j);
        NodeBoxes r{hb_none(), hb_none(), hb_none()};
        if (X.kind == HN_UNION) {
            for (int c : ch) { r.h = hb_union(r.h, nb[c].h); r.i = hb_union(r.i, nb[c].i); r.s = hb_union(r.s, nb[c].s); }
        } else if (X.kind == HN_INTER) {
            r.i = hb_all();
            r.s = hb_all();
            double best = INFINITY;
            for (int c : ch) {
                HBox hc = nb[c].h;
                for (int c2 : ch)
                    if (c2 != c) hc = hb_inter(hc, nb[c2].i);
                r.h = hb_union(r.h, hc);
                r.i = hb_inter(r.i, nb[c].i);
                const double v = hb_empty(nb[c].s) ? -1.0 : (hb_finite(nb[c].s) ? hb_volume(nb[c].s) : INFINITY);
                if (v < best) { best = v; r.s = nb[c].s; }  // every child must shadow: any one child bounds it
            }
        } else if (X.kind == HN_DIFF && ch.size() >= 2) {
            r.h = hb_union(nb[ch[0]].h, hb_inter(nb[ch[1]].h, nb[ch[0]].i));
            r.i = nb[ch[0]].i;
            r.s = r.h;  // diff shadow = some surviving hit past the epsilon
        }
        nb[x] = NodeBoxes{hb_xform(X.M, r.h), hb_xform(X.M, r.i), hb_xform(X.M, r.s)};
    }
    // The culling box of a child also carries its parent's filter on the child's hits:
    // intersection keeps hits inside every sibling, difference keeps child-1 hits inside
    // child 0 (hierarchy.py:52-70); both are boxes in the child's (parent) frame.
    std::vector<HBox> hcull(n);
    for (int x = 0; x < n; ++x) hcull[x] = nb[x].h;
    for (int x = 0; x < n; ++x) {
        const DNode& X = nodes[x];
        if (X.kind != HN_INTER && X.kind != HN_DIFF) continue;
        std::vector<int> ch;
        for (int j = x + 1; j < X.end; j = nodes[j].end) ch.push_back(j);
        for (size_t a = 0; a < ch.size(); ++a) {
            if (X.kind == HN_INTER) {
                for (size_t b = 0; b < ch.size(); ++b)
                    if (b != a) hcull[ch[a]] = hb_inter(hcull[ch[a]], nb[ch[b]].i);
            } else if (a == 1) {
                hcull[ch[1]] = hb_inter(hcull[ch[1]], nb[ch[0]].i);
            }
        }
    }
    std::vector<DBound> out(n);
    for (int x = 0; x < n; ++x) {
        hb_store(hcull[x], out[x].hlo, out[x].hhi);
        hb_store(nb[x].i, out[x].ilo, out[x].ihi);
        hb_store(nb[x].s, out[x].slo, out[x].shi);
    }
    return out;
}

struct HostScene {
    std::vector<DNode> nodes;
    std::vector<uint32_t> texels;
    std::vector<float> lut255;
    int32_t hlevels = 0;
    bool has_ext = false;  // hierarchies or textures
    std::vector<DObj> objs;
    std::vector<DTri> tris;
    std::vector<DTriN> trins;
    std::vector<DFaceBox> fboxes;
    std::vector<DLeaf> leaves;
    std::vector<int32_t> tri_orig;
    std::vector<DMat> mats;
    std::vector<DLight> lights;
    bool has_mesh = false, has_secondary = false;
    int32_t n_objs = 0, n_lights = 0;
    int32_t n_plane = 0, n_sphere = 0, n_box = 0, n_mesh = 0;
    int32_t pow_bits = 0;
    int32_t uniform_hard = -2;  // -2: no specular lobe; -1: mixed or non-integer
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
    H.fboxes.assign(desc->n_triangles, DFaceBox{});
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
        if (!d.spec_zero) {  // the one integer hardness of every specular lobe, or -1
            const int h = d.hard_is_int ? d.hard_int : -1;
            H.uniform_hard = H.uniform_hard == -2 ? h : (H.uniform_hard == h ? h : -1);
        }
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
        for (int k = 0; k < 3; ++k) {
            H.fboxes[i].lo[k] = std::min(t.v0[k], std::min(t.v1[k], t.v2[k]));
            H.fboxes[i].hi[k] = std::max(t.v0[k], std::max(t.v1[k], t.v2[k]));
        }
        set3(H.trins[i].n0, t.n0);
        set3(H.trins[i].n1, t.n1);
        set3(H.trins[i].n2, t.n2);
    }
    // textures: RGBA8 texels (alpha unused), fl32(k / 255) table
    if (desc->n_textures < 0 || (desc->n_textures && !desc->textures))
        return fail(RTX_ERR_INVALID, "rtx_scene_create: bad texture array");
    std::vector<int64_t> tex_off(desc->n_textures);
    for (int t = 0; t < desc->n_textures; ++t) {
        const rtx_texture& tx = desc->textures[t];
        if (tx.width < 1 || tx.height < 1 || !tx.rgb || (int64_t)tx.width * tx.height > (1 << 28))
            return fail(RTX_ERR_INVALID, "texture " + std::to_string(t) + ": bad size or data");
        tex_off[t] = (int64_t)H.texels.size();
        const int64_t n = (int64_t)tx.width * tx.height;
        for (int64_t q = 0; q < n; ++q)
            H.texels.push_back((uint32_t)tx.rgb[3 * q] | ((uint32_t)tx.rgb[3 * q + 1] << 8) | ((uint32_t)tx.rgb[3 * q + 2] << 16));
    }
    if ((int64_t)H.texels.size() > INT32_MAX) return fail(RTX_ERR_INVALID, "textures too large");
    H.lut255.resize(256);
    for (int k = 0; k < 256; ++k) H.lut255[k] = (float)(k / 255.0);  // pixel[c] / 255 (fp64) -> vec3
    // hierarchy structure: parents precede children (preorder), parents are nodes
    std::vector<int32_t> top_ordinal(desc->n_objects, -1), nchild(desc->n_objects, 0), cidx(desc->n_objects, 0);
    std::vector<int32_t> depth(desc->n_objects, 0), root_of(desc->n_objects, -1);
    int32_t n_top = 0;
    for (int i = 0; i < desc->n_objects; ++i) {
        const rtx_object& o = desc->objects[i];
        const std::string tag = "object " + std::to_string(i) + ": ";
        if (o.parent == -1) {
            top_ordinal[i] = n_top++;
            root_of[i] = i;
        } else {
            if (o.parent < 0 || o.parent >= i || desc->objects[o.parent].type != RTX_NODE)
                return fail(RTX_ERR_INVALID, tag + "parent must be an earlier RTX_NODE record");
            if (i > o.parent + 1) {  // preorder: the previous record is the parent or inside a sibling subtree
                int a = i - 1;
                while (a != -1 && a != o.parent) a = desc->objects[a].parent;
                if (a != o.parent) return fail(RTX_ERR_INVALID, tag + "records are not in preorder");
            }
            cidx[i] = nchild[o.parent]++;
            depth[i] = depth[o.parent] + 1;
            root_of[i] = root_of[o.parent];
            if (depth[i] >= kMaxHLevels - 2) return fail(RTX_ERR_INVALID, tag + "hierarchy too deep");
        }
        if (o.type == RTX_NODE && (o.hierarchy_type < RTX_UNION || o.hierarchy_type > RTX_HIER_OTHER))
            return fail(RTX_ERR_INVALID, tag + "bad hierarchy type");
        if (o.texture < -1 || o.texture >= desc->n_textures || (o.texture >= 0 && o.type != RTX_PLANE && o.type != RTX_BOX))
            return fail(RTX_ERR_INVALID, tag + "bad texture index");
    }
    for (int i = 0; i < desc->n_objects; ++i)
        if (desc->objects[i].type == RTX_NODE && desc->objects[i].hierarchy_type == RTX_DIFFERENCE && nchild[i] < 2)
            return fail(RTX_ERR_INVALID, "object " + std::to_string(i) +
                                             ": difference node needs two children (the reference raises IndexError)");
    for (int i = 0; i < desc->n_objects; ++i) {
        const rtx_object& o = desc->objects[i];
        DObj& d = H.objs[i];
        std::memset(&d, 0, sizeof(d));
        const std::string tag = "object " + std::to_string(i) + ": ";
        d.type = o.type;
        d.nmat = o.n_mats;
        if (o.texture >= 0) {
            const rtx_texture& tx = desc->textures[o.texture];
            d.has_tex = 1;
            d.tex_off = (int32_t)tex_off[o.texture];
            d.tex_w = tx.width;
            d.tex_h = tx.height;
            d.tex_scale = o.texture_scale;
            H.has_ext = true;
        }
        d.oid = top_ordinal[root_of[i]];
        if (o.type == RTX_NODE) {
            H.has_ext = true;
            if (o.n_mats > 0 && (o.mat[0] < 0 || o.mat[0] >= desc->n_materials))
                return fail(RTX_ERR_INVALID, tag + "material index out of range");
            continue;
        }
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
                d.r2f = (float)d.r2;
                d.radius = o.radius;
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
                // the padded pre-test's inputs of a static box (rtx_trace.h box_maybe_hit_obj):
                // sorted corners in c / e, max |coordinate| in c[3], as the kernel forms them
                for (int k = 0; k < 3; ++k) {
                    d.c[k] = std::fmin(d.a[k], d.b[k]);
                    d.e[k] = std::fmax(d.a[k], d.b[k]);
                }
                d.c[3] = std::fmax(std::fmax(std::fmax(std::fabs(d.a[0]), std::fabs(d.a[1])),
                                             std::fmax(std::fabs(d.a[2]), std::fabs(d.b[0]))),
                                   std::fmax(std::fabs(d.b[1]), std::fabs(d.b[2])));
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
                // the bounding box's padded pre-test inputs (rtx_trace.h bv_maybe), as for boxes
                for (int k = 0; k < 3; ++k) {
                    d.c[k] = std::fmin(d.bv_a[k], d.bv_b[k]);
                    d.e[k] = std::fmax(d.bv_a[k], d.bv_b[k]);
                }
                d.c[3] = std::fmax(std::fmax(std::fmax(std::fabs(d.bv_a[0]), std::fabs(d.bv_a[1])),
                                             std::fmax(std::fabs(d.bv_a[2]), std::fabs(d.bv_b[0]))),
                                   std::fmax(std::fabs(d.bv_b[1]), std::fabs(d.bv_b[2])));
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
            if (desc->objects[i].parent == -1 && H.objs[i].type == order[g]) {
                grouped.push_back(H.objs[i]);
                counts[g]++;
            }
    std::vector<DObj> all_objs;
    all_objs.swap(H.objs);
    H.objs.swap(grouped);
    H.n_plane = counts[0]; H.n_sphere = counts[1]; H.n_box = counts[2]; H.n_mesh = counts[3];
    // Mesh BVH: median splits on face centroids down to clusters of <= 8 faces, stored in
    // preorder with skip indices (stackless traversal); faces are reordered by cluster and
    // keep their OBJ order index (tri_orig) for closest-hit ties.
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
        const int32_t node0 = (int32_t)H.leaves.size();
        float cmax = 0.0f;
        std::function<void(int32_t, int32_t)> build = [&](int32_t a, int32_t e) {
            const int32_t me = (int32_t)H.leaves.size();
            H.leaves.push_back(DLeaf{});
            DLeaf L{};
            for (int ax = 0; ax < 3; ++ax) { L.lo[ax] = INFINITY; L.hi[ax] = -INFINITY; }
            if (e - a <= RTX_LEAF_FACES) {
                L.first = a;
                L.count = e - a;
                for (int32_t k = a; k < e; ++k) {
                    const DTri& t = H.tris[b0 + idx[k]];
                    for (const float* v : {t.v0, t.v1, t.v2})
                        for (int ax = 0; ax < 3; ++ax) {
                            L.lo[ax] = std::min(L.lo[ax], v[ax]);
                            L.hi[ax] = std::max(L.hi[ax], v[ax]);
                            cmax = std::max(cmax, std::fabs(v[ax]));
                        }
                }
            } else {
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
                const int32_t left = me + 1;
                build(a, mid);
                const int32_t right = (int32_t)H.leaves.size();
                build(mid, e);
                L.first = -1;
                L.count = 0;
                for (int q = 0; q < 3; ++q) {
                    L.lo[q] = std::min(H.leaves[left].lo[q], H.leaves[right].lo[q]);
                    L.hi[q] = std::max(H.leaves[left].hi[q], H.leaves[right].hi[q]);
                }
            }
            L.skip = (int32_t)H.leaves.size() - node0;  // next node after this subtree (mesh-relative)
            H.leaves[me] = L;
        };
        if (n > 0) build(0, n);
        std::vector<DTri> tris(n);
        std::vector<DTriN> trins(n);
        std::vector<DFaceBox> fboxes(n);
        for (int32_t k = 0; k < n; ++k) {
            tris[k] = H.tris[b0 + idx[k]];
            trins[k] = H.trins[b0 + idx[k]];
            fboxes[k] = H.fboxes[b0 + idx[k]];
            H.tri_orig[b0 + k] = idx[k];
        }
        std::copy(tris.begin(), tris.end(), H.tris.begin() + b0);
        std::copy(trins.begin(), trins.end(), H.trins.begin() + b0);
        std::copy(fboxes.begin(), fboxes.end(), H.fboxes.begin() + b0);
        // Per-face boxes pay off when faces are large next to a wave's 8x8 pixel footprint,
        // i.e. for small meshes (TorusMesh 1080p: 165 -> 143 us); on an 81,920-face mesh
        // the cluster boxes already isolate the faces and the extra test costs 9 %.
        d.face_cull = n <= kFaceCullMaxFaces ? 1 : 0;
        d.leaf_begin = node0;
        d.leaf_count = (int32_t)H.leaves.size() - node0;
        d.cmax = cmax;
    }
    // Hierarchies: the subtrees of the top-level nodes, in preorder, as DNode records;
    // their leaves are appended to objs (after the top-level groups, faces in OBJ order).
    std::vector<int32_t> node_of(desc->n_objects, -1);
    for (int i = 0; i < desc->n_objects; ++i) {
        const rtx_object& o = desc->objects[i];
        if (root_of[i] < 0 || desc->objects[root_of[i]].type != RTX_NODE) continue;
        DNode nd;
        std::memset(&nd, 0, sizeof(nd));
        node_of[i] = (int32_t)H.nodes.size();
        nd.parent = o.parent >= 0 ? node_of[o.parent] : -1;
        nd.pkind = o.parent >= 0 ? desc->objects[o.parent].hierarchy_type : -1;
        nd.cidx = cidx[i];
        nd.depth = depth[i];
        nd.oid = top_ordinal[root_of[i]];
        nd.mat0 = o.n_mats > 0 ? o.mat[0] : -1;
        nd.obj = -1;
        if (o.type == RTX_NODE) {
            nd.kind = o.hierarchy_type;
            Mat4 M, Mi;
            make_matrices(o.trs, M, Mi);
            std::memcpy(nd.M, M.m, sizeof(nd.M));
            std::memcpy(nd.Minv, Mi.m, sizeof(nd.Minv));
            H.hlevels = std::max(H.hlevels, nd.depth + 2);
        } else {
            nd.kind = HN_LEAF;
            nd.obj = (int32_t)H.objs.size();
            H.objs.push_back(all_objs[i]);
        }
        H.nodes.push_back(nd);
    }
    for (int i = (int)desc->n_objects - 1; i >= 0; --i) {  // subtree ends
        if (node_of[i] < 0) continue;
        DNode& nd = H.nodes[node_of[i]];
        if (nd.end == 0) nd.end = node_of[i] + 1;
        if (nd.parent >= 0) H.nodes[nd.parent].end = std::max(H.nodes[nd.parent].end, nd.end);
    }
    H.n_objs = (int32_t)H.objs.size();
    H.n_lights = desc->n_lights;
    set3(H.ambient, desc->ambient);
    return RTX_OK;
}

// Validates the camera and fills the scalar part of KParams; table pointers are left for
// the caller (device uploads, or host arrays in the emulation build).
int convert_camera(const rtx_camera_desc* c, KParams& k) {
    if (!c) return fail(RTX_ERR_INVALID, "rtx_camera_set: null argument");
    k = KParams{};
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

// An upper bound of |o| for every camera ray origin (AA/DOF origins plus jitter); +inf if
// a table is not finite.
double camera_origin_bound(const rtx_camera_desc* c) {
    double m = 0.0;
    const int64_t n = (int64_t)c->n_dof * c->n_aa;
    for (int64_t i = 0; i < n; ++i) {
        const float* p = c->aa_origins + 3 * i;
        m = std::max(m, std::sqrt((double)p[0] * p[0] + (double)p[1] * p[1] + (double)p[2] * p[2]));
    }
    if (c->jitter != RTX_JITTER_OFF) m += std::fabs(c->jitter_scale) * (1.0 + 1e-5);
    return std::isfinite(m) ? m * (1.0 + 1e-6) : INFINITY;
}

// Self tests of planes (SceneView::plane_self). A camera ray (origin o, |o| <= omax) hits
// static plane k (point p0, normal n) at P = fl32(o + d t32), t32 = fl32(num0 / den0) of
// fp32 dot products. With num0 = num + A, den0 = den + B (their roundings),
//   t32 den - num = A + e (num + A) - t32 B  (exactly; e: the quotient's rounding),
// and |t32 B| <= 2^-22 |n|_1 |P - o|: so P's offset from the plane, (P - p0).n, stays
// within 2^-20 |n|_1 (|p0|_1 + |o|_1 + |P|_1) however grazing the ray, and the shadow
// test's own num' = fl32((p0 - P).n) within 2^-19 |n|_1 (...) =: b0 + b1 m (m = max |P_i|,
// |P|_1 <= 3m, |o|_1 <= 3 omax). The test needs 1e-4 < num' / denom' to pass; denom' =
// fl32(D.n) is at least c0 - c1 m (directional D: |D.n| less its rounding; point light
// L: |(L - p0).n| less P's offset and the roundings of L - P and the dot). So for
// m < (0.5e-4 c0 - b0) / (b1 + 0.5e-4 c1) the plane cannot occlude its own hit point
// (|num' / denom'| < 0.5e-4). Returns [light][plane < 4] limits (-1: none).
std::vector<float> plane_self_limits(const HostScene& H, double omax) {
    std::vector<float> lim(4 * H.lights.size(), -1.0f);
    if (!std::isfinite(omax)) return lim;
    for (size_t li = 0; li < H.lights.size(); ++li) {
        const DLight& Lt = H.lights[li];
        for (int32_t k = 0; k < std::min(H.n_plane, 4); ++k) {
            const DObj& ob = H.objs[k];
            if (ob.has_speed) continue;
            double n1 = 0.0, p01 = 0.0, h = 0.0, dabs = 0.0, l1 = 0.0;
            for (int a = 0; a < 3; ++a) {
                n1 += std::fabs((double)ob.b[a]);
                p01 += std::fabs((double)ob.a[a]);
            }
            const double b0 = 0x1p-19 * n1 * (p01 + 3.0 * omax), b1 = 0x1p-19 * n1 * 3.0;
            double c0, c1;
            if (Lt.type == LIGHT_DIRECTIONAL) {
                for (int a = 0; a < 3; ++a) {
                    h += (double)Lt.negvec[a] * ob.b[a];
                    dabs += std::fabs((double)Lt.negvec[a] * ob.b[a]);
                }
                c0 = std::fabs(h) - 0x1p-21 * dabs;
                c1 = 0.0;
            } else {
                for (int a = 0; a < 3; ++a) {
                    h += ((double)Lt.vec[a] - ob.a[a]) * ob.b[a];
                    l1 += std::fabs((double)Lt.vec[a]);
                }
                c0 = std::fabs(h) * (1.0 - 1e-12) - b0 - 0x1p-21 * n1 * l1;
                c1 = b1 + 0x1p-21 * n1 * 3.0;
            }
            const double m = (0.5e-4 * c0 - b0) / (b1 + 0.5e-4 * c1);
            if (!(m > 0.0) || !std::isfinite(m)) continue;
            float f = (float)(m * (1.0 - 1e-6));
            if ((double)f > m) f = std::nextafter(f, 0.0f);
            lim[4 * li + k] = f;
        }
    }
    return lim;
}

// $RTX_LENS_BINS=0: lens cameras get no primary-ray bins (experiment, A/B)
bool lens_bins_disabled() {
    return !opt_on(OPT_LENS_BINS);
}

// Primary-ray bins. With one sample per pixel, no lens (dof origin == camera position)
// and no jitter, every primary ray leaves the same origin o (the AA origin, scene.py:60-61)
// in the direction of x u + y v - d w (scene.py:54): a pinhole projection. An object whose
// bounding points all lie in front of o projects inside the rectangle of its projected
// points; padded by 2 pixels (far beyond the ~1e-4 px the fp32 ray setup moves a ray), it
// holds every pixel whose primary ray can hit the object. Rectangles are binned into 8x8
// pixel bins aligned with the strip's columns and the image rows, so a tile that starts
// on a multiple of 8 rows finds in its bin (rtx_kernels.h primary_bin):
//   * objmask: the spheres (bits 0-15) and boxes (16-31) it may hit; spheres are inflated
//     by 2^-8 (|o - c| + r), beyond the fuzz of the reference's fp32 discriminant (a ray
//     can "hit" a sphere it misses by ~2^-10.5 |o - c|); moving objects by their sweep over
//     the frame's times; objects beyond the 16th of a kind are always tested;
//   * rootmask: the hierarchy roots (bit q: the q-th of the first 32) whose hit box
//     (compute_bounds' h over the frame's times) it may meet;
//   * the faces of the scene's one top-level mesh (if it has exactly one) it may hit,
//     nearest first, with a lower bound of their hit t (depth <= t).
// Other tiles and secondary/shadow rays walk everything. Returns false when the camera
// does not qualify, or a mesh face lies near or behind the origin's plane.
//
// Lens cameras (DOF samples, AA spreads, jitter: scene.py:56-65) get object bins from a
// "thick" pinhole. Sample ray k of a pixel leaves S = aa_o + jitter toward the pixel's
// focal point F = P + f bdir from its DOF origin D: X(l) = S + l (F - D). The pinhole ray
// of the pixel from the camera position P is Y(l) = P + l (F - P), and
//   X(l) - Y(l) = (S - D) + (1 - l) (D - P),  |X - Y| <= R1 + |1 - l| A,
// with A = max |D - P| (the aperture spread) and R1 = max |aa_o - D| + jitter_scale. A hit
// at depth z (along -w from P) has l = (z - (S - P).(-w)) / (F - D).(-w), where
// (F - D).(-w) lies in [f cmin - A, f + A] (cmin: the smallest bdir.(-w) of the strip's
// pixel table) and |(S - P).(-w)| <= A + R1: so l, and the deviation, are bounded by the
// object's depth range. An object grown by that deviation contains a point of the
// pinhole ray of every pixel some sample of which hits it, and its pinhole projection
// from P bins the tile as above. The mesh faces keep no bins (their t lower bounds hold
// for one origin only).
bool primary_bins(const HostScene& H, const rtx_camera_desc* c, const std::vector<DBound>& nodeb,
                  std::vector<int32_t>& start, std::vector<int32_t>& faces, std::vector<float>& zmin,
                  std::vector<uint32_t>& objmask, std::vector<uint32_t>& rootmask, int32_t& bins_x,
                  int32_t& mesh_bins, bool* faces_on_device = nullptr) {
    if (faces_on_device) *faces_on_device = false;
    if (c->ncols < 2 || c->height < 2) return false;
    const bool pinhole = c->n_dof == 1 && c->n_aa == 1 && c->jitter == RTX_JITTER_OFF &&
                         c->dof_origins[0] == c->position[0] && c->dof_origins[1] == c->position[1] &&
                         c->dof_origins[2] == c->position[2];
    if (!pinhole && lens_bins_disabled()) return false;
    const double o[3] = {pinhole ? c->aa_origins[0] : c->position[0], pinhole ? c->aa_origins[1] : c->position[1],
                         pinhole ? c->aa_origins[2] : c->position[2]};
    double lensA = 0.0, lensR1 = 0.0;  // the lens bounds A and R1 (above)
    if (!pinhole) {
        for (int32_t kd = 0; kd < c->n_dof; ++kd) {
            const float* D = c->dof_origins + 3 * kd;
            double a2 = 0.0;
            for (int a = 0; a < 3; ++a) a2 += ((double)D[a] - o[a]) * ((double)D[a] - o[a]);
            lensA = std::max(lensA, std::sqrt(a2));
            for (int32_t ka = 0; ka < c->n_aa; ++ka) {
                const float* S = c->aa_origins + 3 * ((size_t)kd * c->n_aa + ka);
                double r2 = 0.0;
                for (int a = 0; a < 3; ++a) r2 += ((double)S[a] - D[a]) * ((double)S[a] - D[a]);
                lensR1 = std::max(lensR1, std::sqrt(r2));
            }
        }
        if (c->jitter != RTX_JITTER_OFF) lensR1 += std::fabs(c->jitter_scale) * (1.0 + 1e-5);
        if (!std::isfinite(lensA) || !std::isfinite(lensR1)) return false;
    }
    const int32_t W = c->ncols, Hh = c->height;
    const double dx = ((double)c->xs[W - 1] - (double)c->xs[0]) / (W - 1);
    const double dy = ((double)c->ys[Hh - 1] - (double)c->ys[0]) / (Hh - 1);
    if (!(dx > 0.0) || !(dy > 0.0)) return false;
    for (int32_t i = 1; i < W; ++i)
        if (!(c->xs[i] > c->xs[i - 1])) return false;
    for (int32_t j = 1; j < Hh; ++j)
        if (!(c->ys[j] > c->ys[j - 1])) return false;
    // lens cameras: the deviation bound R1 + |1 - l| A of a hit at depths [zlo, zhi], padded
    // by 1e-5 of the magnitudes (the fp32 ray setup: origins, focal point, direction)
    const double xm = std::max(std::fabs((double)c->xs[0]), std::fabs((double)c->xs[W - 1]));
    const double ym = std::max(std::fabs((double)c->ys[0]), std::fabs((double)c->ys[Hh - 1]));
    const double cmin = c->d / std::sqrt(xm * xm + ym * ym + c->d * c->d) * (1.0 - 1e-6);
    const double f = c->focal_length, den_lo = f * cmin - lensA, den_hi = f + lensA;
    const double omag = std::sqrt(o[0] * o[0] + o[1] * o[1] + o[2] * o[2]);
    if (!pinhole && !(den_lo > 0.05 * f * cmin)) return false;  // aperture too wide for the bound
    auto lens_pad = [&](double zlo, double zhi) {
        if (pinhole) return 0.0;
        const double R2 = lensA + lensR1, nlo = zlo - R2, nhi = zhi + R2;
        const double lmin = nlo > 0.0 ? nlo / den_hi : 0.0;
        const double lmax = nhi > 0.0 ? nhi / den_lo : 0.0;
        const double m = std::max(std::fabs(1.0 - lmin), std::fabs(1.0 - lmax));
        return (lensR1 + m * lensA) * (1.0 + 1e-5) + 1e-5 * (lmax * den_hi + omag + R2 + f);
    };
    // fractional column / row of a point in the camera's own (fp32) pixel tables and the
    // bin rectangle of a point set (rtx_bins.h: the same arithmetic as the device face pass)
    BinProj BP;
    for (int a = 0; a < 3; ++a) {
        BP.o[a] = o[a];
        BP.u[a] = c->u[a]; BP.v[a] = c->v[a]; BP.w[a] = c->w[a];
    }
    BP.d = c->d;
    BP.xs = c->xs;
    BP.ys = c->ys;
    BP.W = W;
    BP.H = Hh;
    bins_x = (W + 7) / 8;
    const int32_t bins_y = (Hh + 7) / 8;
    const size_t nb = (size_t)bins_x * bins_y;
    using Rect = BinRect;
    auto rect_of = [&](const double (*pts)[3], int n, Rect& R, double& zlo) { return bins_rect(BP, pts, n, R, zlo); };
    auto mark_in = [&](std::vector<uint32_t>& m, const Rect& R, uint32_t bit) {
        for (int32_t by = R.r0; by <= R.r1; ++by)
            for (int32_t bx = R.c0; bx <= R.c1; ++bx) m[(size_t)by * bins_x + bx] |= bit;
    };
    auto mark = [&](const Rect& R, uint32_t bit) { mark_in(objmask, R, bit); };
    auto box_corners = [](const double lo[3], const double hi[3], double (*pts)[3]) {
        for (int q = 0; q < 8; ++q)
            for (int a = 0; a < 3; ++a) pts[q][a] = (q >> a) & 1 ? hi[a] : lo[a];
    };
    objmask.assign(nb, 0u);
    const Rect all{0, bins_x - 1, 0, bins_y - 1};
    // moving objects: moved() = fl32(p + speed * time) over the frame's times, padded
    double tlo = INFINITY, thi = -INFINITY;
    for (int32_t i = 0; i < c->n_times; ++i) {
        tlo = std::min(tlo, (double)(float)c->times[i]);
        thi = std::max(thi, (double)(float)c->times[i]);
    }
    auto sweep = [&](const DObj& ob, double* lo, double* hi) {
        if (!ob.has_speed) return;
        for (int a = 0; a < 3; ++a) {
            const double s0 = (double)ob.speed[a] * tlo, s1 = (double)ob.speed[a] * thi;
            const double pad = 1e-5 * (std::fabs(lo[a]) + std::fabs(hi[a]) + std::fabs(s0) + std::fabs(s1));
            lo[a] += std::min(s0, s1) - pad;
            hi[a] += std::max(s0, s1) + pad;
        }
    };
    // the bins of a box, grown for a lens camera by the deviation over its depth range
    auto box_rect = [&](double* lo, double* hi, Rect& R) {
        double pts[8][3], z;
        box_corners(lo, hi, pts);
        if (!pinhole) {
            double zlo = INFINITY, zhi = -INFINITY;
            for (int q = 0; q < 8; ++q) {
                double zq = 0.0;
                for (int a = 0; a < 3; ++a) zq -= (pts[q][a] - o[a]) * c->w[a];
                zlo = std::min(zlo, zq);
                zhi = std::max(zhi, zq);
            }
            const double g = lens_pad(zlo, zhi);
            for (int a = 0; a < 3; ++a) { lo[a] -= g; hi[a] += g; }
            box_corners(lo, hi, pts);
        }
        return std::isfinite(lo[0] + lo[1] + lo[2] + hi[0] + hi[1] + hi[2]) && rect_of(pts, 8, R, z);
    };
    for (int32_t k = 0; k < H.n_sphere; ++k) {
        const DObj& ob = H.objs[H.n_plane + k];
        const uint32_t bit = 1u << (k & 15);
        double lo[3], hi[3], oc2 = 0.0, sp = 0.0;
        for (int a = 0; a < 3; ++a) {
            oc2 += ((double)ob.a[a] - o[a]) * ((double)ob.a[a] - o[a]);
            if (ob.has_speed) sp += (double)ob.speed[a] * ob.speed[a];
        }
        // lens: every sample origin lies within A + R1 of o; moving: the centre within
        // |speed| max|t| of its place
        const double mt = std::max(std::fabs(tlo), std::fabs(thi));
        const double re = ob.radius + 0x1p-8 * (std::sqrt(oc2) + std::sqrt(sp) * mt + lensA + lensR1 + std::fabs(ob.radius));
        for (int a = 0; a < 3; ++a) { lo[a] = ob.a[a] - re; hi[a] = ob.a[a] + re; }
        sweep(ob, lo, hi);
        Rect R;
        if (H.n_sphere > 16 || !std::isfinite(re) || !box_rect(lo, hi, R)) R = all;
        mark(R, bit);
    }
    for (int32_t k = 0; k < H.n_box; ++k) {
        const DObj& ob = H.objs[H.n_plane + H.n_sphere + k];
        const uint32_t bit = 1u << (16 + (k & 15));
        double lo[3], hi[3];
        for (int a = 0; a < 3; ++a) {
            const double p = 1e-5 * (std::fabs((double)ob.a[a]) + std::fabs((double)ob.b[a]) + std::fabs(o[a]));
            lo[a] = std::min((double)ob.a[a], (double)ob.b[a]) - p;
            hi[a] = std::max((double)ob.a[a], (double)ob.b[a]) + p;
        }
        sweep(ob, lo, hi);
        Rect R;
        if (H.n_box > 16 || !box_rect(lo, hi, R)) R = all;
        mark(R, bit);
    }
    // hierarchy roots (rootmask bit q: the q-th root; the device tests later ones always):
    // their hit boxes (compute_bounds' h over the frame's time range, world frame), padded
    // like the boxes; an empty one is never hit, an unbounded one may be hit anywhere
    rootmask.assign(nb, 0u);
    {
        int32_t q = 0;
        for (int32_t r = 0; r < (int32_t)H.nodes.size() && r < (int32_t)nodeb.size(); r = H.nodes[r].end, ++q) {
            if (q >= 32) break;
            const DBound& B = nodeb[r];
            double lo[3], hi[3];
            bool empty = false, finite = true;
            for (int a = 0; a < 3; ++a) {
                empty = empty || !(B.hlo[a] <= B.hhi[a]);
                finite = finite && std::isfinite(B.hlo[a]) && std::isfinite(B.hhi[a]);
                const double p = 1e-5 * (std::fabs((double)B.hlo[a]) + std::fabs((double)B.hhi[a]) + std::fabs(o[a]));
                lo[a] = (double)B.hlo[a] - p;
                hi[a] = (double)B.hhi[a] + p;
            }
            if (empty) continue;
            Rect R = all;
            if (finite && !box_rect(lo, hi, R)) R = all;
            mark_in(rootmask, R, 1u << q);
        }
    }
    mesh_bins = 0;
    start.assign(nb + 1, 0);
    faces.clear();
    zmin.clear();
    if (H.n_mesh != 1 || !pinhole) return true;
    if (faces_on_device) {  // the mesh's face bins: rtx_bins.hip (rtx_camera_set)
        *faces_on_device = true;
        return true;
    }
    const DObj& m = H.objs[H.n_plane + H.n_sphere + H.n_box];
    std::vector<Rect> rects(m.tri_count);
    // A hit point P = o + t d (|d| = 1 up to rounding) has depth (P - o).(-w) <= t, and a
    // face's depth is smallest at a vertex: min vertex depth bounds every t on the face
    // (lowered by 1e-4 relative, far beyond the rounding of d, of the reference's t and of
    // the fp32 cast)
    std::vector<double> fz(m.tri_count);
    std::vector<int32_t> count(nb + 1, 0);
    for (int32_t f = 0; f < m.tri_count; ++f) {
        const DTri& T = H.tris[m.tri_begin + f];
        double pts[3][3];
        for (int a = 0; a < 3; ++a) { pts[0][a] = T.v0[a]; pts[1][a] = T.v1[a]; pts[2][a] = T.v2[a]; }
        double zlo;
        if (!rect_of(pts, 3, rects[f], zlo)) return true;  // mesh_bins stays 0: walk the BVH
        for (int32_t by = rects[f].r0; by <= rects[f].r1; ++by)
            for (int32_t bx = rects[f].c0; bx <= rects[f].c1; ++bx) ++count[(size_t)by * bins_x + bx];
        fz[f] = zlo * (1.0 - 1e-4);
    }
    for (size_t bb = 0; bb < nb; ++bb) start[bb + 1] = start[bb] + count[bb];
    faces.assign(start.back(), 0);
    std::vector<int32_t> fill(start.begin(), start.end() - 1);
    std::vector<int32_t> order(m.tri_count);
    for (int32_t f = 0; f < m.tri_count; ++f) order[f] = f;
    std::stable_sort(order.begin(), order.end(), [&](int32_t a2, int32_t b2) { return fz[a2] < fz[b2]; });
    for (int32_t f : order)  // nearest first within each bin
        for (int32_t by = rects[f].r0; by <= rects[f].r1; ++by)
            for (int32_t bx = rects[f].c0; bx <= rects[f].c1; ++bx) faces[fill[(size_t)by * bins_x + bx]++] = f;
    zmin.resize(faces.size());
    for (size_t q = 0; q < faces.size(); ++q) {
        float z = (float)fz[faces[q]];
        if ((double)z > fz[faces[q]]) z = std::nextafter(z, -INFINITY);  // round down
        zmin[q] = z;
    }
    mesh_bins = 1;
    return true;
}

// Light grids (DLGrid, rtx_trace.h): shadow rays of point lights against the scene's one
// top-level mesh. A shadow ray from p toward light L is the line through p and L
// (Mesh.shadow_intersect has no t_max, so the part beyond L counts too): every point of
// it lies in direction +-w = +-(p - L) from L. Seen from a light outside the mesh's
// bounding sphere (centre c, radius r) the mesh fills a cone around a = (c - L) / |c - L|;
// its gnomonic plane (x, y) = (q.u, q.v) / q.a maps +w and -w to the same point and each
// face to the triangle of its projected vertices, so the faces whose padded projection
// covers a cell are the only ones a ray looking up that cell can hit. The padding,
// pad_pos = 2^-17 (2|L| + 2 R + |c - L| + r + |c|) in position (R: the largest |w| a lane
// may look up; farther lanes walk the BVH), is beyond the fp32 error of the reference's
// test -- a reported hit lies on the fp32 line o + t fl(L - o) (an error of t only slides
// it along the line, whose directions from L stay +-w) within ~2^-20 of those magnitudes
// of the face (the rounding of o + d t, of fl(L - o), of the plane's num and of the edge
// functions) -- and of the device's cell arithmetic; the cone is widened by the same
// amount. Lights inside or near the sphere, or seeing it under more than ~57 degrees, get
// no grid.
bool light_grids(const HostScene& H, std::vector<DLGrid>& grids, std::vector<int32_t>& start,
                 std::vector<int32_t>& faces, std::vector<float>& d2) {
    grids.assign(H.lights.size(), DLGrid{});
    start.clear();
    faces.clear();
    d2.clear();
    if (H.n_mesh != 1) return false;
    const DObj& m = H.objs[H.n_plane + H.n_sphere + H.n_box];
    const int32_t F = m.tri_count;
    if (F < 1) return false;
    auto vert = [&](int32_t f, int k, int a) -> double {
        const DTri& T = H.tris[m.tri_begin + f];
        return k == 0 ? T.v0[a] : k == 1 ? T.v1[a] : T.v2[a];
    };
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int32_t f = 0; f < F; ++f)
        for (int k = 0; k < 3; ++k)
            for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], vert(f, k, a)); hi[a] = std::max(hi[a], vert(f, k, a)); }
    double c[3], r2 = 0.0;
    for (int a = 0; a < 3; ++a) c[a] = 0.5 * (lo[a] + hi[a]);
    for (int32_t f = 0; f < F; ++f)
        for (int k = 0; k < 3; ++k) {
            double q = 0.0;
            for (int a = 0; a < 3; ++a) q += (vert(f, k, a) - c[a]) * (vert(f, k, a) - c[a]);
            r2 = std::max(r2, q);
        }
    const double r = std::sqrt(r2) * (1.0 + 1e-9);
    if (!std::isfinite(r)) return false;
    const double cmag = std::sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
    auto down = [](double x) { float f = (float)x; return (double)f > x ? std::nextafter(f, -INFINITY) : f; };
    auto up = [](double x) { float f = (float)x; return (double)f < x ? std::nextafter(f, INFINITY) : f; };
    bool any = false;
    for (size_t li = 0; li < H.lights.size(); ++li) {
        const DLight& Lt = H.lights[li];
        if (Lt.type != LIGHT_POINT) continue;
        const double L[3] = {Lt.vec[0], Lt.vec[1], Lt.vec[2]};
        const double Lmag = std::sqrt(L[0] * L[0] + L[1] * L[1] + L[2] * L[2]);
        double wc[3], Dc2 = 0.0;
        for (int a = 0; a < 3; ++a) { wc[a] = c[a] - L[a]; Dc2 += wc[a] * wc[a]; }
        const double Dc = std::sqrt(Dc2);
        const double Rmax = 4.0 * (Dc + r);
        const double pad_pos = 0x1p-17 * (2.0 * Lmag + 2.0 * Rmax + Dc + r + cmag);
        if (!(Dc > 1.25 * (r + pad_pos)) || !std::isfinite(pad_pos)) continue;
        const double theta = std::asin((r + pad_pos) / Dc) + 0x1p-12;
        if (!(theta < 1.0)) continue;
        const double T = std::tan(theta), d_min = Dc - r - pad_pos;
        const double pad_tan = pad_pos * 2.0 * (1.0 + T) / d_min + 0x1p-14 * (1.0 + T * T);
        // basis, rounded to the fp32 values the device uses
        float af[3], uf[3], vf[3];
        for (int a = 0; a < 3; ++a) af[a] = (float)(wc[a] / Dc);
        const int ax = std::fabs(af[0]) <= std::fabs(af[1]) && std::fabs(af[0]) <= std::fabs(af[2]) ? 0
                       : std::fabs(af[1]) <= std::fabs(af[2]) ? 1 : 2;
        double e[3] = {0.0, 0.0, 0.0}, ud[3], vd[3];
        e[ax] = 1.0;
        const double ad[3] = {af[0], af[1], af[2]};
        ud[0] = ad[1] * e[2] - ad[2] * e[1]; ud[1] = ad[2] * e[0] - ad[0] * e[2]; ud[2] = ad[0] * e[1] - ad[1] * e[0];
        const double un = std::sqrt(ud[0] * ud[0] + ud[1] * ud[1] + ud[2] * ud[2]);
        for (int a = 0; a < 3; ++a) uf[a] = (float)(ud[a] / un);
        const double u2[3] = {uf[0], uf[1], uf[2]};
        vd[0] = ad[1] * u2[2] - ad[2] * u2[1]; vd[1] = ad[2] * u2[0] - ad[0] * u2[2]; vd[2] = ad[0] * u2[1] - ad[1] * u2[0];
        const double vn = std::sqrt(vd[0] * vd[0] + vd[1] * vd[1] + vd[2] * vd[2]);
        for (int a = 0; a < 3; ++a) vf[a] = (float)(vd[a] / vn);
        // the faces' projections (gnomonic bounding rectangles)
        std::vector<double> prj(4 * (size_t)F);
        std::vector<double> ext(F), along(F);
        bool ok = true;
        for (int32_t f = 0; f < F && ok; ++f) {
            double x0 = INFINITY, x1 = -INFINITY, y0 = INFINITY, y1 = -INFINITY;
            along[f] = INFINITY;
            for (int k = 0; k < 3; ++k) {
                double wq[3];
                for (int a = 0; a < 3; ++a) wq[a] = vert(f, k, a) - L[a];
                const double qa = wq[0] * ad[0] + wq[1] * ad[1] + wq[2] * ad[2];
                if (!(qa > 0.0)) { ok = false; break; }
                along[f] = std::min(along[f], qa);  // (q - L).a is linear: smallest at a vertex
                const double x = (wq[0] * u2[0] + wq[1] * u2[1] + wq[2] * u2[2]) / qa;
                const double y = (wq[0] * vf[0] + wq[1] * vf[1] + wq[2] * vf[2]) / qa;
                x0 = std::min(x0, x); x1 = std::max(x1, x);
                y0 = std::min(y0, y); y1 = std::max(y1, y);
            }
            double* P = &prj[4 * (size_t)f];
            P[0] = x0; P[1] = x1; P[2] = y0; P[3] = y1;
            ext[f] = std::max(x1 - x0, y1 - y0) + 2.0 * pad_tan;
        }
        if (!ok) continue;
        // cells a quarter of the median padded face extent (a face covers ~25 cells, a
        // cell lists few faces), at least 64 x 64: finer grids measured faster on TorusMesh
        // (G 10 -> 64: 82.5 -> 69.3 us) and the 81,920-face mesh (G 200 -> 400)
        std::nth_element(ext.begin(), ext.begin() + F / 2, ext.end());
        int32_t G = (int32_t)std::min(512.0, std::max(64.0, std::ceil(4.0 * (2.0 * T) / std::max(ext[F / 2], 1e-12))));
        DLGrid g{};
        for (int a = 0; a < 3; ++a) { g.L[a] = Lt.vec[a]; g.a[a] = af[a]; g.u[a] = uf[a]; g.v[a] = vf[a]; }
        g.G = G;
        g.cos2 = down(std::cos(theta) * std::cos(theta));
        g.tmax = up(T);
        g.scale = (float)((double)G / (2.0 * (double)g.tmax));
        g.r2min = up(1e-8 * Dc2);
        g.r2max = down(Rmax * Rmax);
        g.start_off = (int32_t)start.size();
        // cell range of [x0, x1] as the device maps x (clamped to the grid)
        auto cells = [&](double x0, double x1, int32_t& i0, int32_t& i1) {
            auto cell = [&](double x) {
                const double t = std::floor((x + (double)g.tmax) * (double)g.scale);
                return (int32_t)std::min((double)G - 1, std::max(0.0, t));
            };
            i0 = cell(x0);
            i1 = cell(x1);
        };
        std::vector<int32_t> rect(4 * (size_t)F);
        std::vector<int32_t> count((size_t)G * G + 1, 0);
        for (int32_t f = 0; f < F; ++f) {
            const double* P = &prj[4 * (size_t)f];
            int32_t* R = &rect[4 * (size_t)f];
            cells(P[0] - pad_tan, P[1] + pad_tan, R[0], R[1]);
            cells(P[2] - pad_tan, P[3] + pad_tan, R[2], R[3]);
            for (int32_t iy = R[2]; iy <= R[3]; ++iy)
                for (int32_t ix = R[0]; ix <= R[1]; ++ix) ++count[(size_t)iy * G + ix];
        }
        size_t total = faces.size();
        std::vector<int32_t> fill((size_t)G * G);
        for (size_t q = 0; q < (size_t)G * G; ++q) {
            start.push_back((int32_t)total);
            fill[q] = (int32_t)total;
            total += count[q];
        }
        start.push_back((int32_t)total);
        if (total > (size_t)1 << 28) return false;
        faces.resize(total);
        d2.resize(total);
        // |q - L| >= (q - L).a >= along[f] for every point q of face f; a reported hit lies
        // within pad_pos of the face, and the lane's fp32 |w|^2 is within 2^-21 of its own:
        // (along - 2 pad_pos)^2, rounded down, stays below it whenever the face can occlude
        std::vector<float> key(F);
        for (int32_t f = 0; f < F; ++f) {
            const double k = along[f] - 2.0 * pad_pos;
            key[f] = k > 0.0 ? down(k * k * (1.0 - 1e-6)) : 0.0f;
        }
        std::vector<int32_t> order(F);
        for (int32_t f = 0; f < F; ++f) order[f] = f;
        std::stable_sort(order.begin(), order.end(), [&](int32_t x, int32_t y) { return key[x] < key[y]; });
        for (int32_t f : order) {
            const int32_t* R = &rect[4 * (size_t)f];
            for (int32_t iy = R[2]; iy <= R[3]; ++iy)
                for (int32_t ix = R[0]; ix <= R[1]; ++ix) {
                    const int32_t q = fill[(size_t)iy * G + ix]++;
                    faces[q] = f;
                    d2[q] = key[f];
                }
        }
        grids[li] = g;
        any = true;
    }
    return any;
}


// Heavy tiles of the primary-ray face bins (SceneView::bin_heavy): a bin whose list holds
// more than kHeavyChunk faces is split into chunks of kHeavyChunk consecutive entries, each
// tested by one wave of k_mesh_chunks; the bin's chunks are numbered consecutively.
// Measured on the 81,920-face mesh at 1080p: the silhouette tiles' lists (up to ~770 faces,
// where lanes that miss the mesh keep the early exit from firing) were tested one face at
// a time by one wave and set the frame's length. Returns false when no bin is heavy.
// Lists of at most kHeavyMin faces stay in the render kernel's walk (build knob
// RTX_HEAVY_MIN): with every list longer than 16 chunked, TorusMesh's lists of 17-32 faces
// measured 45.9 -> 57.7 us (profiles/r06/s7/); from 25 faces on, it is unchanged (45.9 us)
// and the 81,920-face mesh gains 4 % (0.1560 -> 0.1498 ms, profiles/r06/s8/).
#ifndef RTX_HEAVY_MIN
#define RTX_HEAVY_MIN 24
#endif
constexpr int32_t kHeavyMin = RTX_HEAVY_MIN;
bool heavy_chunks(const std::vector<int32_t>& bstart, std::vector<int32_t>& bheavy, std::vector<int2>& items) {
    bheavy.clear();
    items.clear();
    if (bstart.size() < 2) return false;
    const size_t nb = bstart.size() - 1;
    bheavy.assign(nb, -1);
    for (size_t b = 0; b < nb; ++b) {
        const int32_t len = bstart[b + 1] - bstart[b];
        if (len <= kHeavyMin) continue;
        bheavy[b] = (int32_t)items.size();  // (items in bin order: a bin's chunks are consecutive)
        for (int32_t c = 0; c * kHeavyChunk < len; ++c) items.push_back(make_int2((int32_t)b, c));
    }
    return !items.empty();
}

constexpr int32_t kDsgG = 512;  // cells per side of a directional light's shadow grid

// Shadow grids of directional lights (DSGrid, rtx_trace.h), per camera (the motion-time
// range [tlo, thi] of the frame bounds the moving objects). Light li's shadow ray from p is
// the half-line p + t d (d = fl32 -direction, LIGHT.negvec; t > 1e-4 or 1e-3). On two
// fp32 unit vectors e1, e2 across d, its points project to p.e + t d.e: a hit point x of
// an object (|x| <= Rx) projects within t |d.e| <= (Rx + |p|) |d.e| / |d| of p's
// projection. So p's projection lies in the object's footprint -- the projection of its
// bounding box (a sphere: c.e +- r |e|; a moving object: its box swept over the time
// range; a hierarchy root: its shadow box, compute_bounds' s, outside of which its
// shadow_intersect is false) -- grown by that drift, by the fuzz of the fp32 sphere
// discriminant (a ray can "hit" a sphere it misses by ~2^-10.5 |p - c|; grown by 2^-8
// (|p| + |c| + r), as primary_bins), and by 2^-18 of the magnitudes (the device's fp32
// dot products and cell arithmetic); every cell the grown footprint meets, widened by one
// cell, lists the object. The grid spans the footprints' union (with two spare cells a
// side) for origins with max |p_i| <= pmax (5/4 of the objects' extent + 1). Objects
// beyond the 16th of a kind, and roots with unbounded shadow boxes, are `always` tested;
// roots with empty ones never. nb: the nodes' bounds for [tlo, thi] (hierarchy scenes).
//
// Self tests. A camera ray's closest hit on a static box B sits at P = fl32(o + d t32),
// within delta <= 2^-23 (|P| + |o|) + 2^-24 |P| (the roundings of t32, d t32 and the sum)
// of the exact ray point at the reference's entry t, which lies on B's boundary. A shadow
// ray P + t D can then enter B only at t <= delta / |D_a| for an axis a with P outside B's
// slab (inside B every slab entry is <= 0), so B occludes it only if delta / min |D_a|
// (over D_a != 0) exceeds 1e-4. self_boxes marks the boxes where 2^-21 (|P|max + |o|max)
// -- twice the bound -- stays below 1e-4 min |D_a| / 2: their own shadow test cannot pass
// for such a hit point and is skipped. omax bounds |o| of the camera's sample origins
// (camera_origin_bound).
// rects != nullptr: the cells are left to the device (k_dsg_fill) -- `cells` stays empty,
// *rects gets each object's cell rectangle and *ncells the grids' total cell count.
bool dir_shadow_grids(const HostScene& H, const std::vector<DBound>& nb, double tlo, double thi,
                      std::vector<DSGrid>& grids, std::vector<DSCell>& cells, std::vector<DSRect>* rects = nullptr,
                      size_t* ncells = nullptr) {
    grids.assign(H.lights.size(), DSGrid{});
    cells.clear();
    if (rects) rects->clear();
    size_t ncell = 0;
    struct Ob {
        double lo[3], hi[3];  // bounding box
        double c[3], r;       // a static sphere: centre and radius (r < 0: a box)
        double fuzz;          // the sphere discriminant's fuzz applies (spheres, moving ones too)
        uint32_t bit, root;   // DSCell bits
    };
    std::vector<Ob> obs;
    uint32_t always = 0, always_root = 0;
    double R = 0.0;  // the largest |coordinate| of the gridded bounds
    auto keep = [&](Ob& o) {
        for (int a = 0; a < 3; ++a) R = std::max(R, std::max(std::fabs(o.lo[a]), std::fabs(o.hi[a])));
        obs.push_back(o);
    };
    for (int32_t k = 0; k < H.n_sphere + H.n_box; ++k) {
        const bool sphere = k < H.n_sphere;
        const DObj& ob = H.objs[H.n_plane + k];
        const int32_t j = sphere ? k : k - H.n_sphere;
        const uint32_t bit = 1u << ((sphere ? 0 : 16) + (j & 15));
        Ob o{};
        o.bit = bit;
        o.fuzz = sphere ? 1.0 : 0.0;
        o.r = sphere && !ob.has_speed ? ob.radius : -1.0;
        for (int a = 0; a < 3; ++a) {
            double lo, hi;
            if (sphere) {
                lo = ob.a[a] - ob.radius;
                hi = ob.a[a] + ob.radius;
                o.c[a] = ob.a[a];
            } else {
                lo = std::min((double)ob.a[a], (double)ob.b[a]);
                hi = std::max((double)ob.a[a], (double)ob.b[a]);
            }
            if (ob.has_speed) {  // moved(): p + speed * time in fp32, swept over [tlo, thi]
                const double s0 = (double)ob.speed[a] * tlo, s1 = (double)ob.speed[a] * thi;
                const double pad = 1e-5 * (std::fabs(lo) + std::fabs(hi) + std::fabs(s0) + std::fabs(s1));
                lo += std::min(s0, s1) - pad;
                hi += std::max(s0, s1) + pad;
            }
            o.lo[a] = lo;
            o.hi[a] = hi;
        }
        bool ok = j < 16 && (sphere ? H.n_sphere : H.n_box) <= 16;
        for (int a = 0; a < 3; ++a) ok = ok && std::isfinite(o.lo[a]) && std::isfinite(o.hi[a]);
        if (!ok) {
            always |= bit;
            continue;
        }
        keep(o);
    }
    int32_t q = 0;
    for (int32_t r = 0; r < (int32_t)H.nodes.size() && r < (int32_t)nb.size(); r = H.nodes[r].end, ++q) {
        if (q >= 32) break;  // the device tests roots beyond the 32nd always
        const DBound& B = nb[r];
        Ob o{};
        o.root = 1u << q;
        o.r = -1.0;
        bool empty = false, finite = true;
        for (int a = 0; a < 3; ++a) {
            o.lo[a] = B.slo[a];
            o.hi[a] = B.shi[a];
            empty = empty || !(B.slo[a] <= B.shi[a]);
            finite = finite && std::isfinite(o.lo[a]) && std::isfinite(o.hi[a]);
        }
        if (empty) continue;  // shadow_intersect is false for every ray
        if (!finite) {
            always_root |= o.root;
            continue;
        }
        keep(o);
    }
    if (obs.empty()) return false;
    // A few spheres alone are cheaper to test than the cell lookup (its dependent load):
    // MirrorRefraction, four spheres, measured 1 % slower with a grid (profiles/r04/root_bins/)
    {
        const bool spheres_only = std::all_of(obs.begin(), obs.end(), [](const Ob& o) { return o.r >= 0.0; });
        if (spheres_only && (double)obs.size() < opt(OPT_DSGRID_MIN)) return false;
    }
    // 512 x 512 cells (2 MB per light): finer grids measured faster up to 512 (DepthOfField
    // 4K 5.09 -> 5.01 ms, NovelScene1 17.48 -> 16.96 ms, NovelScene2 79.2 -> 76.7 ms from 64;
    // 1024 within 0.5 %, profiles/r04/dsgrid_g/)
    const int32_t G = kDsgG;
    const double pmax = 1.25 * R + 1.0, pm = std::sqrt(3.0) * pmax;  // pm >= |p| of a gridded origin
    bool any = false;
    for (size_t li = 0; li < H.lights.size(); ++li) {
        const DLight& Lt = H.lights[li];
        if (Lt.type != LIGHT_DIRECTIONAL) continue;
        const double d[3] = {Lt.negvec[0], Lt.negvec[1], Lt.negvec[2]};
        const double dn = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
        if (!(dn > 0.0) || !std::isfinite(dn)) continue;
        // e1, e2: unit vectors across d, rounded to the fp32 values the device uses
        const double a[3] = {d[0] / dn, d[1] / dn, d[2] / dn};
        const int ax = std::fabs(a[0]) <= std::fabs(a[1]) && std::fabs(a[0]) <= std::fabs(a[2]) ? 0
                       : std::fabs(a[1]) <= std::fabs(a[2]) ? 1 : 2;
        double x[3] = {0.0, 0.0, 0.0};
        x[ax] = 1.0;
        double e1[3] = {a[1] * x[2] - a[2] * x[1], a[2] * x[0] - a[0] * x[2], a[0] * x[1] - a[1] * x[0]};
        double n1 = std::sqrt(e1[0] * e1[0] + e1[1] * e1[1] + e1[2] * e1[2]);
        float f1[3], f2[3];
        for (int q = 0; q < 3; ++q) f1[q] = (float)(e1[q] / n1);
        double e2[3] = {a[1] * f1[2] - a[2] * f1[1], a[2] * f1[0] - a[0] * f1[2], a[0] * f1[1] - a[1] * f1[0]};
        const double n2 = std::sqrt(e2[0] * e2[0] + e2[1] * e2[1] + e2[2] * e2[2]);
        for (int q = 0; q < 3; ++q) f2[q] = (float)(e2[q] / n2);
        const double g1[3] = {f1[0], f1[1], f1[2]}, g2[3] = {f2[0], f2[1], f2[2]};
        auto dot3 = [](const double* p, const double* q) { return p[0] * q[0] + p[1] * q[1] + p[2] * q[2]; };
        const double drift_rel = std::max(std::fabs(dot3(d, g1)), std::fabs(dot3(d, g2))) / dn * (1.0 + 1e-9);
        const double len1 = std::sqrt(dot3(g1, g1)), len2 = std::sqrt(dot3(g2, g2));
        // grown footprints
        std::vector<double> fp(4 * obs.size());
        double U0 = INFINITY, U1 = -INFINITY, V0 = INFINITY, V1 = -INFINITY;
        for (size_t i = 0; i < obs.size(); ++i) {
            const Ob& o = obs[i];
            double rx = 0.0;
            for (int q = 0; q < 3; ++q) rx += std::max(o.lo[q] * o.lo[q], o.hi[q] * o.hi[q]);
            rx = std::sqrt(rx);  // >= |x| of every point of the box
            double pad = (rx + pm) * drift_rel + 0x1p-18 * (rx + pm) + o.fuzz * 0x1p-8 * (pm + rx);
            double u0, u1, v0, v1;
            if (o.r >= 0.0) {
                const double cu = dot3(o.c, g1), cv = dot3(o.c, g2);
                u0 = cu - o.r * len1; u1 = cu + o.r * len1;
                v0 = cv - o.r * len2; v1 = cv + o.r * len2;
            } else {
                pad += 1e-5 * (pm + rx);
                u0 = v0 = INFINITY;
                u1 = v1 = -INFINITY;
                for (int q = 0; q < 8; ++q) {
                    const double p[3] = {q & 1 ? o.hi[0] : o.lo[0], q & 2 ? o.hi[1] : o.lo[1], q & 4 ? o.hi[2] : o.lo[2]};
                    const double pu = dot3(p, g1), pv = dot3(p, g2);
                    u0 = std::min(u0, pu); u1 = std::max(u1, pu);
                    v0 = std::min(v0, pv); v1 = std::max(v1, pv);
                }
            }
            double* F = &fp[4 * i];
            F[0] = u0 - pad; F[1] = u1 + pad; F[2] = v0 - pad; F[3] = v1 + pad;
            U0 = std::min(U0, F[0]); U1 = std::max(U1, F[1]);
            V0 = std::min(V0, F[2]); V1 = std::max(V1, F[3]);
        }
        if (!std::isfinite(U0 + U1 + V0 + V1)) continue;
        // two spare cells a side: the device's rounding cannot carry an origin from off the
        // grid into a footprint
        const double wu = (U1 - U0) * (1.0 + 1e-6) + 1e-9, wv = (V1 - V0) * (1.0 + 1e-6) + 1e-9;
        DSGrid g{};
        for (int q = 0; q < 3; ++q) { g.e1[q] = f1[q]; g.e2[q] = f2[q]; }
        g.G = G;
        g.pmax = (float)pmax;
        if ((double)g.pmax > pmax) g.pmax = std::nextafter(g.pmax, 0.0f);
        g.su = (float)((G - 4) / wu);
        g.sv = (float)((G - 4) / wv);
        g.u0 = (float)(U0 - 2.0 / g.su);
        g.v0 = (float)(V0 - 2.0 / g.sv);
        g.off = (int32_t)ncell;
        g.always = always;
        g.always_root = always_root;
        ncell += (size_t)G * G;
        if (!rects) cells.resize(ncell, DSCell{0u, 0u});
        auto cell = [&](double u, double o0, double s) {  // as the device maps it, +-1 below
            return (int32_t)std::floor((u - o0) * s);
        };
        for (size_t i = 0; i < obs.size(); ++i) {
            const double* F = &fp[4 * i];
            const int32_t i0 = std::max(0, cell(F[0], g.u0, g.su) - 1), i1 = std::min(G - 1, cell(F[1], g.u0, g.su) + 1);
            const int32_t j0 = std::max(0, cell(F[2], g.v0, g.sv) - 1), j1 = std::min(G - 1, cell(F[3], g.v0, g.sv) + 1);
            if (rects) {
                if (i0 <= i1 && j0 <= j1) rects->push_back(DSRect{g.off, i0, i1, j0, j1, obs[i].bit, obs[i].root, 0u});
                continue;
            }
            for (int32_t jy = j0; jy <= j1; ++jy)
                for (int32_t ix = i0; ix <= i1; ++ix) {
                    DSCell& c = cells[(size_t)g.off + (size_t)jy * G + ix];
                    c.obj |= obs[i].bit;
                    c.root |= obs[i].root;
                }
        }
        grids[li] = g;
        any = true;
    }
    if (ncells) *ncells = ncell;
    return any;
}

// The self-test marks of the grids (DSGrid.self_boxes, see above): per camera, as they
// depend on omax (camera_origin_bound); the grids and their cells depend on the frame's
// time range only.
void dir_self_boxes(const HostScene& H, std::vector<DSGrid>& grids, double omax) {
    for (size_t li = 0; li < grids.size() && li < H.lights.size(); ++li) {
        DSGrid& g = grids[li];
        g.self_boxes = 0u;
        if (g.G == 0 || H.n_box > 16 || !std::isfinite(omax) || !opt_on(OPT_SELF_SKIP)) continue;
        const DLight& Lt = H.lights[li];
        double dmin = INFINITY;
        for (int q = 0; q < 3; ++q)
            if (Lt.negvec[q] != 0.0f) dmin = std::min(dmin, std::fabs((double)Lt.negvec[q]));
        for (int32_t k = 0; k < H.n_box; ++k) {
            const DObj& ob = H.objs[H.n_plane + H.n_sphere + k];
            if (ob.has_speed) continue;
            double pm = 0.0;
            for (int q = 0; q < 3; ++q) {
                const double m = std::max(std::fabs((double)ob.a[q]), std::fabs((double)ob.b[q]));
                pm += m * m;
            }
            const double delta = 0x1p-21 * (std::sqrt(pm) + omax);
            if (2.0 * delta < 1e-4 * dmin) g.self_boxes |= 1u << (16 + k);
        }
    }
}

}  // namespace

// ------------------------------------------------------------------ scene-specialized kernels
// k_render loops over the scene's planes, spheres, boxes, meshes and lights with counts
// read at run time; with the counts as compile-time constants the loops unroll and every
// scene record is loaded up front (TSP 1080p: 57.9 -> 39.7 us/frame). rtx_render
// therefore compiles, once per process and scene shape, render_body with those counts
// pinned (hiprtc, same flags as the library; the code object is also cached on disk,
// $RTX_JIT_CACHE or /tmp/rtx_jit_<uid>). Results are identical: only loop bounds become
// constants. RTX_JIT=0 keeps the generic kernels.
#include "rtx_jit_sources.inc"

namespace {

// Scene properties the specialized kernels pin (from the converted records).
struct SceneTraits {
    int fc_mode = 0;              // RTX_FACE_CULL_MODE of the top-level meshes: 0 none, 1 all, 2 mixed
    bool any_speed = false;       // some top-level object moves (else the JIT pins a static scene)
    uint32_t light_dir_mask = 0;  // bit i: light i is directional (JIT, <= 8 lights)
    int32_t uniform_hard = -1;    // >= 0: every specular lobe's integer hardness (JIT)
};
SceneTraits scene_traits(const HostScene& H) {
    SceneTraits t;
    int n_fc = 0, n_m = 0;
    for (const DObj& o : H.objs)
        if (o.type == RTX_MESH) { ++n_m; n_fc += o.face_cull ? 1 : 0; }
    t.fc_mode = n_fc == 0 ? 0 : n_fc == n_m ? 1 : 2;
    for (const DObj& o : H.objs) t.any_speed = t.any_speed || o.has_speed;
    t.uniform_hard = H.uniform_hard >= 0 ? H.uniform_hard : -1;
    for (size_t i = 0; i < H.lights.size() && i < 32; ++i)
        if (H.lights[i].type == LIGHT_DIRECTIONAL) t.light_dir_mask |= 1u << i;
    return t;
}

struct JitEntry {
    hipModule_t mod = nullptr;
    hipFunction_t fn = nullptr;
    bool baked = false;  // the source carries one scene's record values (jit_baked_records)
    int refs = 0;        // scenes whose resolved kernels hold it
};
std::mutex g_jit_mu;
std::map<std::string, JitEntry> g_jit;
// Kernels with baked records belong to one scene's values, so they are not kept for the
// life of the process: once no scene holds one it joins an idle list, and beyond
// kJitIdleBaked idle modules the oldest is unloaded (its scenes' buffers were freed with
// hipFree, which waits for their kernels). The disk cache keeps at most kJitDiskBaked
// baked code objects (rtx_b_*.co, oldest removed first).
// (options jit_idle_baked / jit_disk_baked set the caps, 8 and 64; the tests lower them.)
size_t jit_cap(Opt o) { return (size_t)std::max(0.0, opt(o)); }
std::list<std::string> g_jit_idle;  // baked keys with refs == 0, oldest first

// A scene drops its hold on a resolved kernel (camera change or rtx_scene_destroy).
void jit_release(const std::string& key) {
    if (key.empty()) return;
    std::lock_guard<std::mutex> lock(g_jit_mu);
    auto it = g_jit.find(key);
    if (it == g_jit.end() || --it->second.refs > 0 || !it->second.baked) return;
    g_jit_idle.push_back(key);
    const size_t cap = jit_cap(OPT_JIT_IDLE_BAKED);
    while (g_jit_idle.size() > cap) {
        auto old = g_jit.find(g_jit_idle.front());
        g_jit_idle.pop_front();
        if (old == g_jit.end() || old->second.refs > 0) continue;
        (void)hipModuleUnload(old->second.mod);
        g_jit.erase(old);
    }
}

// Keeps the newest kJitDiskBaked baked code objects of the disk cache.
void jit_prune_disk(const std::string& dir) {
    DIR* d = opendir(dir.c_str());
    if (!d) return;
    std::vector<std::pair<time_t, std::string>> files;
    while (dirent* e = readdir(d)) {
        const std::string n = e->d_name;
        if (n.rfind("rtx_b_", 0) != 0 || n.size() < 3 || n.compare(n.size() - 3, 3, ".co") != 0) continue;
        struct stat st;
        const std::string path = dir + "/" + n;
        if (lstat(path.c_str(), &st) == 0 && S_ISREG(st.st_mode)) files.emplace_back(st.st_mtime, path);
    }
    closedir(d);
    const size_t cap = jit_cap(OPT_JIT_DISK_BAKED);
    if (files.size() <= cap) return;
    std::sort(files.begin(), files.end());
    for (size_t i = 0; i + cap < files.size(); ++i) (void)unlink(files[i].second.c_str());
}

// Sample-parallel mapping (render_body_spp) for the hierarchy/texture kernels when a
// pixel has >= spp_min samples (option, default 16): a wave then traces one pixel's nearly
// identical AA/time samples, so the wave-uniform subtree culling stays effective
// (NovelScene1 108 -> 30 ms, NovelScene2 741 -> 161 ms). The flat-scene kernels keep
// the 8x8-tile mapping, whose waves are already coherent (same lens sample across a
// tile; DepthOfField 4K: 11.1 ms tiles vs 19.3 ms sample-parallel). Option spp: 0 never
// uses it, 1 always (tests compare both mappings).
bool use_spp_mode(int spp, bool ext) {
    if (spp < 1 || spp >= (1 << 20)) return false;  // udiv_small's range
    const double m = opt(OPT_SPP);
    if (m == 0.0) return false;
    if (m == 1.0) return true;
    return ext && spp >= opt(OPT_SPP_MIN);
}

// Host-computed origin terms of primary rays (RTX_PRIM_ORIGIN kernels; option prim_origin).
bool prim_origin_enabled() { return opt_on(OPT_PRIM_ORIGIN); }

// The measured tile schedule (tile_schedule; option tile_sched).
bool tile_sched_enabled() { return opt_on(OPT_TILE_SCHED); }
// Threads per block of a scene-specialized tile-mapped kernel (one 8x8 tile per wave).
// The secondary-ray and mesh kernels -- the tile-scheduled kinds, whose waves differ most in
// length -- run in one-wave blocks (option tile_block, 64 or 256): MirrorRefraction 36.7 ->
// 35.9 us, TorusMesh 47.4 -> 46.4 us; TwoSpheresPlane keeps 256 (64: 21.9 -> 22.3 us;
// profiles/r05/noslp/abl_block_*.log).
int jit_block(bool mesh, bool sec, bool ext, bool spp) {
    if (ext) return kBlock<true>;
    if (spp || !(mesh || sec)) return kBlock<false>;
    return opt(OPT_TILE_BLOCK) == 64.0 ? 64 : kBlock<false>;
}

bool jit_enabled() { return opt_on(OPT_JIT); }

// The on-disk code-object cache: option jit_cache or /tmp/rtx_jit_<uid>, created with
// mkdir(2) mode 0700. It is used only when it is a real directory (not a symlink) owned
// by this user and not writable by group or others; otherwise another local user could
// plant code objects under the predictable names, so kernels are compiled uncached.
// Returns "" when the cache must not be used.
std::string jit_cache_dir() {
    const std::string e = opt_str(OPT_JIT_CACHE);
    const std::string dir = !e.empty() ? e : "/tmp/rtx_jit_" + std::to_string((long)getuid());
    (void)mkdir(dir.c_str(), 0700);
    struct stat st;
    if (lstat(dir.c_str(), &st) != 0 || !S_ISDIR(st.st_mode) || st.st_uid != getuid() ||
        (st.st_mode & (S_IWGRP | S_IWOTH)) != 0)
        return "";
    return dir;
}

// The library's own compile-time experiment knobs (rtx_kernels.h / rtx_trace.h defaults or
// -D overrides of this build), forwarded to hiprtc so a specialized kernel is built with
// the same block size, tiling and launch bounds the host launches it with; they are part
// of the cache key through the option list.
#define RTX_STR2(x) #x
#define RTX_STR(x) RTX_STR2(x)
const char* const kLibMacros[] = {
    "-DRTX_TILE=" RTX_STR(RTX_TILE),
    "-DRTX_PPL=" RTX_STR(RTX_PPL),
    "-DRTX_BLOCK_FLAT=" RTX_STR(RTX_BLOCK_FLAT),
    "-DRTX_LB_XWAVES=" RTX_STR(RTX_LB_XWAVES),
    "-DRTX_LB_WAVES(MESH,SEC)=" RTX_STR(RTX_LB_WAVES(MESH, SEC)),
    "-DRTX_ABLATE=" RTX_STR(RTX_ABLATE),
#if defined(RTX_TOOLS_BUILD)
    "-DRTX_TOOLS_BUILD",
#endif
    "-DRTX_HIER_INLINE=" RTX_STR(RTX_HIER_INLINE),
    "-DRTX_HEAVY_CHUNK=" RTX_STR(RTX_HEAVY_CHUNK),
#ifdef RTX_PAD
    "-DRTX_PAD=" RTX_STR(RTX_PAD),
#endif
};
#undef RTX_STR
#undef RTX_STR2

// gfx arch of a device ordinal, resolved once per device.
std::string device_arch(int device) {
    static std::mutex mu;
    static std::map<int, std::string> archs;
    std::lock_guard<std::mutex> lock(mu);
    auto it = archs.find(device);
    if (it != archs.end()) return it->second;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return "";
    std::string arch = prop.gcnArchName;
    arch = arch.substr(0, arch.find(':'));
    archs[device] = arch;
    return arch;
}

// Returns the specialized kernel, or nullptr (the caller then launches the generic one)
// and its name in *name_out. Modules are loaded per device: the in-memory cache key
// carries the device ordinal (a hipFunction_t belongs to the device it was loaded on);
// the on-disk code object depends on the arch only.
// The scene's object, material and light records as constant arrays of the specialized
// kernel's source (rtx_kernels.h RTX_BAKED_RECORDS): the bytes rtx_scene_create uploads,
// as 32-bit words. The kernel then depends on the records' values, not only on the scene's
// shape: a changed scene is a new rtx_scene and compiles (or loads from the code-object
// cache) its own kernel. RTX_JIT_BAKE=0 keeps the records in device memory.
template <class T>
void baked_array(std::string& out, const char* name, const std::vector<T>& v) {
    static_assert(sizeof(T) % 4 == 0, "records are whole 32-bit words");
    out += "alignas(16) static constexpr unsigned ";
    out += name;
    out += "[] = {";
    std::vector<uint32_t> w(v.size() * sizeof(T) / 4);
    if (!v.empty()) memcpy(w.data(), v.data(), w.size() * 4);
    if (w.empty()) w.push_back(0u);  // (never read: the scene has no such record)
    char buf[16];
    for (uint32_t x : w) {
        snprintf(buf, sizeof(buf), "0x%xu,", x);
        out += buf;
    }
    out += "};\n";
}
std::string jit_baked_records(const std::vector<DObj>& objs, const std::vector<DMat>& mats,
                              const std::vector<DLight>& lights) {
    std::string s = "namespace rtx_baked {\n";
    baked_array(s, "kObjs", objs);
    baked_array(s, "kMats", mats);
    baked_array(s, "kLights", lights);
    return s + "}\n#define RTX_BAKED_RECORDS 1\n";
}

bool jit_bake_enabled() { return opt_on(OPT_JIT_BAKE); }

// What a scene-specialized kernel is built from: its name, hiprtc source and options.
struct JitSpec {
    std::string name, src;
    std::vector<std::string> opts;
    bool baked = false;  // the source carries the scene's record values
};

// What the scene-specialized kernels pin of a scene (object and light counts, static
// scene, light kinds, pow loop length, a uniform integer hardness) and -- camera -- of its
// camera (sample counts: the 1-spp loops vanish; divisor kind, jitter mode).
void jit_fixed_opts(const SceneView& v, const KParams& kp, const SceneTraits& tr, bool camera,
                    std::vector<std::string>& opts) {
    for (const std::string& o :
         {std::string("-DRTX_FIXED_COUNTS"), "-DRTX_FIXED_NP=" + std::to_string(v.n_plane),
          "-DRTX_FIXED_NS=" + std::to_string(v.n_sphere), "-DRTX_FIXED_NB=" + std::to_string(v.n_box),
          "-DRTX_FIXED_NM=" + std::to_string(v.n_mesh), "-DRTX_FIXED_NL=" + std::to_string(v.n_lights),
          "-DRTX_FACE_CULL_MODE=" + std::to_string(tr.fc_mode),
          "-DRTX_FIXED_STATIC=" + std::to_string(tr.any_speed ? 0 : 1),
          "-DRTX_FIXED_LDIR=" + std::to_string(tr.light_dir_mask) + "u",
          "-DRTX_FIXED_POWBITS=" + std::to_string(v.pow_bits)})
        opts.push_back(o);
    if (tr.uniform_hard >= 0) opts.push_back("-DRTX_FIXED_HARD=" + std::to_string(tr.uniform_hard));
    if (!camera) return;
    for (const std::string& o :
         {std::string("-DRTX_FIXED_SAMPLES"), "-DRTX_FIXED_NDOF=" + std::to_string(kp.n_dof),
          "-DRTX_FIXED_NAA=" + std::to_string(kp.n_aa), "-DRTX_FIXED_NTIMES=" + std::to_string(kp.n_times),
          "-DRTX_FIXED_DIVPOW2=" + std::to_string(kp.div_pow2), "-DRTX_FIXED_JMODE=" + std::to_string(kp.jitter)})
        opts.push_back(o);
}

// The specialized kernel of a scene and camera for arch (false: the generic kernel runs).
// Host code only, so the tests' host build can print it (tools/jit_offline.py compiles it
// to ISA without a GPU).
bool jit_spec(const std::string& arch, const SceneView& v, const KParams& kp, const SceneTraits& tr, bool mesh,
              bool sec, bool ext, bool cnt, bool jit, bool spp, bool out8, const std::string& baked, JitSpec& out) {
    const int fc_mode = tr.fc_mode;
    if (v.n_plane + v.n_sphere + v.n_box + v.n_mesh > 32 || v.n_lights > 8) return false;  // code size
    // CSG/texture kernels: the unrolled loops raise their (already high) register
    // pressure and the specialized kernel measured slower (NovelScene1 105 -> 134 ms)
    if (ext && !opt_on(OPT_JIT_EXT)) return false;  // (option jit_ext: specialize them anyway)
    // -fno-slp-vectorize: the SLP pass packs pairs of scalar f32 operations into v_pk_*_f32,
    // which on gfx950 issue at the cost of the two scalar operations and add the v_mov that
    // gather their register pairs; without it the kernels need fewer VGPRs (TwoSpheresPlane
    // 68 -> 62: 8 waves/SIMD instead of 7; TorusMesh and DepthOfField lose their scratch
    // spills) and run faster: TSP 1080p 24.1 -> 21.5 us, MirrorRefraction 40.2 -> 38.3 us,
    // TorusMesh 48.9 -> 46.7 us, DepthOfField 4K 4.62 -> 4.38 ms (profiles/r05/noslp/).
    std::vector<std::string> opts = {"--offload-arch=" + arch, "-O3", "-std=c++17", "-ffp-contract=off",
                                     "-fno-slp-vectorize"};
    jit_fixed_opts(v, kp, tr, true, opts);
    // the strip width too: the tile index arithmetic becomes multiplications by constants
    // (TSP 1080p 27.85 -> 27.37 us, profiles/r03/ncols/; one compile per strip width)
    if (!spp) opts.push_back("-DRTX_FIXED_NCOLS=" + std::to_string(kp.ncols));
    if (!spp && !ext && kp.tile_time != nullptr) opts.push_back("-DRTX_TILE_SCHED=1");
    if (!spp && !ext && kp.po_valid) opts.push_back("-DRTX_PRIM_ORIGIN=1");
    if (out8) opts.push_back("-DRTX_OUT8=1");  // uint8 framebuffer (rtx_render_rgb8)
    // secondary-ray frames keep their material index in a register: 3 LDS words per frame
    if (sec && v.n_mats <= 64) opts.push_back("-DRTX_FRAME_MATBITS=6");
    if (sec && !mesh && !ext) {
        opts.push_back("-DRTX_DEFER_TIES=1");  // (rtx_trace.h closest_hit)
        // hit_t64 inlined (no call in the kernel): MirrorRefraction 35.7 -> 35.3 us; the
        // other kernels measured slower with it (TSP +2.3 %, TM +1.8 %, DOF +1.2 %,
        // profiles/r05/noslp/ab_t64_inline.log)
        opts.push_back("-DRTX_HIT_T64_INLINE=1");
        opts.push_back("-DRTX_TIE_CALL=1");  // (rtx_trace.h tie_takes)
        // the frames of chain levels 0-5 in LDS (18 KB per block with 3-word frames), deeper
        // ones in scratch, at <= 72 VGPRs: 7-8 blocks per CU instead of 5.
        // MirrorRefraction 38.7 -> 36.4 us (twice on one box; levels 8/7/5/4/3 and 6-8 waves
        // within 36.4-37.2 us, profiles/r05/noslp/ab_frame_levels*.log). Round 4 measured
        // 8 levels at 6 waves equal: the SLP-free build (§6q) has the registers for it.
        opts.push_back("-DRTX_FRAME_LDS_LEVELS=6");
        opts.push_back("-URTX_LB_WAVES");
        opts.push_back("-DRTX_LB_WAVES(MESH,SEC)=7");
    }
    opts.push_back(std::string("-DRTX_PRIMARY_BINS=") + (kp.S.bins_on ? "1" : "0"));
    // a mesh's face bins read through LDS (rtx_trace.h BinLds; option bin_lds)
    if (mesh && !ext && kp.S.bins_on && kp.S.mesh_bins && opt_on(OPT_BIN_LDS)) opts.push_back("-DRTX_BIN_LDS=1");
    opts.push_back(std::string("-DRTX_LIGHT_GRIDS=") + (v.lgrid_on ? "1" : "0"));
    opts.push_back(std::string("-DRTX_DIR_GRIDS=") + (kp.S.dsg_on ? "1" : "0"));
    // (records and mesh data staged in LDS -- RTX_LDS_OBJS / RTX_LDS_TRIS kernels -- measured
    // slower; jit_flags can still request them)
    for (const char* m : kLibMacros) opts.push_back(m);
    if (!ext && jit_block(mesh, sec, ext, spp) != kBlock<false>) {
        opts.push_back("-URTX_BLOCK_FLAT");
        opts.push_back("-DRTX_BLOCK_FLAT=" + std::to_string(jit_block(mesh, sec, ext, spp)));
    }
    if (!sec && !ext && (!mesh || fc_mode == 1)) {
        // flat scenes and small meshes (every face box-culled): 6 waves/SIMD. With the
        // host-side box precomputes the DepthOfField kernel fits 80 VGPRs with no more
        // scratch than at 5: DepthOfField 4K 6.60 -> 6.28 ms, TorusMesh 1080p 54.6 -> 52.1 us,
        // twice on one box; 7 and 8 waves are slower (6.60 / 6.89 ms; profiles/r03/lb6/). (Round 2:
        // small meshes 4 -> 5 waves, 70.2 -> 66.2 us.) The 81,920-face mesh, which has no face
        // boxes, keeps the mesh kernels' 4 (1.4 % slower at 5).
        opts.push_back("-URTX_LB_WAVES");
        opts.push_back("-DRTX_LB_WAVES(MESH,SEC)=6");
    }
    // one-sample flat scenes of primary and shadow rays: the scheduler's max-ILP strategy
    // (TwoSpheresPlane 22.2 -> 22.0 us, three times on one box; MirrorRefraction within
    // noise either way; it spills the mesh and multi-sample kernels' registers: TorusMesh
    // +7 %, DepthOfField +8 %; profiles/r05/noslp/ab_sched_unroll.log, ab_ilp.log)
    // With them, the kernel arguments preloaded into SGPRs (one dependent scalar load fewer
    // at every wave's start: TwoSpheresPlane 22.08 -> 21.91 us, twice on one box,
    // profiles/r05/noslp/ab_kernarg.log).
    if (!mesh && !ext && !sec && kp.n_dof * kp.n_aa * kp.n_times == 1 && opt_on(OPT_JIT_ILP)) {
        opts.push_back("-mllvm");
        opts.push_back("-amdgpu-sched-strategy=max-ilp");
        opts.push_back("-mllvm");
        opts.push_back("-amdgpu-kernarg-preload-count=16");
    }
    {  // option jit_flags (tools: cost probes, occupancy bounds); part of the cache key
        std::istringstream is(opt_str(OPT_JIT_FLAGS));
        for (std::string o; is >> o;) opts.push_back(o);
    }
    auto b = [](bool x) { return x ? "true" : "false"; };
    // kernel name: rtx_jit_render_<mesh><sec><ext><count><jitter> (tells profiles apart)
    std::string name = "rtx_jit_render_";
    for (bool f : {mesh, sec, ext, cnt, jit}) name += f ? '1' : '0';
    // the parity-mode jitter (replayed noise table) is a different specialization from the
    // production Philox one: the name says which ran
    if (jit && kp.jitter == RTX_JITTER_REPLAY) name += "_replay";
    if (spp) name += "_spp";
    if (out8) name += "_rgb8";
    // one-sample flat-scene kernels: the scene records as literals (jit_baked_records).
    // MirrorRefraction 1080p 49.4 -> 44.3 us, TorusMesh 65.3 -> 60.1, TwoSpheresPlane equal
    // (profiles/r03/bake/). Multi-sample kernels keep reading them per sample
    // (RTX_RELOAD_RECORDS): baked, DepthOfField 4K slows 7.0 -> 9.8 ms.
    const bool one_sample = kp.n_dof * kp.n_aa * kp.n_times == 1;
    const std::string prelude = (!ext && !spp && one_sample && jit_bake_enabled()) ? baked : std::string();
    // (The frame parameters stay behind a pointer: passed by value in the kernel arguments,
    // one dependent scalar load fewer per wave, they measured equal on TSP/MR/TM,
    // profiles/r04/kp_byval/.)
    // (a product library's kernels are never cost-probe builds, whatever jit_flags say)
#if defined(RTX_TOOLS_BUILD)
    const std::string tools_guard;
#else
    const std::string tools_guard = "#undef RTX_TOOLS_BUILD\n";
#endif
    const std::string src = tools_guard + prelude + std::string("#include \"rtx_kernels.h\"\nextern \"C\" __global__ RTX_RENDER_BOUNDS(") +
                            b(mesh) + ", " + b(sec) + ", " + b(ext) + ") void " + name + "(const rtx::KParams* "
                            "__restrict__ P, const rtx::Launch L) {\n  rtx::" + (spp ? "render_body_spp<" : "render_body<") +
                            b(mesh) + ", " + b(sec) +
                            ", " + b(ext) + ", " + b(cnt) + ", " + b(jit) + ">(P, L);\n}\n";
    out.name = name;
    out.src = src;
    out.opts = opts;
    out.baked = !prelude.empty();
    return true;
}

// A hierarchy scene's node table as the compile-time constants of the specialized split
// passes (rtx_trace.h namespace csg: the traversals unrolled over the trees, node fields and
// matrices as literals). "" when the scene does not qualify: a difference with fewer than
// two children, a non-finite matrix, or trees whose unrolled traversals would be large
// (csg_cost: node visits of the unrolled code, a deep tree's walk-ups repeat its siblings).
constexpr int64_t kCsgMaxNodes = 512, kCsgMaxCost = 6000;
int64_t csg_cost(const std::vector<DNode>& N) {
    auto kids = [&](int x, const std::function<void(int)>& f) {
        for (int j = x + 1; j < N[x].end; j = N[j].end) f(j);
    };
    std::function<int64_t(int)> inside = [&](int x) -> int64_t {
        int64_t c = 1;
        if (N[x].kind != HN_LEAF && N[x].kind != HN_OTHER) kids(x, [&](int j) { c += inside(j); });
        return c;
    };
    std::function<int64_t(int)> material = [&](int x) -> int64_t {
        int64_t c = 1;
        if (N[x].kind != HN_LEAF) kids(x, [&](int j) { c += inside(j) + material(j); });
        return c;
    };
    auto walk = [&](int cur, int stop) {
        int64_t c = 0;
        for (; cur != stop; cur = N[cur].parent) {
            const int a = N[cur].parent;
            if (N[a].kind == HN_INTER || N[a].kind == HN_DIFF) {
                kids(a, [&](int j) { if (j != cur) c += inside(j); });
                if (N[a].kind == HN_DIFF && N[cur].cidx != 0) c += material(a + 1);
            }
            ++c;
        }
        return c;
    };
    std::function<int64_t(int, int)> enumerate = [&](int x, int root) -> int64_t {
        if (N[x].kind == HN_LEAF) return 1 + walk(x, root);
        int64_t c = 1;
        kids(x, [&](int j) { c += enumerate(j, root); });
        return c;
    };
    int64_t total = (int64_t)N.size();  // (the shadow walk)
    for (int r = 0; r < (int)N.size(); r = N[r].end) total += enumerate(r, r);
    for (int i = 0; i < (int)N.size(); ++i)
        if (N[i].kind == HN_DIFF) {
            const int c0 = i + 1, c1 = N[c0].end;
            total += enumerate(c0, c0) + enumerate(c1, c1) + inside(c0) + inside(c1);
        }
    return total;
}
std::string jit_csg_tables(const std::vector<DNode>& N) {
    if (N.empty() || (int64_t)N.size() > kCsgMaxNodes) return "";
    for (size_t i = 0; i < N.size(); ++i) {
        const DNode& d = N[i];
        if (d.kind == HN_DIFF && (i + 1 >= (size_t)d.end || N[i + 1].end >= d.end)) return "";
        for (int k = 0; k < 16; ++k)
            if (!std::isfinite(d.M[k]) || !std::isfinite(d.Minv[k])) return "";
    }
    if (csg_cost(N) > kCsgMaxCost) return "";
    std::string s = "namespace rtx_csg {\nstruct CNode {\n    int kind, parent, cidx, depth, end, pkind, obj, mat0, oid;\n};\n";
    s += "constexpr int kCount = " + std::to_string(N.size()) + ";\nconstexpr CNode kNode[] = {";
    char buf[160];
    for (const DNode& d : N) {
        snprintf(buf, sizeof(buf), "{%d,%d,%d,%d,%d,%d,%d,%d,%d},", d.kind, d.parent, d.cidx, d.depth, d.end, d.pkind,
                 d.obj, d.mat0, d.oid);
        s += buf;
    }
    auto mats = [&](const char* name, bool inv) {  // hexadecimal float literals: exact
        s += std::string("};\nconstexpr float ") + name + "[][16] = {";
        for (const DNode& d : N) {
            s += "{";
            for (int k = 0; k < 16; ++k) {
                snprintf(buf, sizeof(buf), "%af,", (double)(inv ? d.Minv[k] : d.M[k]));
                s += buf;
            }
            s += "},";
        }
    };
    mats("kM", false);
    mats("kMinv", true);
    return s + "};\n}  // namespace rtx_csg\n#define RTX_CSG_STATIC 1\n";
}

// The camera's node boxes (option jit_csg 2) and the scene's object records (3) for the
// specialized split passes (rtx_trace.h csg::hbox / obj, RTX_CSG_BAKED 2 / 3): the bytes
// the camera and scene uploads hold. Measured slower: with both, NovelScene1 11.4 -> 48.7 ms
// (the literals' live ranges spill 429 VGPRs, profiles/r06/s14/).
std::string jit_csg_baked(const std::vector<DBound>& bounds, const std::vector<DObj>& objs, int level) {
    std::string s = "namespace rtx_csg {\n";
    baked_array(s, "kBoxes", split_bounds(bounds));
    if (level >= 3) baked_array(s, "kObjs", objs);
    return s + "}  // namespace rtx_csg\n#define RTX_CSG_BAKED " + std::to_string(level) + "\n";
}

// The split pass kernel specialized on a node table (rtx_split.h split_trace / split_shadow,
// with the static traversals): the library's own kernel build otherwise.
JitSpec jit_split_spec(const std::string& arch, const std::string& tables, bool mesh, bool sec, bool cnt, bool jit,
                       int pass, bool rayreg, const std::vector<std::string>& fixed) {
    JitSpec sp;
    sp.opts = {"--offload-arch=" + arch, "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize"};
    // the scene's counts (jit_fixed_opts; NovelScene1 11.41 -> 11.31 ms, profiles/r06/s17/ f1).
    // Not the camera's: 11.18 ms, but then every camera with other sample counts compiles
    // its own ~20 s pair of passes (the GPU suite's NovelScene cameras: 8.7 -> 13+ min)
    sp.opts.insert(sp.opts.end(), fixed.begin(), fixed.end());
    for (const char* m : kLibMacros) sp.opts.push_back(m);
    // rays in registers, or the LDS stack (option csg_rays; the launch sizes the LDS from it)
    sp.opts.push_back(rayreg ? "-DRTX_CSG_RAYREG=1" : "-DRTX_CSG_RAYREG=0");
    // the shadow pass with its rays in registers: at most 128 VGPRs (4 waves/SIMD), which its
    // precompiled form's LDS stack had imposed (1 wave bound: 129 VGPRs, NovelScene1 13.35 ms
    // against 11.36 bounded, profiles/r06/s13/)
    if (pass == 1 && rayreg) {
        sp.opts.push_back("-URTX_LB_SPLIT_B");
        sp.opts.push_back("-DRTX_LB_SPLIT_B=4");
    }
    {
        std::istringstream is(opt_str(OPT_JIT_FLAGS));
        for (std::string o; is >> o;) sp.opts.push_back(o);
    }
    auto b = [](bool x) { return x ? "true" : "false"; };
    std::string args = std::string("<") + b(mesh);
    if (pass == 0) {
        sp.name = "rtx_jit_split_trace_";
        for (bool f : {mesh, sec, cnt, jit}) sp.name += f ? '1' : '0';
        args += std::string(", ") + b(sec) + ", " + b(cnt) + ", " + b(jit) + ">";
    } else if (pass == 2) {
        sp.name = "rtx_jit_split_shade_";
        for (bool f : {mesh, sec}) sp.name += f ? '1' : '0';
        args += std::string(", ") + b(sec) + ">";
    } else {
        sp.name = "rtx_jit_split_shadow_";
        for (bool f : {mesh, cnt}) sp.name += f ? '1' : '0';
        args += std::string(", ") + b(cnt) + ">";
    }
#if defined(RTX_TOOLS_BUILD)
    const std::string tools_guard;
#else
    const std::string tools_guard = "#undef RTX_TOOLS_BUILD\n";
#endif
    sp.src = tools_guard + tables + "#include \"rtx_split.h\"\nextern \"C\" __global__ __launch_bounds__(rtx::kBlock<true>, " +
             (pass == 0 ? "RTX_LB_SPLIT_A" : pass == 1 ? "RTX_LB_SPLIT_B" : "5") + ") void " + sp.name +
             "(const rtx::KParams* __restrict__ Pp, const rtx::Launch L, rtx::SplitBuf sb) {\n  rtx::" +
             (pass == 0 ? "split_trace" : pass == 1 ? "split_shadow" : "split_shade") + args + "(Pp, L, sb);\n}\n";
    sp.baked = true;  // (the scene's own kernel: pruned from memory and disk as the baked ones)
    return sp;
}

// Scene-specialized kernels compiled on a host thread (option jit_async, the default): a
// scene's first frames render with the precompiled generic kernel -- the same bytes
// (tests/test_gpu_parity.py test_scene_specialized_kernel_equals_generic) -- while hiprtc
// compiles (~0.3 s), and the render that finds the compile done loads and launches the
// specialized kernel (jit_poll). A cold process's first TwoSpheresPlane 1080p frame then
// costs a generic launch instead of a compile. rtx_jit_wait blocks until they are ready
// (bench.py's timed region, graph captures). One compile at a time (g_compile_mu); the
// jobs of a key are shared by the scenes that ask for it (g_jit_jobs, by device key).
std::mutex g_compile_mu;
std::mutex g_jobs_mu;
std::map<std::string, std::shared_future<std::string>> g_jit_jobs;

// hiprtc's code object of a spec ("" when it fails to compile), stored in the disk cache.
std::string jit_compile(const JitSpec& sp, const std::string& path, const std::string& dir) {
    std::lock_guard<std::mutex> lock(g_compile_mu);
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, sp.src.c_str(), "rtx_jit_render.hip", kJitNumHeaders, kJitHeaderSrcs,
                            kJitHeaderNames) != HIPRTC_SUCCESS)
        return std::string();
    std::vector<const char*> copts;
    for (const auto& o : sp.opts) copts.push_back(o.c_str());
    const hiprtcResult rc = hiprtcCompileProgram(prog, (int)copts.size(), copts.data());
    if (rc != HIPRTC_SUCCESS) {
        size_t n = 0;
        hiprtcGetProgramLogSize(prog, &n);
        std::string log(n, '\0');
        hiprtcGetProgramLog(prog, &log[0]);
        fprintf(stderr, "librtx: scene-specialized kernel failed to compile, using the generic one:\n%s\n",
                log.c_str());
        hiprtcDestroyProgram(&prog);
        return std::string();
    }
    size_t n = 0;
    hiprtcGetCodeSize(prog, &n);
    std::string code(n, '\0');
    hiprtcGetCode(prog, &code[0]);
    hiprtcDestroyProgram(&prog);
    if (!path.empty()) {
        const std::string tmp = path + "." + std::to_string((long)getpid());
        std::ofstream f(tmp, std::ios::binary);
        if (f.write(code.data(), (std::streamsize)code.size())) {
            f.close();
            (void)rename(tmp.c_str(), path.c_str());
            if (sp.baked) jit_prune_disk(dir);
        }
    }
    return code;
}

// The loaded kernel of device key dkey: an existing module (one more scene holds it) or
// code loaded now; nullptr when it fails to load. Caller holds g_jit_mu.
hipFunction_t jit_load_locked(const std::string& dkey, const std::string& code, const std::string& name, bool baked) {
    auto it = g_jit.find(dkey);
    if (it != g_jit.end()) {
        if (it->second.refs++ == 0 && it->second.baked) g_jit_idle.remove(dkey);
        return it->second.fn;
    }
    JitEntry e;
    hipError_t he = hipModuleLoadData(&e.mod, code.data());
    if (he == hipSuccess) he = hipModuleGetFunction(&e.fn, e.mod, name.c_str());
    if (he != hipSuccess) {
        fprintf(stderr, "librtx: scene-specialized kernel %s failed to load (%s), using the generic one\n",
                name.c_str(), hipGetErrorString(he));
        return nullptr;
    }
    e.baked = baked;
    e.refs = 1;
    g_jit[dkey] = e;
    return e.fn;
}

}  // namespace

// A resolved kernel variant of a scene's camera: the specialized kernel, or the generic one
// while its compile runs on a host thread (pending) or for good (fn == nullptr).
struct JitSlot {
    bool done = false;
    hipFunction_t fn = nullptr;
    int block = 0;    // its threads per block (jit_block when resolved)
    std::string name;
    std::string key;  // its g_jit entry (released by free_camera)
    bool pending = false;
    std::shared_future<std::string> fut;  // the compile (pending)
    std::string dkey;                     // the device key it loads under (pending)
    bool baked = false;
    bool lds = true;  // a split pass: its rays on the LDS stack (else registers, no LDS)
};

namespace {

// Resolves slot r: the specialized kernel from memory or the disk cache, or a compile --
// started on a host thread (jit_async: r.pending, the generic kernel renders meanwhile) or
// waited for. r.fn == nullptr and !r.pending: the generic kernel.
void jit_start(int device, const JitSpec& sp, JitSlot& r);
void jit_render_kernel(int device, const SceneView& v, const KParams& kp, const SceneTraits& tr, bool mesh, bool sec,
                       bool ext, bool cnt, bool jit, bool spp, bool out8, const std::string& baked, JitSlot& r) {
    r.fn = nullptr;
    r.pending = false;
    if (!jit_enabled()) return;
    const std::string arch = device_arch(device);
    if (arch.empty()) return;
    JitSpec sp;
    if (!jit_spec(arch, v, kp, tr, mesh, sec, ext, cnt, jit, spp, out8, baked, sp)) return;
    jit_start(device, sp, r);
}

// The specialized split pass (pass 0 trace, 1 shadow) of a hierarchy scene whose node table
// is `tables` (jit_csg_tables; "" or option jit_csg 0: the precompiled passes run).
void jit_split_kernel(int device, const std::string& tables, bool mesh, bool sec, bool cnt, bool jit, int pass,
                      bool rayreg, const std::vector<std::string>& fixed, JitSlot& r) {
    r.fn = nullptr;
    r.pending = false;
    if (!jit_enabled() || !opt_on(OPT_JIT_CSG) || tables.empty()) return;
    const std::string arch = device_arch(device);
    if (arch.empty()) return;
    jit_start(device, jit_split_spec(arch, tables, mesh, sec, cnt, jit, pass, rayreg, fixed), r);
}

// Resolves slot r for spec sp: the kernel from memory or the disk cache, or a compile on a
// host thread (r.pending).
void jit_start(int device, const JitSpec& sp, JitSlot& r) {
    std::string key = sp.src;
    for (const auto& o : sp.opts) key += "\n" + o;
    r.name = sp.name;
    const std::string dkey = key + "\n#device " + std::to_string(device);
    {
        std::lock_guard<std::mutex> lock(g_jit_mu);
        auto it = g_jit.find(dkey);
        if (it != g_jit.end()) {
            if (it->second.refs++ == 0 && it->second.baked) g_jit_idle.remove(dkey);
            r.key = dkey;
            r.fn = it->second.fn;
            return;
        }
    }
    if (opt_on(OPT_JIT_DUMP)) {  // tools/jit_resource.sh
        fprintf(stderr, "librtx: jit %s:", sp.name.c_str());
        for (const auto& o : sp.opts) fprintf(stderr, " '%s'", o.c_str());
        fprintf(stderr, "\n%s", sp.src.c_str());
    }
    std::shared_future<std::string> fut;
    {
        std::lock_guard<std::mutex> lock(g_jobs_mu);
        auto jt = g_jit_jobs.find(dkey);
        if (jt != g_jit_jobs.end()) {
            fut = jt->second;  // another scene's compile of the same kernel
        } else {
            std::string all = key;
            for (int h = 0; h < kJitNumHeaders; ++h) all += kJitHeaderSrcs[h];
            char hash[32];
            snprintf(hash, sizeof(hash), "%016zx", std::hash<std::string>{}(all));
            const std::string dir = jit_cache_dir();
            const std::string path = dir.empty() ? "" : dir + (sp.baked ? "/rtx_b_" : "/rtx_") + hash + ".co";
            std::string code;
            if (!path.empty()) {
                std::ifstream f(path, std::ios::binary);
                if (f) { std::stringstream ss; ss << f.rdbuf(); code = ss.str(); }
            }
            if (!code.empty()) {
                std::lock_guard<std::mutex> jl(g_jit_mu);
                r.fn = jit_load_locked(dkey, code, sp.name, sp.baked);
                if (r.fn) r.key = dkey;
                return;
            }
            for (auto e = g_jit_jobs.begin(); e != g_jit_jobs.end();)  // finished jobs nobody picked up
                e = e->second.wait_for(std::chrono::seconds(0)) == std::future_status::ready ? g_jit_jobs.erase(e)
                                                                                               : std::next(e);
            fut = std::async(std::launch::async, [sp, path, dir] { return jit_compile(sp, path, dir); }).share();
            g_jit_jobs[dkey] = fut;
        }
    }
    r.pending = true;
    r.fut = fut;
    r.dkey = dkey;
    r.baked = sp.baked;
}

// Picks up slot r's finished compile (wait: blocks until it is done): loads the kernel, or
// settles on the generic one when the compile failed.
void jit_poll(JitSlot& r, bool wait) {
    if (!r.pending) return;
    if (!wait && r.fut.wait_for(std::chrono::seconds(0)) != std::future_status::ready) return;
    const std::string& code = r.fut.get();
    r.pending = false;
    {
        std::lock_guard<std::mutex> lock(g_jobs_mu);
        g_jit_jobs.erase(r.dkey);
    }
    if (!code.empty()) {
        std::lock_guard<std::mutex> lock(g_jit_mu);
        r.fn = jit_load_locked(r.dkey, code, r.name, r.baked);
        if (r.fn) r.key = r.dkey;
    }
    r.fut = std::shared_future<std::string>();
}

}  // namespace

// ------------------------------------------------------------------ scene object
struct rtx_scene {
    int device = 0;
    SceneView view{};
    bool has_mesh = false, has_secondary = false, has_ext = false;
    SceneTraits traits;  // what the scene-specialized kernels pin
    int32_t hlevels = 0;
    // host copies for the per-time-range hierarchy bounds
    std::vector<DNode> h_nodes;
    std::vector<DObj> h_objs;
    std::vector<DTri> h_tris;
    std::vector<DBox> h_bounds_abi;
    HostScene h_bins;   // objs/tris and type counts, for the camera's primary-ray face bins
    void* d_lgrid = nullptr;        // light grids (per scene: lights and mesh are static)
    void* d_lg_start = nullptr;
    void* d_lg_faces = nullptr;
    void* d_lg_d2 = nullptr;
    void* d_bounds_abi = nullptr;   // for the time of the last rtx_intersect / rtx_occluded
    void* d_nodes = nullptr;
    void* d_nmat = nullptr;
    void* d_texels = nullptr;
    void* d_lut = nullptr;
    void* d_objs = nullptr;
    void* d_tris = nullptr;
    void* d_trins = nullptr;
    void* d_fboxes = nullptr;
    void* d_mats = nullptr;
    void* d_lights = nullptr;
    void* d_leaves = nullptr;
    void* d_tri_orig = nullptr;
    // camera: every per-camera table (pixel tables, sample origins, motion times, replayed
    // noise, hierarchy bounds, self-test limits, shadow-grid headers, primary-ray bins, tile
    // schedule, and the KParams block) in ONE device buffer, uploaded with one copy and
    // reused by later cameras while it is large enough (rtx_camera_set)
    bool cam_set = false;
    KParams kp{};
    char* d_cam = nullptr;
    size_t cam_cap = 0;
    char* h_cam = nullptr;  // pinned bounce buffer of the camera uploads (pinned_copy)
    size_t h_cam_cap = 0;
    KParams* d_kp = nullptr;  // (inside d_cam)
    // per frame time range [tlo, thi] (not per camera): the hierarchy bounds and the
    // directional lights' shadow-grid headers and cells (the cells in their own buffer)
    bool tr_valid = false;
    float tr_lo = 0.0f, tr_hi = 0.0f;
    std::vector<DBound> tr_bounds;
    std::vector<DSGrid> tr_grids;
    bool tr_grids_on = false, tr_dsg_off = false;
    double tr_dsg_min = 0.0;
    void* d_dsg_cells = nullptr;
    // the kernel resolved for each (counters, jitter, sample-parallel) variant of the
    // current camera: looked up (and compiled) once per camera, not per frame; nullptr
    // after a lookup means the generic kernel; 16-27: the split hierarchy passes
    // (16 + 4 pass + 2 counters + jitter, jit_split_kernel)
    JitSlot resolved[28];
    std::string last_kernel;  // name of the kernel the last render call launched
    std::string jit_baked;    // the scene records as constant arrays (jit_baked_records)
    std::string csg_tables;   // the hierarchy node table (jit_csg_tables)
    // fp32 staging of the rgb8 entry points when no scene-specialized kernel is available
    float* d_scratch = nullptr;
    size_t scratch_floats = 0;
    // the measured tile schedule (tile_schedule): dispatch order and wave durations of a
    // whole frame's tiles; state 0 none, 1 measure the next whole frame, 2 sort, 3 ordered,
    // 4 measured and left in row-major order
    void* d_tile_perm = nullptr;
    void* d_tile_time = nullptr;
    // heavy tiles of the primary-ray bins (heavy_chunks): chunk items and their per-frame
    // closest faces, inside d_cam; heavy_n chunks (0: none)
    const int2* d_heavy_items = nullptr;
    uint2* d_mesh_hits = nullptr;
    int32_t heavy_n = 0;
    int tile_sched = 0;
    bool tile_xcd = false;            // the schedule table's layout (option xcd_map when sorted)
    hipEvent_t tile_event = nullptr;  // recorded after the measuring launch
    // the split hierarchy passes (rtx_split.h, render_split): the record arrays of one
    // chunk (kept while the scene lives, reused by every frame), the per-chunk append
    // counters of a frame, the per-block redo flags (all zero between renders), and what the
    // pool sizing learned: deeper records per sample (split_ratio), read back without a
    // stall from the last frame's counters (split_pending: h_split_count is in flight)
    uint32_t* d_split = nullptr;
    int64_t split_cap = 0;
    unsigned int* d_split_count = nullptr;
    int64_t split_nchunk_cap = 0;
    uint32_t* d_split_redo = nullptr;  // per chunk block: list entry, then flag (2 words)
    int64_t split_redo_cap = 0;
    double split_ratio = -1.0;
    unsigned int* h_split_count = nullptr;  // pinned
    std::vector<std::pair<int64_t, int64_t>> split_chunks;  // (samples, records) of the read-back frame's chunks
    bool split_pending = false;
    hipEvent_t split_read = nullptr;     // the readback's completion
    hipEvent_t split_done = nullptr;     // the last split render's completion (cross-stream order)
    hipStream_t split_stream = nullptr;  // its stream
    bool split_used = false;
    // the device face bins' scratch (rtx_bins.hip; per camera, reused while large enough):
    // the pixel tables and stage-1 arrays, then the (bin, rank) pairs
    char* d_mb = nullptr;
    size_t mb_cap = 0;
    char* d_mb2 = nullptr;
    size_t mb2_cap = 0;
    MeshBinsDev mbd{};
    // buffers a captured graph may still reference: freed only with the scene
    std::vector<void*> split_retired;
    bool split_captured = false;
};

namespace {

template <class T>
int upload(void** dptr, const std::vector<T>& v) {
    if (v.empty()) { *dptr = nullptr; return RTX_OK; }
    RTX_HIP(hipMalloc(dptr, sizeof(T) * v.size()));
    RTX_HIP(hipMemcpy(*dptr, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice));
    return RTX_OK;
}

// Host-to-device uploads of rtx_camera_set go through the scene's pinned buffer (grown as
// needed) and a copy kernel that reads it over the bus: hipMemcpy from pageable memory
// set up the runtime's staging on a process's first camera upload (~7 ms), and a copy from
// pinned memory the copy engine (~6 ms); the kernel's first launch costs ~1 ms.
int pinned_reserve(rtx_scene* s, size_t n) {
    if (s->h_cam_cap >= n) return RTX_OK;
    (void)hipHostFree(s->h_cam);
    s->h_cam = nullptr;
    s->h_cam_cap = 0;
    RTX_HIP(hipHostMalloc((void**)&s->h_cam, n + n / 4, hipHostMallocDefault));
    s->h_cam_cap = n + n / 4;
    return RTX_OK;
}
// The first n bytes of the pinned buffer (whole 16-byte words) to dst (16-byte aligned);
// blocking, so the buffer can be refilled as soon as it returns.
int pinned_upload(rtx_scene* s, void* dst, size_t n, size_t off = 0) {  // (bytes [off, off + n) of the buffer)
    if (n == 0) return RTX_OK;
    if ((n & 15) || (off & 15) || (reinterpret_cast<uintptr_t>(dst) & 15))
        return fail(RTX_ERR_INVALID, "pinned_upload: unaligned");
    void* hp = nullptr;
    RTX_HIP(hipHostGetDevicePointer(&hp, s->h_cam + off, 0));
    const int64_t w = (int64_t)(n / 16);
    hipLaunchKernelGGL(k_stage_copy, dim3((unsigned)std::min<int64_t>(1024, (w + 255) / 256)), dim3(256), 0, nullptr,
                       (const uint4*)hp, (uint4*)dst, w);
    RTX_HIP(hipGetLastError());
    RTX_HIP(hipStreamSynchronize(nullptr));
    return RTX_OK;
}

// A device buffer of at least n bytes (grown, contents dropped).
int grow(char** p, size_t* cap, size_t n) {
    if (*cap >= n) return RTX_OK;
    (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    RTX_HIP(hipMalloc((void**)p, n + n / 4));
    *cap = n + n / 4;
    return RTX_OK;
}

size_t a256(size_t n) { return (n + 255) & ~(size_t)255; }

// Forgets the camera (its kernels are specialized on its sample counts); the device
// buffers stay for the next camera (free_scene frees them).
void free_camera(rtx_scene* s) {
    s->tile_sched = 0;
    s->cam_set = false;
    for (auto& r : s->resolved) {  // specialized on the camera's sample counts
        jit_release(r.key);
        r = JitSlot{};
    }
}

void free_scene(rtx_scene* s) {
    free_camera(s);
    (void)hipFree(s->d_cam);
    (void)hipHostFree(s->h_cam);
    (void)hipFree(s->d_dsg_cells);
    (void)hipFree(s->d_scratch);
    (void)hipFree(s->d_mb);
    (void)hipFree(s->d_mb2);
    if (s->split_done) (void)hipEventSynchronize(s->split_done);
    (void)hipFree(s->d_split);
    (void)hipFree(s->d_split_count);
    (void)hipFree(s->d_split_redo);
    for (void* p : s->split_retired) (void)hipFree(p);
    if (s->split_read) { (void)hipEventSynchronize(s->split_read); (void)hipEventDestroy(s->split_read); }
    if (s->split_done) (void)hipEventDestroy(s->split_done);
    (void)hipHostFree(s->h_split_count);
    if (s->tile_event) (void)hipEventDestroy(s->tile_event);
    for (void* p : {s->d_objs, s->d_tris, s->d_trins, s->d_fboxes, s->d_mats, s->d_lights, s->d_leaves, s->d_tri_orig, s->d_nodes, s->d_nmat,
                    s->d_texels, s->d_lut, s->d_bounds_abi, s->d_lgrid, s->d_lg_start, s->d_lg_faces, s->d_lg_d2})
        (void)hipFree(p);
    delete s;
}

}  // namespace

namespace {
// Option setup_log: the host time of each step of a setup call, printed to stderr.
struct SetupLog {
    const char* what;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now(), t = t0;
    std::string line;
    explicit SetupLog(const char* w) : what(w) {}
    size_t staged = 0;  // bytes of camera tables staged by the earlier steps
    // staged_total: the staging buffer's size after this step (its tables' bytes are logged)
    void mark(const char* step, size_t staged_total = SIZE_MAX) {
        if (!opt_on(OPT_SETUP_LOG)) return;
        const auto n = std::chrono::steady_clock::now();
        char buf[128];
        snprintf(buf, sizeof(buf), " %s %.3f", step, std::chrono::duration<double, std::milli>(n - t).count());
        line += buf;
        if (staged_total != SIZE_MAX) {
            snprintf(buf, sizeof(buf), " [%zu B]", staged_total - staged);
            line += buf;
            staged = staged_total;
        }
        t = n;
    }
    ~SetupLog() {
        if (opt_on(OPT_SETUP_LOG) && !line.empty())
            fprintf(stderr, "librtx: %s ms:%s (total %.3f)\n", what, line.c_str(),
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
};

// Layout of the camera tables: 256-byte aligned segments of one device buffer. put()
// records where a table goes and where it comes from (the source must stay alive until
// write(); p == nullptr: zero-filled); write() fills the pinned buffer once, with no growing
// host vector to copy (DepthOfField's 1.5 MB of bins: 0.2 ms of reallocation copies).
struct CamStage {
    struct Seg {
        size_t off;
        const void* p;
        size_t n;
        bool dev;  // filled on the device after the upload: not written (nor uploaded)
    };
    std::vector<Seg> segs;
    size_t bytes = 0;
    size_t put(const void* p, size_t n, bool dev = false) {
        const size_t off = (bytes + 255) & ~(size_t)255;
        segs.push_back(Seg{off, p, n, dev});
        bytes = off + std::max<size_t>(n, 4);
        return off;
    }
    template <class T>
    size_t put(const std::vector<T>& v) { return put(v.empty() ? nullptr : v.data(), sizeof(T) * v.size()); }
    size_t size() const { return (bytes + 15) & ~(size_t)15; }  // (whole 16-byte words)
    // the byte ranges to upload: the segments not filled on the device, merged, in whole
    // 16-byte words (a segment's next neighbour starts 256-aligned, so the rounding stays
    // short of it)
    std::vector<std::pair<size_t, size_t>> runs() const {
        std::vector<std::pair<size_t, size_t>> r;
        for (const Seg& g : segs) {
            if (g.dev) continue;
            const size_t end = (g.off + std::max<size_t>(g.n, 4) + 15) & ~(size_t)15;
            if (!r.empty() && r.back().second == g.off) r.back().second = end;
            else if (!r.empty() && ((r.back().second + 255) & ~(size_t)255) == g.off) r.back().second = end;
            else r.emplace_back(g.off, end);
        }
        return r;
    }
    void write(char* h) const {
        for (const Seg& g : segs) {
            if (g.p) memcpy(h + g.off, g.p, g.n);
            else if (!g.dev) memset(h + g.off, 0, std::max<size_t>(g.n, 4));
        }
    }
};

}  // namespace

namespace {
// Stage 1 of the device face bins of the scene's one mesh (option dev_bins; rtx_bins.hip):
// uploads the pixel tables, bins every face, and reads the bins' face counts back (a copy
// kernel into the mapped pinned buffer: no copy engine) into start (prefix sums, nb + 1).
// *npairs: the total; mesh_bins 0 when a face cannot be projected (the BVH walk, as on
// the host). Leaves the faces' order in the scene's scratch for stage 2.
int mesh_bins_dev1(rtx_scene* s, const rtx_camera_desc* c, int32_t bins_x, std::vector<int32_t>& start,
                   int32_t* npairs, int32_t* mesh_bins, SetupLog& slog) {
    const HostScene& H = s->h_bins;
    const DObj& m = H.objs[H.n_plane + H.n_sphere + H.n_box];
    const int32_t n = m.tri_count, W = c->ncols, Hh = c->height;
    const int32_t nb = bins_x * ((Hh + 7) / 8);
    *npairs = 0;
    *mesh_bins = 0;
    start.assign((size_t)nb + 1, 0);
    const size_t oys = a256(sizeof(float) * W), tb = oys + a256(sizeof(float) * Hh);
    int rc;
    if ((rc = grow(&s->d_mb, &s->mb_cap, tb + mesh_bins_bytes1(n, nb)))) return rc;
    if ((rc = pinned_reserve(s, tb))) return rc;
    memcpy(s->h_cam, c->xs, sizeof(float) * W);
    memcpy(s->h_cam + oys, c->ys, sizeof(float) * Hh);
    if ((rc = pinned_upload(s, s->d_mb, (tb + 15) & ~(size_t)15))) return rc;
    slog.mark("face bins: scratch + tables");
    BinProj P;
    for (int a = 0; a < 3; ++a) {
        P.o[a] = c->aa_origins[a];  // (a pinhole: every primary ray leaves aa_o[0])
        P.u[a] = c->u[a]; P.v[a] = c->v[a]; P.w[a] = c->w[a];
    }
    P.d = c->d;
    P.xs = reinterpret_cast<const float*>(s->d_mb);
    P.ys = reinterpret_cast<const float*>(s->d_mb + oys);
    P.W = W;
    P.H = Hh;
    const float* tris = reinterpret_cast<const float*>(static_cast<const DTri*>(s->d_tris) + m.tri_begin);
    RTX_HIP(mesh_bins_stage1(P, tris, (int32_t)(sizeof(DTri) / sizeof(float)), n, bins_x, nb, s->d_mb + tb, s->mbd,
                             nullptr));
    if (opt_on(OPT_SETUP_LOG)) {
        RTX_HIP(hipStreamSynchronize(nullptr));
        slog.mark("face bins: rects + sort");
    }
    // the counts and the flag (the segment after them) to the host
    const size_t cb = a256(sizeof(int32_t) * ((size_t)nb + 1)) + 16;
    if ((rc = pinned_reserve(s, cb))) return rc;
    void* hp = nullptr;
    RTX_HIP(hipHostGetDevicePointer(&hp, s->h_cam, 0));
    hipLaunchKernelGGL(k_stage_copy, dim3((unsigned)std::min<size_t>(1024, (cb / 16 + 255) / 256)), dim3(256), 0, nullptr,
                       (const uint4*)s->mbd.count, (uint4*)hp, (int64_t)(cb / 16));
    RTX_HIP(hipGetLastError());
    RTX_HIP(hipStreamSynchronize(nullptr));
    const int32_t* cnt = reinterpret_cast<const int32_t*>(s->h_cam);
    if (*reinterpret_cast<const int32_t*>(s->h_cam + cb - 16) != 0) return RTX_OK;  // walk the BVH
    for (int32_t b = 0; b < nb; ++b) start[b + 1] = start[b] + cnt[b];
    // the fill cursors of stage 2: the bins' starts
    memcpy(s->h_cam, start.data(), sizeof(int32_t) * nb);
    if ((rc = pinned_upload(s, s->mbd.count, (sizeof(int32_t) * nb + 15) & ~(size_t)15))) return rc;
    *npairs = start[nb];
    *mesh_bins = 1;
    return RTX_OK;
}

// Stage 2: the bins' face lists and depth bounds into the camera buffer.
int mesh_bins_dev2(rtx_scene* s, int32_t bins_x, int32_t nb, int32_t npairs, int32_t* faces, float* zmin) {
    const HostScene& H = s->h_bins;
    const int32_t n = H.objs[H.n_plane + H.n_sphere + H.n_box].tri_count;
    if (int rc = grow(&s->d_mb2, &s->mb2_cap, mesh_bins_bytes2(n, npairs))) return rc;
    RTX_HIP(mesh_bins_stage2(s->mbd, n, bins_x, nb, npairs, s->d_mb2, faces, zmin, nullptr));
    RTX_HIP(hipStreamSynchronize(nullptr));
    return RTX_OK;
}

}  // namespace

extern "C" {

int rtx_abi_version(void) { return RTX_ABI_VERSION; }

int rtx_set_option(const char* name, const char* value) {
    if (!name || !value) return fail(RTX_ERR_INVALID, "rtx_set_option: null argument");
    for (int i = 0; i < OPT_COUNT; ++i) {
        if (strcmp(kOpts[i].name, name) != 0) continue;
        std::lock_guard<std::mutex> lock(g_opt_mu);
        OptVal& o = opt_table()[i];
        if (kOpts[i].str) {
            o.s = value;
            return RTX_OK;
        }
        char* end = nullptr;
        const double v = strtod(value, &end);
        if (end == value || *end != '\0' || !std::isfinite(v))
            return fail(RTX_ERR_INVALID, std::string("rtx_set_option: ") + name + " takes a number, got '" + value + "'");
        o.v = v;
        return RTX_OK;
    }
    return fail(RTX_ERR_INVALID, std::string("rtx_set_option: no option '") + name + "'");
}

int rtx_get_option(const char* name, char* value, int32_t cap) {
    if (!name || !value || cap < 1) return fail(RTX_ERR_INVALID, "rtx_get_option: bad argument");
    for (int i = 0; i < OPT_COUNT; ++i) {
        if (strcmp(kOpts[i].name, name) != 0) continue;
        std::string v;
        if (kOpts[i].str) {
            v = opt_str((Opt)i);
        } else {
            char buf[64];
            snprintf(buf, sizeof(buf), "%.17g", opt((Opt)i));
            v = buf;
        }
        if ((int64_t)v.size() >= cap) return fail(RTX_ERR_INVALID, "rtx_get_option: buffer too small");
        memcpy(value, v.c_str(), v.size() + 1);
        return RTX_OK;
    }
    return fail(RTX_ERR_INVALID, std::string("rtx_get_option: no option '") + name + "'");
}

const char* rtx_option_name(int32_t i) { return i >= 0 && i < OPT_COUNT ? kOpts[i].name : nullptr; }

int32_t rtx_jit_wait(rtx_scene* s, int32_t block) {
    if (!s) return fail(RTX_ERR_INVALID, "rtx_jit_wait: null scene");
    int32_t n = 0;
    for (JitSlot& r : s->resolved) {
        jit_poll(r, block != 0);
        n += r.pending ? 1 : 0;
    }
    return n;
}

int rtx_graph_launch(void* graph_exec, int32_t n, void* stream) {
    if (!graph_exec || n < 0) return fail(RTX_ERR_INVALID, "rtx_graph_launch: null graph or n < 0");
    for (int32_t i = 0; i < n; ++i)
        RTX_HIP(hipGraphLaunch(static_cast<hipGraphExec_t>(graph_exec), static_cast<hipStream_t>(stream)));
    return RTX_OK;
}

const char* rtx_last_error(void) { return g_last_error.c_str(); }

const char* rtx_last_kernel(const rtx_scene* s) { return s ? s->last_kernel.c_str() : ""; }

int32_t rtx_jit_modules(void) {
    std::lock_guard<std::mutex> lock(g_jit_mu);
    return (int32_t)g_jit.size();
}

int rtx_scene_create(const rtx_scene_desc* desc, rtx_scene** out) {
    if (!out) return fail(RTX_ERR_INVALID, "rtx_scene_create: null argument");
    *out = nullptr;
    HostScene H;
    int rc = convert_scene(desc, H);
    if (rc) return rc;
    rtx_scene* s = new rtx_scene();
    if (hipGetDevice(&s->device) != hipSuccess) { delete s; return fail(RTX_ERR_HIP, "hipGetDevice failed"); }
    if ((rc = upload(&s->d_objs, H.objs)) || (rc = upload(&s->d_tris, H.tris)) || (rc = upload(&s->d_trins, H.trins)) ||
        (rc = upload(&s->d_fboxes, H.fboxes)) ||
        (rc = upload(&s->d_mats, H.mats)) || (rc = upload(&s->d_lights, H.lights)) ||
        (rc = upload(&s->d_leaves, H.leaves)) || (rc = upload(&s->d_tri_orig, H.tri_orig)) ||
        (rc = upload(&s->d_texels, H.texels)) || (rc = upload(&s->d_lut, H.lut255))) {
        free_scene(s);
        return rc;
    }
    {
        std::vector<DNodeHot> hot;
        std::vector<DNodeMat> mat;
        split_nodes(H.nodes, hot, mat);
        if ((rc = upload(&s->d_nodes, hot)) || (rc = upload(&s->d_nmat, mat))) {
            free_scene(s);
            return rc;
        }
    }
    s->has_mesh = H.has_mesh;
    s->has_secondary = H.has_secondary;
    s->has_ext = H.has_ext;
    s->hlevels = H.hlevels;
    s->traits = scene_traits(H);
    s->jit_baked = jit_baked_records(H.objs, H.mats, H.lights);
    {  // primary-ray bins (per camera, rtx_camera_set)
        s->h_bins.objs = H.objs;
        if (H.n_mesh == 1) s->h_bins.tris = H.tris;
        s->h_bins.n_plane = H.n_plane; s->h_bins.n_sphere = H.n_sphere;
        s->h_bins.n_box = H.n_box; s->h_bins.n_mesh = H.n_mesh;
        s->h_bins.lights = H.lights;  // and the shadow grids of directional lights
        s->h_bins.nodes = H.nodes;
    }
    if (!H.nodes.empty()) {
        s->h_nodes = H.nodes;
        s->csg_tables = jit_csg_tables(H.nodes);
        s->h_objs = H.objs;
        s->h_tris = H.tris;
        if ((rc = upload(&s->d_bounds_abi, std::vector<DBox>(3 * H.nodes.size())))) {
            free_scene(s);
            return rc;
        }
    }
    SceneView& v = s->view;
    v.objs = (cptr<DObj>)s->d_objs;
    v.tris = (cptr<DTri>)s->d_tris;
    v.trins = (cptr<DTriN>)s->d_trins;
    v.fboxes = (cptr<DFaceBox>)s->d_fboxes;
    v.mats = (cptr<DMat>)s->d_mats;
    v.lights = (cptr<DLight>)s->d_lights;
    v.leaves = (cptr<DLeaf>)s->d_leaves;
    v.tri_orig = (cptr<int32_t>)s->d_tri_orig;
    v.n_objs = H.n_objs;
    v.n_objs_all = (int32_t)H.objs.size();
    v.n_mats = (int32_t)H.mats.size();
    v.n_lights = H.n_lights;
    v.n_plane = H.n_plane; v.n_sphere = H.n_sphere; v.n_box = H.n_box; v.n_mesh = H.n_mesh;
    v.pow_bits = H.pow_bits;
    std::memcpy(v.ambient, H.ambient, sizeof(v.ambient));
    v.nodes = (cptr<DNodeHot>)s->d_nodes;
    v.nmat = (cptr<DNodeMat>)s->d_nmat;
    v.texels = (cptr<uint32_t>)s->d_texels;
    v.lut255 = (cptr<float>)s->d_lut;
    v.n_nodes = (int32_t)H.nodes.size();
    v.n_tris = (int32_t)H.tris.size();
    v.n_leaves = (int32_t)H.leaves.size();
    v.hlevels = H.hlevels;
    {  // light grids for the shadow rays of point lights (option lgrid 0: walk the BVH)
        std::vector<DLGrid> grids;
        std::vector<int32_t> gstart, gfaces;
        std::vector<float> gd2;
        if (opt_on(OPT_LGRID) && light_grids(H, grids, gstart, gfaces, gd2)) {
            if (gfaces.empty()) { gfaces.push_back(0); gd2.push_back(0.0f); }
            if (opt_on(OPT_SETUP_LOG))
                fprintf(stderr, "librtx: light grids: %zu grids %zu B, starts %zu B, faces %zu B, d2 %zu B\n", grids.size(),
                        sizeof(DLGrid) * grids.size(), sizeof(int32_t) * gstart.size(), sizeof(int32_t) * gfaces.size(),
                        sizeof(float) * gd2.size());
            if ((rc = upload(&s->d_lgrid, grids)) || (rc = upload(&s->d_lg_start, gstart)) ||
                (rc = upload(&s->d_lg_faces, gfaces)) || (rc = upload(&s->d_lg_d2, gd2))) {
                free_scene(s);
                return rc;
            }
            v.lgrid = (cptr<DLGrid>)s->d_lgrid;
            v.lg_start = (cptr<int32_t>)s->d_lg_start;
            v.lg_faces = (cptr<int32_t>)s->d_lg_faces;
            v.lg_d2 = (cptr<float>)s->d_lg_d2;
            v.lgrid_on = 1;
        }
    }
    {  // the first launch of any of the library's kernels loads its code object (~1 ms):
       // once per process, here rather than in the first camera upload
        static std::once_flag loaded;
        std::call_once(loaded, [] {
            hipLaunchKernelGGL(k_stage_copy, dim3(1), dim3(64), 0, nullptr, nullptr, nullptr, (int64_t)0);
            (void)hipGetLastError();
        });
        // a scene whose one mesh gets device face bins: the sorts' one-time setup (once per
        // process), here rather than in the first camera upload
        static std::once_flag sorts;
        if (H.n_mesh == 1 && opt_on(OPT_DEV_BINS)) std::call_once(sorts, [] { mesh_bins_warm(); });
    }
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
    SetupLog slog("rtx_camera_set");
    KParams k;
    int rc = convert_camera(c, k);
    if (rc) return rc;
    free_camera(s);
    const size_t nsamp = (size_t)c->n_dof * c->n_aa;
    std::vector<float> times(c->n_times);
    for (int i = 0; i < c->n_times; ++i) times[i] = (float)c->times[i];  // current_time * speed casts to fp32
    const auto mm = std::minmax_element(times.begin(), times.end());
    const double omax = camera_origin_bound(c);
    k.S = s->view;
    slog.mark("convert");
    // what depends on the frame's time range only: computed again when it changes
    const bool dsg_off = !opt_on(OPT_DSGRID);  // every shadow ray tests every object
    const double dsg_min = opt(OPT_DSGRID_MIN);  // (dir_shadow_grids reads it)
    if (!s->tr_valid || s->tr_lo != *mm.first || s->tr_hi != *mm.second || s->tr_dsg_off != dsg_off ||
        s->tr_dsg_min != dsg_min) {
        s->tr_bounds.clear();
        if (!s->h_nodes.empty())  // hierarchy bounds over the frame's motion-time range
            s->tr_bounds = compute_bounds(s->h_nodes, s->h_objs, s->h_tris, *mm.first, *mm.second);
        std::vector<DSCell> cells;
        std::vector<DSRect> rects;
        size_t ncells = 0;
        s->tr_grids.clear();
        s->tr_dsg_off = dsg_off;
        s->tr_dsg_min = dsg_min;
        s->tr_grids_on = !dsg_off && dir_shadow_grids(s->h_bins, s->tr_bounds, *mm.first, *mm.second, s->tr_grids,
                                                      cells, &rects, &ncells);
        (void)hipDeviceSynchronize();  // (frames of the previous camera may still read the cells)
        (void)hipFree(s->d_dsg_cells);
        s->d_dsg_cells = nullptr;
        if (s->tr_grids_on) {  // the cells, then the rectangles k_dsg_fill reads
            const size_t n = sizeof(DSCell) * ncells, nr = sizeof(DSRect) * rects.size();
            RTX_HIP(hipMalloc(&s->d_dsg_cells, n + std::max<size_t>(nr, 16)));
            if (nr) {
                if ((rc = pinned_reserve(s, nr))) return rc;
                memcpy(s->h_cam, rects.data(), nr);
                if ((rc = pinned_upload(s, (char*)s->d_dsg_cells + n, nr))) return rc;
            }
            hipLaunchKernelGGL(k_dsg_fill, dim3((unsigned)((ncells + 255) / 256)), dim3(256), 0, nullptr,
                               (const DSRect*)((char*)s->d_dsg_cells + n), (int32_t)rects.size(),
                               (DSCell*)s->d_dsg_cells, (int64_t)ncells, s->tr_grids.empty() ? 0 : kDsgG);
            RTX_HIP(hipGetLastError());
            RTX_HIP(hipStreamSynchronize(nullptr));
        }
        s->tr_valid = true;
        s->tr_lo = *mm.first;
        s->tr_hi = *mm.second;
    }
    slog.mark("time-range grids");
    CamStage st;
    const size_t o_xs = st.put(c->xs, sizeof(float) * c->ncols), o_ys = st.put(c->ys, sizeof(float) * c->height);
    const size_t o_dof = st.put(c->dof_origins, sizeof(float) * 3 * c->n_dof);
    const size_t o_aa = st.put(c->aa_origins, sizeof(float) * 3 * nsamp);
    const size_t o_times = st.put(times);
    size_t o_noise = 0, o_bounds = 0, o_pself = 0, o_dsg = 0, o_bstart = 0, o_bfaces = 0, o_bz = 0, o_bmask = 0;
    size_t o_tperm = 0, o_ttime = 0;
    const bool replay = c->jitter == RTX_JITTER_REPLAY;
    if (replay) o_noise = st.put(c->noise, sizeof(float) * 3 * (size_t)c->ncols * c->height * nsamp);
    slog.mark("tables", st.size());
    // (put() keeps pointers: every staged table lives until the upload)
    std::vector<DBox> boxes;
    std::vector<float> pself_lim;
    std::vector<DSGrid> grids;
    std::vector<int32_t> ident;
    if (!s->h_nodes.empty()) {
        boxes = split_bounds(s->tr_bounds);
        o_bounds = st.put(boxes);
    }
    // self tests of planes (option self_skip 0: none). Scenes with secondary rays get none:
    // MirrorRefraction measured 1.4 % slower with them (most of its shadow rays leave
    // deeper levels, which pay the check and never skip), TSP 3 % and TM 2 % faster
    // (profiles/r04/plane_self/)
    const bool pself = opt_on(OPT_SELF_SKIP) && s->view.n_plane > 0 && !s->h_bins.lights.empty() && !s->has_secondary;
    if (pself) {
        pself_lim = plane_self_limits(s->h_bins, omax);
        o_pself = st.put(pself_lim);
    }
    if (s->tr_grids_on) {  // the grid headers with this camera's self-test marks
        grids = s->tr_grids;
        dir_self_boxes(s->h_bins, grids, omax);
        o_dsg = st.put(grids);
    }
    slog.mark("self tests", st.size());
    std::vector<int32_t> bstart, bfaces;
    std::vector<float> bz;
    std::vector<uint32_t> bmask, brmask;
    int32_t bins_x = 0, mesh_bins = 0, dev_pairs = 0;
    bool dev_faces = false;  // the mesh's face bins are built on the device (rtx_bins.hip)
    const bool bins = opt_on(OPT_BINS) &&
                      primary_bins(s->h_bins, c, s->tr_bounds, bstart, bfaces, bz, bmask, brmask, bins_x, mesh_bins,
                                   opt_on(OPT_DEV_BINS) ? &dev_faces : nullptr);
    if (bins && dev_faces) {
        if ((rc = mesh_bins_dev1(s, c, bins_x, bstart, &dev_pairs, &mesh_bins, slog))) return rc;
        dev_faces = dev_pairs > 0;
        slog.mark("face bins: counts read back");
    }
    if (bins) {
        if (bfaces.empty() && !dev_faces) { bfaces.push_back(0); bz.push_back(0.0f); }
        bmask.insert(bmask.end(), brmask.begin(), brmask.end());  // [object masks | root masks]
        o_bstart = st.put(bstart);
        if (!dev_faces) {  // (the device-filled lists go last: below)
            o_bfaces = st.put(bfaces);
            o_bz = st.put(bz);
        }
        o_bmask = st.put(bmask);
    }
    std::vector<int32_t> bheavy;
    std::vector<int2> hitems;
    size_t o_bheavy = 0, o_hitems = 0, o_mhits = 0;
    const bool heavy = bins && mesh_bins && !s->has_ext && opt_on(OPT_HEAVY_TILES) && heavy_chunks(bstart, bheavy, hitems);
    if (heavy) {
        o_bheavy = st.put(bheavy);
        o_hitems = st.put(hitems);
        // (o_mhits: below, device-filled)
    }
    slog.mark("bins", st.size());
    // the measured tile schedule (tile_schedule): identity order until measured
    const bool tsched = tile_sched_enabled() && !s->has_ext && (s->has_secondary || s->has_mesh);
    int64_t tiles = 0;
    if (tsched) {
        const int64_t wpb = kBlock<false> / 64;
        tiles = (int64_t)((c->ncols + 7) / 8) * ((c->height + 7) / 8);
        const int64_t nw = (tiles + wpb - 1) / wpb * wpb;
        ident.resize((size_t)nw);
        std::iota(ident.begin(), ident.end(), 0);
        o_tperm = st.put(ident);
        // (o_ttime: below, device-filled)
    }
    const size_t o_kp = st.put(nullptr, sizeof(KParams));
    // the segments the device fills, last: the host stages (and uploads) only what precedes
    // them -- the face lists of device bins, the heavy tiles' per-frame hits (the chunk pass
    // writes them) and the tile times (a measured frame writes them before they are read)
    const size_t host_bytes = st.size();
    if (dev_faces) {
        o_bfaces = st.put(nullptr, sizeof(int32_t) * dev_pairs, true);
        o_bz = st.put(nullptr, sizeof(float) * dev_pairs, true);
    }
    if (heavy) o_mhits = st.put(nullptr, sizeof(uint2) * 64 * hitems.size(), true);
    if (tsched) {
        const int64_t nw = (tiles + kBlock<false> / 64 - 1) / (kBlock<false> / 64) * (kBlock<false> / 64);
        o_ttime = st.put(nullptr, sizeof(uint32_t) * nw, true);
    }
    slog.mark("tile schedule", st.size());
    // one device buffer for all of it, reused while large enough; its old contents may still
    // be read by frames of the previous camera
    (void)hipDeviceSynchronize();
    if (s->cam_cap < st.size()) {
        (void)hipFree(s->d_cam);
        s->d_cam = nullptr;
        s->cam_cap = 0;
        const size_t cap = st.size() + st.size() / 4;
        RTX_HIP(hipMalloc((void**)&s->d_cam, cap));
        s->cam_cap = cap;
    }
    char* const D = s->d_cam;
    slog.mark("sync+alloc");
    k.xs = (cptr<float>)(D + o_xs);
    k.ys = (cptr<float>)(D + o_ys);
    k.dof_o = (cptr<float>)(D + o_dof);
    k.aa_o = (cptr<float>)(D + o_aa);
    k.times = (cptr<float>)(D + o_times);
    k.noise = replay ? (cptr<float>)(D + o_noise) : nullptr;
    if (!s->h_nodes.empty()) bind_boxes(k.S, (const DBox*)(D + o_bounds), s->h_nodes.size());
    if (pself) k.S.plane_self = (cptr<float>)(D + o_pself);
    if (s->tr_grids_on) {
        k.S.dsgrid = (cptr<DSGrid>)(D + o_dsg);
        k.S.dsg_cells = (cptr<DSCell>)s->d_dsg_cells;
        k.S.dsg_on = 1;
    }
    if (bins) {
        k.S.bin_objmask = (cptr<uint32_t>)(D + o_bmask);
        k.S.bin_rootmask = (cptr<uint32_t>)(D + o_bmask) + brmask.size();
        k.S.mesh_bins = mesh_bins;
        k.S.bin_start = (cptr<int32_t>)(D + o_bstart);
        k.S.bin_faces = (cptr<int32_t>)(D + o_bfaces);
        k.S.bin_zmin = (cptr<float>)(D + o_bz);
        k.S.bins_x = bins_x;
        k.S.bins_on = 1;
    }
    s->heavy_n = 0;
    s->d_heavy_items = nullptr;
    s->d_mesh_hits = nullptr;
    if (heavy) {
        k.S.bin_heavy = (cptr<int32_t>)(D + o_bheavy);
        k.S.mesh_hits = reinterpret_cast<const uint2*>(D + o_mhits);
        s->d_heavy_items = reinterpret_cast<const int2*>(D + o_hitems);
        s->d_mesh_hits = reinterpret_cast<uint2*>(D + o_mhits);
        s->heavy_n = (int32_t)hitems.size();
    }
#if defined(RTX_WAVE_LOG)  // tools/wave_timeline.py builds only
    if (const char* e = getenv("RTX_WAVE_LOG_PTR"))
        k.wave_log = reinterpret_cast<unsigned long long*>((uintptr_t)strtoull(e, nullptr, 0));
#endif
    // one sample, no jitter, static scene: every primary ray starts at aa_o[0], so its
    // origin-only plane and sphere terms are per-frame constants (closest_hit's fp32
    // operations, here once; RTX_PRIM_ORIGIN kernels read them)
    // (flat primary + shadow scenes: TwoSpheresPlane 24.09 -> 23.59 us, TorusMesh -0.6 %;
    // MirrorRefraction measured 1 % slower with them, profiles/r04/prim_origin/)
    if (c->n_dof == 1 && c->n_aa == 1 && c->jitter == RTX_JITTER_OFF && !s->traits.any_speed && !s->has_ext &&
        !s->has_secondary && s->view.n_plane <= 4 && s->view.n_sphere <= 16 && prim_origin_enabled()) {
        const f3 o = mk(c->aa_origins[0], c->aa_origins[1], c->aa_origins[2]);
        int oi = 0;
        for (int q = 0; q < s->view.n_plane; ++q, ++oi) {
            const DObj& ob = s->h_bins.objs[oi];
            k.po_pnum[q] = dot(sub(moved(ob, ob.a, 0.0f), o), ld3(ob.b));
        }
        for (int q = 0; q < s->view.n_sphere; ++q, ++oi) {
            const DObj& ob = s->h_bins.objs[oi];
            const f3 oc = sub(o, moved(ob, ob.a, 0.0f));
            k.po_soc[q][0] = oc.x; k.po_soc[q][1] = oc.y; k.po_soc[q][2] = oc.z;
            k.po_sq[q] = dot(oc, oc);
        }
        k.po_valid = 1;
    }
    if (tsched) {
        k.tile_perm = (cptr<int32_t>)(D + o_tperm);
        k.tile_time = reinterpret_cast<unsigned int*>(D + o_ttime);
        k.tile_n = (int32_t)tiles;
        s->d_tile_perm = D + o_tperm;
        s->d_tile_time = D + o_ttime;
        s->tile_sched = 1;
    }
    if ((rc = pinned_reserve(s, host_bytes))) return rc;
    st.write(s->h_cam);
    memcpy(s->h_cam + o_kp, &k, sizeof(KParams));
    for (const auto& r : st.runs())  // (the segments the device fills are not uploaded)
        if ((rc = pinned_upload(s, D + r.first, r.second - r.first, r.first))) return rc;
    slog.mark("upload");
    if (dev_faces) {
        if ((rc = mesh_bins_dev2(s, bins_x, (int32_t)(bstart.size() - 1), dev_pairs, reinterpret_cast<int32_t*>(D + o_bfaces),
                                 reinterpret_cast<float*>(D + o_bz))))
            return rc;
        slog.mark("device face bins (stage 2)");
    }
    s->d_kp = reinterpret_cast<KParams*>(D + o_kp);
    s->kp = k;
    s->cam_set = true;
    return RTX_OK;
}

namespace {
int render_launch(rtx_scene* s, Launch L, uint64_t* counters_dev, void* stream, bool out8, int32_t nframes = 1);

int render_rows(const char* fn, rtx_scene* s, int32_t row0, int32_t nrows, void* out_dev, uint64_t* counters_dev,
                void* stream, bool out8, int32_t nframes = 1, int64_t fstride = 0) {
    if (!s) return fail(RTX_ERR_INVALID, std::string(fn) + ": null scene");
    if (!s->cam_set) return fail(RTX_ERR_STATE, std::string(fn) + ": rtx_camera_set was not called");
    if (row0 < 0 || nrows < 0 || (int64_t)row0 + nrows > s->kp.height)
        return fail(RTX_ERR_INVALID, std::string(fn) + ": row range outside the image");
    const int64_t block_bytes = (int64_t)nrows * s->kp.ncols * 3 * (out8 ? 1 : 4);
    if (nframes < 1 || nframes > 65535 || (nframes > 1 && fstride < block_bytes) || (!out8 && fstride % 4))
        return fail(RTX_ERR_INVALID, std::string(fn) + ": need 1 <= nframes <= 65535 and frames that do not overlap");
    if (nrows == 0) return RTX_OK;
    if (!out_dev) return fail(RTX_ERR_INVALID, std::string(fn) + ": null framebuffer");
    Launch L;
    L.fb = static_cast<float*>(out_dev);
    L.row0 = row0;
    L.nrows = nrows;
    L.gphase = 0;
    L.gstride = 0;
    L.fstride = nframes > 1 ? fstride : 0;
    return render_launch(s, L, counters_dev, stream, out8, nframes);
}

int render_groups(const char* fn, rtx_scene* s, int32_t phase, int32_t stride, void* out_dev, uint64_t* counters_dev,
                  void* stream, bool out8, int32_t nframes = 1, int64_t fstride = 0) {
    if (!s) return fail(RTX_ERR_INVALID, std::string(fn) + ": null scene");
    if (!s->cam_set) return fail(RTX_ERR_STATE, std::string(fn) + ": rtx_camera_set was not called");
    const int32_t nrows = rtx_group_rows(s->kp.height, phase, stride);
    if (nrows < 0) return fail(RTX_ERR_INVALID, std::string(fn) + ": need 0 <= phase < stride");
    const int64_t block_bytes = (int64_t)nrows * s->kp.ncols * 3 * (out8 ? 1 : 4);
    if (nframes < 1 || nframes > 65535 || (nframes > 1 && fstride < block_bytes) || (!out8 && fstride % 4))
        return fail(RTX_ERR_INVALID, std::string(fn) + ": need 1 <= nframes <= 65535 and frames that do not overlap");
    if (nrows == 0) return RTX_OK;
    if (!out_dev) return fail(RTX_ERR_INVALID, std::string(fn) + ": null framebuffer");
    Launch L;
    L.fb = static_cast<float*>(out_dev);
    L.row0 = 0;
    L.nrows = nrows;
    L.gphase = phase;
    L.gstride = stride;
    L.fstride = nframes > 1 ? fstride : 0;
    return render_launch(s, L, counters_dev, stream, out8, nframes);
}
}  // namespace

int rtx_render(rtx_scene* s, int32_t row0, int32_t nrows, float* fb_dev, uint64_t* counters_dev, void* stream) {
    return render_rows("rtx_render", s, row0, nrows, fb_dev, counters_dev, stream, false);
}

int rtx_render_rgb8(rtx_scene* s, int32_t row0, int32_t nrows, uint8_t* out_dev, uint64_t* counters_dev,
                    void* stream) {
    return render_rows("rtx_render_rgb8", s, row0, nrows, out_dev, counters_dev, stream, true);
}

int rtx_render_frames(rtx_scene* s, int32_t row0, int32_t nrows, void* out_dev, int32_t rgb8, int32_t nframes,
                      int64_t frame_stride_bytes, uint64_t* counters_dev, void* stream) {
    return render_rows("rtx_render_frames", s, row0, nrows, out_dev, counters_dev, stream, rgb8 != 0, nframes,
                       frame_stride_bytes);
}

int rtx_render_groups_frames(rtx_scene* s, int32_t phase, int32_t stride, void* out_dev, int32_t rgb8,
                             int32_t nframes, int64_t frame_stride_bytes, uint64_t* counters_dev, void* stream) {
    return render_groups("rtx_render_groups_frames", s, phase, stride, out_dev, counters_dev, stream, rgb8 != 0,
                         nframes, frame_stride_bytes);
}

int32_t rtx_group_rows(int32_t height, int32_t phase, int32_t stride) {
    if (height < 0 || stride < 1 || phase < 0 || phase >= stride) return -1;
    const int32_t groups = (height + 7) / 8;
    if (phase >= groups) return 0;
    const int32_t mine = (groups - 1 - phase) / stride + 1;  // groups phase, phase + stride, ...
    int32_t rows = mine * 8;
    if ((groups - 1) % stride == phase) rows -= groups * 8 - height;  // the short last group
    return rows;
}

int rtx_render_groups(rtx_scene* s, int32_t phase, int32_t stride, float* fb_dev, uint64_t* counters_dev,
                      void* stream) {
    return render_groups("rtx_render_groups", s, phase, stride, fb_dev, counters_dev, stream, false);
}

int rtx_render_groups_rgb8(rtx_scene* s, int32_t phase, int32_t stride, uint8_t* out_dev, uint64_t* counters_dev,
                           void* stream) {
    return render_groups("rtx_render_groups_rgb8", s, phase, stride, out_dev, counters_dev, stream, true);
}

namespace {
bool stream_capturing(hipStream_t st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}

int launch_to_rgb8(const float* fb, uint8_t* out, int64_t n, hipStream_t st) {
    if ((reinterpret_cast<uintptr_t>(fb) & 15) == 0 && (reinterpret_cast<uintptr_t>(out) & 3) == 0)
        hipLaunchKernelGGL(k_to_rgb8, dim3((unsigned)((n / 4 + 256) / 256)), dim3(256), 0, st, fb, out, n);
    else
        hipLaunchKernelGGL(k_to_rgb8_unaligned, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, fb, out, n);
    RTX_HIP(hipGetLastError());
    return RTX_OK;
}

// The hierarchy/texture scenes in three passes (rtx_split.h), the default: NovelScene1
// 2048x1024 AA32 25.8 -> 22.3 ms, NovelScene2 133.9 -> 98.1 ms (twice on one box,
// profiles/r04/split/). Option split 0 launches the one-kernel form (render_body_spp).
bool split_enabled() { return opt_on(OPT_SPLIT); }

// The measured tile schedule (option tile_sched 0: off). A frame's 8x8 tiles cost very
// different amounts where some pixels follow long reflect/refract chains or cross a mesh
// (MirrorRefraction 1080p: waves of 2 to 32 us; TorusMesh: 4 to 28 us), and a long wave
// dispatched late sets the frame's end (profiles/r04/wave_timeline/). The first whole
// frame after a camera upload records each wave's duration; before the next whole frame
// the host sorts the tiles longest first (one stream synchronization per camera) and,
// where the durations are heavy-tailed (max > 3 x mean), later frames dispatch in that
// order (MirrorRefraction 41.4 -> 38.6 us, TorusMesh 52.8 -> 49.7 us with orders measured
// on the same box, profiles/r04/tile_order/; TwoSpheresPlane and DepthOfField gain
// nothing). The order changes when tiles run, not what they compute.
int tile_schedule(rtx_scene* s, hipStream_t st, uint32_t wpb) {
    if (s->tile_sched != 2) return RTX_OK;
    if (stream_capturing(st)) return RTX_OK;
    const int32_t n = s->kp.tile_n;
    std::vector<uint32_t> t((size_t)n);
    RTX_HIP(hipEventSynchronize(s->tile_event));  // the measuring launch (maybe on another stream)
    RTX_HIP(hipMemcpyAsync(t.data(), s->d_tile_time, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, st));
    RTX_HIP(hipStreamSynchronize(st));
    double sum = 0.0;
    uint32_t mx = 0;
    for (uint32_t v : t) { sum += v; mx = std::max(mx, v); }
    const double mean = n > 0 ? sum / n : 0.0;
    if (!(mean > 0.0) || (double)mx <= 3.0 * mean) {
        s->tile_sched = 4;
        return RTX_OK;
    }
    std::vector<int32_t> order((size_t)n);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return t[a] > t[b]; });
    s->tile_xcd = opt_on(OPT_XCD_MAP);  // (the frames that follow this table keep its layout)
    // the launch's blocks: its waves are the table's nw entries (rtx_camera_set pads the
    // tiles to whole 256-thread blocks), wpb per block. Dispatch position p (block p / wpb)
    // reads the entry of its slot (pixel_rc's xcd_block): the p-th dispatched wave renders
    // the p-th longest tile, and each XCD reads its own lines
    const uint32_t nw = (uint32_t)((n + kBlock<false> / 64 - 1) / (kBlock<false> / 64) * (kBlock<false> / 64));
    const uint32_t nb = nw / wpb;
    std::vector<int32_t> perm((size_t)nb * wpb);
    for (uint32_t p = 0; p < nb * wpb; ++p) {
        const uint32_t slot = (s->tile_xcd ? xcd_block(p / wpb, nb, wpb) : p / wpb) * wpb + p % wpb;
        perm[slot] = p < (uint32_t)n ? order[p] : (int32_t)p;
    }
    RTX_HIP(hipMemcpyAsync(s->d_tile_perm, perm.data(), sizeof(int32_t) * perm.size(), hipMemcpyHostToDevice, st));
    RTX_HIP(hipStreamSynchronize(st));  // (perm is a local: wait for the copy)
    s->tile_sched = 3;
    return RTX_OK;
}

// Record bytes of one chunk of the split passes (option split_bytes, default 2 GiB; 40 B
// per record): NovelScene1 (67 M samples, ~1.8 records each) renders in 3 chunks.
int64_t split_budget() { return (int64_t)std::max(4096.0, opt(OPT_SPLIT_BYTES)); }
// Option split_ratio >= 0: a fixed deeper-record pool per sample instead of the learned
// one (the tests force the redo path with a tiny pool).
double split_fixed_ratio() { return opt(OPT_SPLIT_RATIO) >= 0.0 ? opt(OPT_SPLIT_RATIO) : -1.0; }

// The deeper-record pool learns from the counters of an earlier frame once they have
// arrived on the host (never waits): at least 1/8 more than the fullest chunk needed.
void split_learn(rtx_scene* s, int levels) {
    if (!s->split_pending || hipEventQuery(s->split_read) != hipSuccess) return;
    s->split_pending = false;
    double need = 0.0;
    for (size_t c = 0; c < s->split_chunks.size(); ++c)
        if (s->split_chunks[c].first > 0)
            need = std::max(need, (double)s->h_split_count[c] / (double)s->split_chunks[c].first);
    const double want = std::min<double>(levels - 1, need * 1.125 + 1.0 / 64);
    if (want > s->split_ratio) s->split_ratio = want;
}

// Frees a split buffer, or keeps it for the scene's life when a captured graph may use it.
void split_release(rtx_scene* s, void* p) {
    if (!p) return;
    if (s->split_captured) s->split_retired.push_back(p);
    else (void)hipFree(p);
}

constexpr int64_t kRedoBlocks = 2048;  // grid of the split passes' redo launch

int render_split(rtx_scene* s, Launch L, const KParams* kp, size_t hbytes, hipStream_t st, int sel, int32_t nframes,
                 bool cnt) {
    constexpr int B = kBlock<true>;
    const int spp = s->kp.n_dof * s->kp.n_aa * s->kp.n_times;
    const int64_t npix = (int64_t)L.nrows * s->kp.ncols;
    if (npix <= 0 || nframes <= 0) return RTX_OK;
    const int levels = s->has_secondary ? kMaxDepth : 1;
    const int ppb = spp_pixels_per_block(spp, B);
    const bool capturing = stream_capturing(st);
    const double fixed = split_fixed_ratio();
    if (s->split_ratio < 0.0) s->split_ratio = levels > 1 ? 1.0 : 0.0;
    if (!capturing) split_learn(s, levels);
    // counting renders reserve every level (a redone block would count its rays twice)
    const double ratio = levels == 1 ? 0.0 : cnt ? (double)(levels - 1) : fixed >= 0.0 ? fixed : s->split_ratio;
    // the records of one chunk: within the budget and 3/4 of the device's free memory, the
    // budget halved when an allocation fails anyway
    int64_t budget = split_budget();
    {
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) == hipSuccess)
            budget = std::min<int64_t>(budget, (int64_t)((fr + (size_t)s->split_cap * kSpBytes) / 4 * 3));
    }
    SplitPlan pl;
    for (;;) {
        pl = split_plan(npix, spp, ppb, ratio, budget);
        if (pl.cap >= (1ll << 31) && pl.chunk > ppb) { budget /= 2; continue; }  // (record indices are int32)
        if (pl.cap >= (1ll << 31)) return fail(RTX_ERR_INVALID, "rtx_render: split chunk too large");
        if (s->split_cap >= pl.cap) break;
        if (capturing)
            return fail(RTX_ERR_STATE, "rtx_render: render a hierarchy/texture scene once before capturing it "
                                       "(its record buffer is allocated on first use)");
        split_release(s, s->d_split);
        s->d_split = nullptr;
        s->split_cap = 0;
        const hipError_t e = hipMalloc((void**)&s->d_split, (size_t)pl.cap * kSpBytes);
        if (e == hipSuccess) {
            s->split_cap = pl.cap;
            break;
        }
        s->d_split = nullptr;
        (void)hipGetLastError();
        if (e != hipErrorOutOfMemory || pl.chunk <= ppb)
            return fail(RTX_ERR_HIP, std::string("rtx_render: split records: ") + hipGetErrorString(e));
        budget = std::min(budget, pl.cap * kSpBytes) / 2;
    }
    const int64_t chunk = pl.chunk, cap = s->split_cap;
    const int64_t nchunk = (npix + chunk - 1) / chunk;
    const int64_t nblk = (chunk + ppb - 1) / ppb;
    if (s->split_nchunk_cap < nchunk || s->split_redo_cap < nblk) {
        if (capturing) return fail(RTX_ERR_STATE, "rtx_render: render a hierarchy/texture scene once before capturing it");
        if (s->split_pending) {
            (void)hipEventSynchronize(s->split_read);
            s->split_pending = false;
        }
    }
    if (s->split_nchunk_cap < nchunk) {
        split_release(s, s->d_split_count);
        (void)hipHostFree(s->h_split_count);
        s->d_split_count = nullptr;
        s->h_split_count = nullptr;
        s->split_nchunk_cap = 0;
        RTX_HIP(hipMalloc((void**)&s->d_split_count, 2 * sizeof(unsigned int) * nchunk));
        RTX_HIP(hipHostMalloc((void**)&s->h_split_count, 2 * sizeof(unsigned int) * nchunk));
        s->split_nchunk_cap = nchunk;
    }
    if (s->split_redo_cap < nblk) {  // flags all zero between renders: the redo launch clears what it lists
        split_release(s, s->d_split_redo);
        s->d_split_redo = nullptr;
        s->split_redo_cap = 0;
        RTX_HIP(hipMalloc((void**)&s->d_split_redo, 2 * sizeof(uint32_t) * nblk));
        RTX_HIP(hipMemsetAsync(s->d_split_redo, 0, 2 * sizeof(uint32_t) * nblk, st));
        s->split_redo_cap = nblk;
    }
    if (!s->split_read) RTX_HIP(hipEventCreateWithFlags(&s->split_read, hipEventDisableTiming));
    if (!s->split_done) RTX_HIP(hipEventCreateWithFlags(&s->split_done, hipEventDisableTiming));
    // one scene's renders share these buffers: a render on another stream waits for the last one
    if (!capturing && s->split_used && s->split_stream != st)
        RTX_HIP(hipStreamWaitEvent(st, s->split_done, 0));
    // the trace and shadow passes specialized on the scene's CSG trees, when compiled
    // (jit_split_kernel; the precompiled passes render meanwhile: the same bytes)
    JitSlot* sk[3];
    for (int pass = 0; pass < 3; ++pass) {
        // (the shade pass has no counter or jitter variants: one slot; option csg_shade)
        JitSlot& r = s->resolved[pass == 2 ? 24 : 16 + 4 * pass + (cnt ? 2 : 0) + ((sel & 1) ? 1 : 0)];
        if (pass == 2 && !r.done && !opt_on(OPT_CSG_SHADE)) {
            r.done = true;  // (the precompiled shade pass)
            r.fn = nullptr;
        }
        if (!r.done) {
            r.block = B;
            // option jit_csg 2 / 3: the camera's boxes / and the object records as literals too
            const int bake = opt(OPT_JIT_CSG) >= 3.0 ? 3 : opt(OPT_JIT_CSG) >= 2.0 ? 2 : 0;
            const bool can = !s->csg_tables.empty() && s->tr_valid && s->tr_bounds.size() == s->h_nodes.size();
            r.lds = pass < 2 && (((int)opt(OPT_CSG_RAYS) >> pass) & 1) == 0;
            std::vector<std::string> fixed;
            jit_fixed_opts(s->view, s->kp, s->traits, false, fixed);
            jit_split_kernel(s->device,
                             bake && can ? s->csg_tables + jit_csg_baked(s->tr_bounds, s->h_objs, bake) : s->csg_tables,
                             s->has_mesh, s->has_secondary, cnt, (sel & 1) != 0, pass, !r.lds, fixed, r);
            if (r.pending && !opt_on(OPT_JIT_ASYNC) && !capturing) jit_poll(r, true);
            r.done = true;
        } else if (r.pending && !capturing) {
            jit_poll(r, false);
        }
        sk[pass] = &r;
    }
    if (sk[0]->fn && sk[1]->fn && jit_enabled()) {
        s->last_kernel = "rtx_jit_split_";
        for (bool f : {s->has_mesh, s->has_secondary, cnt, (sel & 1) != 0}) s->last_kernel += f ? '1' : '0';
    }
    auto launch = [&](int pass, const RenderLaunch& r, const Launch& Lc, const SplitBuf& sb) {
        if (sk[pass]->fn && jit_enabled()) {
            const KParams* kpp = r.kp;
            Launch La = Lc;
            SplitBuf sbb = sb;
            void* args[] = {(void*)&kpp, (void*)&La, (void*)&sbb};
            // (rays in registers: no LDS stack, option csg_rays)
            const unsigned lds = sk[pass]->lds ? (unsigned)r.lds_bytes : 0u;
            return hipModuleLaunchKernel(sk[pass]->fn, r.nblocks, 1, 1, B, 1, 1, lds, r.stream, args, nullptr);
        }
        return s->has_mesh ? launch_split_m1(sel, pass, r, Lc, sb) : launch_split_m0(sel, pass, r, Lc, sb);
    };
    char* base = reinterpret_cast<char*>(L.fb);
    for (int32_t f = 0; f < nframes; ++f) {
        Launch Lc = L;
        Lc.fb = reinterpret_cast<float*>(base + f * L.fstride);
        Lc.fstride = 0;
        Lc.redo = RedoList{nullptr, nullptr, nullptr};
        RTX_HIP(hipMemsetAsync(s->d_split_count, 0, 2 * sizeof(unsigned int) * nchunk, st));
        int64_t c = 0;
        for (int64_t p0 = 0; p0 < npix; p0 += chunk, ++c) {
            const int64_t np = std::min(chunk, npix - p0), nq = np * spp;
            Lc.pix0 = (int32_t)p0;
            uint32_t* const redo_n = s->d_split_count + nchunk + c;
            uint32_t* const redo_list = s->d_split_redo;
            uint32_t* const redo_flag = s->d_split_redo + s->split_redo_cap;
            const SplitBuf sb{s->d_split, s->d_split_count + c, redo_n, redo_list, redo_flag, nq, cap};
            RenderLaunch r{kp, (unsigned)((nq + B - 1) / B), 1u, hbytes * B, st, true};
            RTX_HIP(launch(0, r, Lc, sb));
            RTX_HIP(launch(1, r, Lc, sb));
            r.nblocks = (unsigned)((np + ppb - 1) / ppb);
            RTX_HIP(launch(2, r, Lc, sb));
            // the blocks whose chains found the pool full, again in the one-kernel form: a
            // small grid strides over the list (a few microseconds when it is empty)
            if (levels > 1) {
                Launch Lf = Lc;
                Lf.redo = RedoList{redo_n, redo_list, redo_flag};
                r.nblocks = (unsigned)std::min<int64_t>((np + ppb - 1) / ppb, kRedoBlocks);
                RTX_HIP(s->has_mesh ? launch_render_ext_m1(sel, r, Lf) : launch_render_ext_m0(sel, r, Lf));
            }
        }
    }
    if (!capturing) {
        if (levels > 1 && !cnt && fixed < 0.0 && !s->split_pending) {  // what this frame's chains used
            RTX_HIP(hipMemcpyAsync(s->h_split_count, s->d_split_count, sizeof(unsigned int) * nchunk,
                                   hipMemcpyDeviceToHost, st));
            RTX_HIP(hipEventRecord(s->split_read, st));
            s->split_chunks.clear();
            for (int64_t p0 = 0; p0 < npix; p0 += chunk) s->split_chunks.emplace_back(std::min(chunk, npix - p0) * spp, cap);
            s->split_pending = true;
        }
        RTX_HIP(hipEventRecord(s->split_done, st));
        s->split_stream = st;
        s->split_used = true;
    } else {
        s->split_captured = true;
    }
    return RTX_OK;
}

int render_launch(rtx_scene* s, Launch L, uint64_t* counters_dev, void* stream, bool out8, int32_t nframes) {
    const int32_t nrows = L.nrows;
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess || cur != s->device)
        return fail(RTX_ERR_STATE, "rtx_render: the scene lives on device " + std::to_string(s->device) +
                                       ", the current device is " + std::to_string(cur));
    L.counters = reinterpret_cast<unsigned long long*>(counters_dev);
    hipStream_t st = (hipStream_t)stream;
    const bool cnt = counters_dev != nullptr;
    const bool jit = s->kp.jitter != RTX_JITTER_OFF;
    const int sel = (s->has_mesh ? 16 : 0) | (s->has_secondary ? 8 : 0) | (s->has_ext ? 4 : 0) | (cnt ? 2 : 0) | (jit ? 1 : 0);
    const KParams* kp = s->d_kp;
    const size_t hbytes = (size_t)s->hlevels * 9 * sizeof(float);
    const int blk = s->has_ext ? kBlock<true> : kBlock<false>;
    const int spp = s->kp.n_dof * s->kp.n_aa * s->kp.n_times;
    const bool spp_mode = use_spp_mode(spp, s->has_ext);
    // pixel mapping: one lane per pixel (8x8 tiles per wave); sample-parallel: blocks of
    // spp_pixels_per_block pixels (rtx_kernels.h render_body_spp)
    auto blocks = [&](bool sm) {
        return sm ? ((int64_t)nrows * s->kp.ncols + spp_pixels_per_block(spp, blk) - 1) / spp_pixels_per_block(spp, blk)
                  : (launch_items(nrows, s->kp.ncols) + blk - 1) / blk;
    };
    int64_t nblocks = blocks(spp_mode);
    if (nblocks > 0x7fffffff || blocks(false) > 0x7fffffff) return fail(RTX_ERR_INVALID, "rtx_render: launch too large");
    {
#if RTX_TILE_ORDER == 2  // (experiment builds only): a multiplier coprime to the launch's wave count
        const uint64_t T = (uint64_t)nblocks * (blk / 64) * RTX_PPL;
        uint64_t m = std::max<uint64_t>(1, (uint64_t)((double)T * 0.6180339887498949));
        while (T > 1 && std::gcd(m, T) != 1) ++m;
        L.perm = (uint32_t)(T > 1 ? m % T : 1);
#else
        L.perm = 1;
#endif
        L.pix0 = 0;
        L.tperm = 0;
        L.tlog = 0;
        L.xcd = opt_on(OPT_XCD_MAP) ? 1 : 0;
        L.redo = RedoList{nullptr, nullptr, nullptr};
    }
    // the heavy tiles' chunks of a tile-mapped launch, just before it (the sample-parallel
    // and split kernels pass no pixel-in-tile and walk the lists). One pass serves every
    // frame of a batched launch: the frames share the camera, and the chunks test the mesh
    // at times[0] (meshes do not move, provided/geometry/mesh.py ignores speed)
    auto heavy_pass = [&](bool tiles) -> int {
        if (s->heavy_n <= 0 || !tiles || s->has_ext) return RTX_OK;
        hipLaunchKernelGGL(k_mesh_chunks, dim3((unsigned)s->heavy_n), dim3(64), 0, st, kp, L,  // (a wave per chunk)
                           s->d_heavy_items, s->heavy_n, s->d_mesh_hits, (int32_t)opt(OPT_CHUNK_MODE));
        RTX_HIP(hipGetLastError());
        return RTX_OK;
    };
    JitSlot& rs = s->resolved[(out8 ? 8 : 0) | (cnt ? 4 : 0) | (jit ? 2 : 0) | (spp_mode ? 1 : 0)];
    if (!rs.done) {
        rs.block = jit_block(s->has_mesh, s->has_secondary, s->has_ext, spp_mode);
        jit_render_kernel(s->device, s->view, s->kp, s->traits, s->has_mesh, s->has_secondary, s->has_ext, cnt, jit,
                          spp_mode, out8, s->jit_baked, rs);
        if (rs.pending && !opt_on(OPT_JIT_ASYNC) && !stream_capturing(st)) jit_poll(rs, true);
        rs.done = true;
    } else if (rs.pending && !stream_capturing(st)) {
        jit_poll(rs, false);  // (a capture records the kernel that runs now: no module load inside it)
    }
    if (rs.fn && jit_enabled()) {
        void* args[] = {(void*)&kp, (void*)&L};
        // whole-frame launches follow the measured tile schedule
        const bool whole = s->tile_sched != 0 && !spp_mode && L.row0 == 0 && L.nrows == s->kp.height &&
                           L.gstride == 0;
        // (a captured launch neither measures nor sorts: its replays run later, and the
        // schedule's state machine follows eager frames only)
        const bool capturing = whole && stream_capturing(st);
        if (whole && !capturing) {
            if (int rc = tile_schedule(s, st, (uint32_t)rs.block / 64)) return rc;
            L.tlog = s->tile_sched == 1;
        }
        if (whole) L.tperm = s->tile_sched == 3;
        if (L.tperm) L.xcd = s->tile_xcd ? 1 : 0;
        if (int rc = heavy_pass(!spp_mode)) return rc;
        // (a one-wave-block kernel: the same waves in four times the blocks)
        const int64_t jblocks = rs.block == blk ? nblocks : nblocks * (blk / rs.block);  // (blk: 256 here)
        RTX_HIP(hipModuleLaunchKernel(rs.fn, (unsigned)jblocks, (unsigned)nframes, 1, rs.block, 1, 1,
                                      s->has_ext ? (unsigned)(hbytes * rs.block) : 0u, st, args, nullptr));
        if (L.tlog) {  // measured: sorted before the next whole frame
            if (!s->tile_event) RTX_HIP(hipEventCreateWithFlags(&s->tile_event, hipEventDisableTiming));
            RTX_HIP(hipEventRecord(s->tile_event, st));
            s->tile_sched = 2;
        }
        s->last_kernel = L.tperm ? rs.name + "+tiles" : rs.name;
        return RTX_OK;
    }
    if (out8 && nframes > 1) {  // generic kernels: the uint8 fallback below, one frame at a time
        char* base = reinterpret_cast<char*>(L.fb);
        const int64_t fstride = L.fstride;
        L.fstride = 0;
        for (int32_t f = 0; f < nframes; ++f) {
            L.fb = reinterpret_cast<float*>(base + f * fstride);
            if (int rc = render_launch(s, L, counters_dev, stream, true, 1)) return rc;
        }
        return RTX_OK;
    }
    if (out8) {  // no specialized uint8 kernel: fp32 into the scene's scratch, then convert
        const size_t n = (size_t)nrows * s->kp.ncols * 3;
        if (s->scratch_floats < n) {
            (void)hipFree(s->d_scratch);
            s->d_scratch = nullptr;
            s->scratch_floats = 0;
            RTX_HIP(hipMalloc((void**)&s->d_scratch, n * sizeof(float)));
            s->scratch_floats = n;
        }
        uint8_t* out = reinterpret_cast<uint8_t*>(L.fb);
        L.fb = s->d_scratch;
        if (int rc = render_launch(s, L, counters_dev, stream, false)) return rc;
        s->last_kernel += "+k_to_rgb8";
        return launch_to_rgb8(s->d_scratch, out, (int64_t)n, st);
    }
    char gname[48];
    snprintf(gname, sizeof(gname), "%s_%d%d%d%d%d%s", s->has_ext ? "k_render_ext" : "k_render", s->has_mesh ? 1 : 0,
             s->has_secondary ? 1 : 0, s->has_ext ? 1 : 0, cnt ? 1 : 0, jit ? 1 : 0,
             (spp_mode && s->has_ext) ? "_spp" : "");
    s->last_kernel = gname;
    if (s->has_ext && split_enabled() && s->view.n_lights <= 32 && s->view.n_mats <= kSpMaxMats &&
        s->kp.n_times <= kSpMaxTimes) {
        snprintf(gname, sizeof(gname), "k_split_%d%d%d%d", s->has_mesh ? 1 : 0, s->has_secondary ? 1 : 0, cnt ? 1 : 0,
                 jit ? 1 : 0);
        s->last_kernel = gname;
        return render_split(s, L, kp, hbytes, st, sel & 11, nframes, cnt);
    }
    if (s->has_ext) {  // precompiled in rtx_kern_ext_m{0,1}.hip
        const RenderLaunch rl{kp, (unsigned)nblocks, (unsigned)nframes, hbytes * kBlock<true>, st, spp_mode};
        RTX_HIP(s->has_mesh ? launch_render_ext_m1(sel, rl, L) : launch_render_ext_m0(sel, rl, L));
        return RTX_OK;
    }
    // the flat-scene kernels use the tile mapping here (their sample-parallel variants
    // are reached through the scene-specialized kernels only)
    if (spp_mode) nblocks = blocks(false);
    if (int rc = heavy_pass(true)) return rc;
#define RTX_LAUNCH(M, S, C, J) \
    hipLaunchKernelGGL((k_render<M, S, false, C, J>), dim3((unsigned)nblocks, (unsigned)nframes), dim3(kBlock<false>), \
                       0, st, kp, L)
#define RTX_CASE(n) \
    case n: RTX_LAUNCH(((n) & 16) != 0, ((n) & 8) != 0, ((n) & 2) != 0, ((n) & 1) != 0); break
    switch (sel) {
        RTX_CASE(0); RTX_CASE(1); RTX_CASE(2); RTX_CASE(3);
        RTX_CASE(8); RTX_CASE(9); RTX_CASE(10); RTX_CASE(11);
        RTX_CASE(16); RTX_CASE(17); RTX_CASE(18); RTX_CASE(19);
        RTX_CASE(24); RTX_CASE(25); RTX_CASE(26); RTX_CASE(27);
    }
#undef RTX_CASE
#undef RTX_LAUNCH
    RTX_HIP(hipGetLastError());
    return RTX_OK;
}
}  // namespace

namespace {
// The scene view for one motion time (hierarchy bounds uploaded in stream order).
int view_at(rtx_scene* s, double time, hipStream_t stream, SceneView& v) {
    v = s->view;
    if (s->h_nodes.empty()) return RTX_OK;
    const float t = (float)time;
    s->h_bounds_abi = split_bounds(compute_bounds(s->h_nodes, s->h_objs, s->h_tris, t, t));
    RTX_HIP(hipMemcpyAsync(s->d_bounds_abi, s->h_bounds_abi.data(), sizeof(DBox) * s->h_bounds_abi.size(),
                           hipMemcpyHostToDevice, stream));
    bind_boxes(v, (const DBox*)s->d_bounds_abi, s->h_nodes.size());
    return RTX_OK;
}
}  // namespace

int rtx_intersect(rtx_scene* s, int64_t n, const float* ro, const float* rd, double time, double* t_dev,
                  int32_t* obj_dev, int32_t* mat_dev, float* normal_dev, float* position_dev, void* stream) {
    if (!s || n < 0 || (n > 0 && (!ro || !rd))) return fail(RTX_ERR_INVALID, "rtx_intersect: bad argument");
    if (n == 0) return RTX_OK;
    SceneView view;
    int rc = view_at(s, time, (hipStream_t)stream, view);
    if (rc) return rc;
    const dim3 grid((unsigned)((n + 255) / 256)), block(256);
    const size_t lds = s->has_ext ? (size_t)s->hlevels * 9 * sizeof(float) * 256 : 0;
#define RTX_ISECT(M, X)                                                                                          \
    hipLaunchKernelGGL((k_intersect<M, X>), grid, block, lds, (hipStream_t)stream, view, n, ro, rd, (float)time, \
                       t_dev, obj_dev, mat_dev, normal_dev, position_dev)
    if (s->has_mesh) { if (s->has_ext) RTX_ISECT(true, true); else RTX_ISECT(true, false); }
    else { if (s->has_ext) RTX_ISECT(false, true); else RTX_ISECT(false, false); }
#undef RTX_ISECT
    RTX_HIP(hipGetLastError());
    return RTX_OK;
}

int rtx_occluded(rtx_scene* s, int64_t n, const float* ro, const float* rd, const double* tmax, double time,
                 uint8_t* occ, void* stream) {
    if (!s || n < 0 || (n > 0 && (!ro || !rd || !tmax || !occ))) return fail(RTX_ERR_INVALID, "rtx_occluded: bad argument");
    if (n == 0) return RTX_OK;
    SceneView view;
    int rc = view_at(s, time, (hipStream_t)stream, view);
    if (rc) return rc;
    const dim3 grid((unsigned)((n + 255) / 256)), block(256);
    const size_t lds = s->has_ext ? (size_t)s->hlevels * 9 * sizeof(float) * 256 : 0;
#define RTX_OCC(M, X) \
    hipLaunchKernelGGL((k_occluded<M, X>), grid, block, lds, (hipStream_t)stream, view, n, ro, rd, tmax, (float)time, occ)
    if (s->has_mesh) { if (s->has_ext) RTX_OCC(true, true); else RTX_OCC(true, false); }
    else { if (s->has_ext) RTX_OCC(false, true); else RTX_OCC(false, false); }
#undef RTX_OCC
    RTX_HIP(hipGetLastError());
    return RTX_OK;
}

int rtx_fb_to_rgb8(const float* fb, uint8_t* out, int64_t n, void* stream) {
    if (n < 0 || (n > 0 && (!fb || !out))) return fail(RTX_ERR_INVALID, "rtx_fb_to_rgb8: bad argument");
    if (n == 0) return RTX_OK;
    return launch_to_rgb8(fb, out, n, (hipStream_t)stream);
}

}  // extern "C"
