// rtx_hostemu.hip — TESTS ONLY. Runs the device source of librtx.so (rtx_api.hip +
// rtx_trace.h, unchanged) on the host CPU so kernel logic can be checked against the
// oracle in a container without a GPU. Not part of the product: the product path
// (python-raytracer_amd/rtx) never loads this library, and it has no HIP calls.
#include "../../python-raytracer_amd/csrc/rtx_api.hip"

// the hierarchy/texture kernels live in their own translation units; the host emulation
// never launches a kernel
namespace rtx {
hipError_t launch_render_ext_m0(int, const RenderLaunch&, const Launch&) { return hipErrorNotSupported; }
hipError_t launch_render_ext_m1(int, const RenderLaunch&, const Launch&) { return hipErrorNotSupported; }
hipError_t launch_split_m0(int, int, const RenderLaunch&, const Launch&, const SplitBuf&) { return hipErrorNotSupported; }
hipError_t launch_split_m1(int, int, const RenderLaunch&, const Launch&, const SplitBuf&) { return hipErrorNotSupported; }
void mesh_bins_warm() {}
size_t mesh_bins_bytes1(int32_t, int32_t) { return 0; }
size_t mesh_bins_bytes2(int32_t, int32_t) { return 0; }
hipError_t mesh_bins_stage1(const BinProj&, const float*, int32_t, int32_t, int32_t, int32_t, void*, MeshBinsDev&,
                            hipStream_t) { return hipErrorNotSupported; }
hipError_t mesh_bins_stage2(MeshBinsDev&, int32_t, int32_t, int32_t, int32_t, void*, int32_t*, float*, hipStream_t) {
    return hipErrorNotSupported;
}
}  // namespace rtx

#include <omp.h>
#include <chrono>

namespace {
void bind_view(const HostScene& H, SceneView& v) {
    v.objs = (cptr<DObj>)H.objs.data();
    v.tris = (cptr<DTri>)H.tris.data();
    v.trins = (cptr<DTriN>)H.trins.data();
    v.fboxes = (cptr<DFaceBox>)H.fboxes.data();
    v.mats = (cptr<DMat>)H.mats.data();
    v.lights = (cptr<DLight>)H.lights.data();
    v.leaves = (cptr<DLeaf>)H.leaves.data();
    v.tri_orig = (cptr<int32_t>)H.tri_orig.data();
    v.n_objs = H.n_objs;
    v.n_lights = H.n_lights;
    v.n_plane = H.n_plane; v.n_sphere = H.n_sphere; v.n_box = H.n_box; v.n_mesh = H.n_mesh;
    v.pow_bits = H.pow_bits;
    std::memcpy(v.ambient, H.ambient, sizeof(v.ambient));
    v.texels = (cptr<uint32_t>)H.texels.data();
    v.lut255 = (cptr<float>)H.lut255.data();
    v.n_nodes = (int32_t)H.nodes.size();
    v.hlevels = H.hlevels;
}

// The device forms of the hierarchy records, as rtx_scene_create / rtx_camera_set upload
// them: split nodes and the boxes for the time range [tlo, thi].
struct Nodes {
    std::vector<DNodeHot> hot;
    std::vector<DNodeMat> mat;
    std::vector<DBound> bounds;
    std::vector<DBox> boxes;
    void bind(const HostScene& H, SceneView& v, float tlo, float thi) {
        split_nodes(H.nodes, hot, mat);
        bounds = compute_bounds(H.nodes, H.objs, H.tris, tlo, thi);
        boxes = split_bounds(bounds);
        v.nodes = (cptr<DNodeHot>)hot.data();
        v.nmat = (cptr<DNodeMat>)mat.data();
        bind_boxes(v, boxes.data(), H.nodes.size());
    }
};

// The light grids rtx_scene_create builds (RTX_LGRID=0: none), bound to the view.
struct Grids {
    std::vector<DLGrid> grids;
    std::vector<int32_t> start, faces;
    std::vector<float> d2;
    void bind(const HostScene& H, SceneView& v) {
        if (!opt_on(OPT_LGRID) || !light_grids(H, grids, start, faces, d2)) return;
        if (faces.empty()) { faces.push_back(0); d2.push_back(0.0f); }
        v.lgrid = (cptr<DLGrid>)grids.data();
        v.lg_start = (cptr<int32_t>)start.data();
        v.lg_faces = (cptr<int32_t>)faces.data();
        v.lg_d2 = (cptr<float>)d2.data();
        v.lgrid_on = 1;
    }
};

// The directional lights' shadow grids rtx_camera_set builds for the motion-time range
// [tlo, thi] (RTX_DSGRID=0: none).
struct DirGrids {
    std::vector<DSGrid> grids;
    std::vector<DSCell> cells;
    std::vector<float> pself;
    void bind(const HostScene& H, SceneView& v, float tlo, float thi, double omax = INFINITY) {
        // the planes' self tests, as rtx_camera_set
        if (opt_on(OPT_SELF_SKIP) && H.n_plane > 0 && !H.lights.empty()) {
            pself = plane_self_limits(H, omax);
            v.plane_self = (cptr<float>)pself.data();
        }
        if (!opt_on(OPT_DSGRID)) return;
        std::vector<DBound> nb;
        if (!H.nodes.empty()) nb = compute_bounds(H.nodes, H.objs, H.tris, tlo, thi);
        if (!dir_shadow_grids(H, nb, tlo, thi, grids, cells)) return;
        dir_self_boxes(H, grids, omax);
        v.dsgrid = (cptr<DSGrid>)grids.data();
        v.dsg_cells = (cptr<DSCell>)cells.data();
        v.dsg_on = 1;
    }
};

// The heavy tiles' chunks (rtx_api.hip heavy_chunks, rtx_kernels.h mesh_chunk), as the
// k_mesh_chunks pass computes them before each frame, for every chunk and pixel.
struct Heavy {
    std::vector<int32_t> bheavy;
    std::vector<int2> items;
    std::vector<uint2> hits;
    void bind(const HostScene& H, KParams& k, const std::vector<int32_t>& bstart) {
        if (!k.S.bins_on || !k.S.mesh_bins || H.has_ext || !heavy_chunks(bstart, bheavy, items)) return;
        hits.resize(items.size() * 64);
        k.S.bin_heavy = (cptr<int32_t>)bheavy.data();
#pragma omp parallel for schedule(dynamic, 4)
        for (int64_t w = 0; w < (int64_t)items.size(); ++w)
            for (int lane = 0; lane < 64; ++lane)
                hits[(size_t)w * 64 + lane] = mesh_chunk(k, items[(size_t)w].x, items[(size_t)w].y, lane);
        k.S.mesh_hits = hits.data();
    }
};

// Dispatch over the kernel template flags, as rtx_render's launch switch does.
template <bool MESH, bool SEC, bool X>
void pixel_jit(const KParams& k, float* fb, int32_t row0, int32_t rr, int32_t cc, Tally& tl, const FrameStack& fs,
               const HStack& hs, bool jit, int32_t bin) {
    if (jit) render_pixel<MESH, SEC, X, true, true>(k, fb, row0, rr, cc, tl, fs, hs, bin);
    else render_pixel<MESH, SEC, X, true, false>(k, fb, row0, rr, cc, tl, fs, hs, bin);
}
void pixel_any(const HostScene& H, const KParams& k, float* fb, int32_t row0, int32_t rr, int32_t cc, Tally& tl,
               const FrameStack& fs, const HStack& hs, bool jit, int32_t tile_row) {
    // the face bin of the pixel's 8x8 tile, as render_body picks it (image row of the
    // tile's first row, strip column of its first column)
    const int32_t bin = primary_bin(k.S, tile_row, cc & ~7);
    const int sel = (H.has_mesh ? 4 : 0) | (H.has_secondary ? 2 : 0) | (H.has_ext ? 1 : 0);
    switch (sel) {
        case 0: pixel_jit<false, false, false>(k, fb, row0, rr, cc, tl, fs, hs, jit, bin); break;
        case 1: pixel_jit<false, false, true>(k, fb, row0, rr, cc, tl, fs, hs, jit, bin); break;
        case 2: pixel_jit<false, true, false>(k, fb, row0, rr, cc, tl, fs, hs, jit, bin); break;
        case 3: pixel_jit<false, true, true>(k, fb, row0, rr, cc, tl, fs, hs, jit, bin); break;
        case 4: pixel_jit<true, false, false>(k, fb, row0, rr, cc, tl, fs, hs, jit, bin); break;
        case 5: pixel_jit<true, false, true>(k, fb, row0, rr, cc, tl, fs, hs, jit, bin); break;
        case 6: pixel_jit<true, true, false>(k, fb, row0, rr, cc, tl, fs, hs, jit, bin); break;
        case 7: pixel_jit<true, true, true>(k, fb, row0, rr, cc, tl, fs, hs, jit, bin); break;
    }
}
}  // namespace

extern "C" int rtx_hostemu_render(const rtx_scene_desc* sd, const rtx_camera_desc* cd, int32_t row0, int32_t nrows,
                                  float* fb, uint64_t* counters, int threads) {
    HostScene H;
    int rc = convert_scene(sd, H);
    if (rc) return rc;
    KParams k;
    if ((rc = convert_camera(cd, k))) return rc;
    if (row0 < 0 || nrows < 0 || row0 + nrows > cd->height) return fail(RTX_ERR_INVALID, "bad rows");
    bind_view(H, k.S);
    Grids lg;
    lg.bind(H, k.S);
    std::vector<float> times(cd->n_times);
    for (int i = 0; i < cd->n_times; ++i) times[i] = (float)cd->times[i];
    const auto mm = std::minmax_element(times.begin(), times.end());
    Nodes nv;
    nv.bind(H, k.S, *mm.first, *mm.second);
    DirGrids dg;
    dg.bind(H, k.S, *mm.first, *mm.second, camera_origin_bound(cd));
    std::vector<int32_t> bstart, bfaces;
    std::vector<float> bz;
    std::vector<uint32_t> bmask, brmask;
    int32_t bins_x = 0, mesh_bins = 0;
    if (opt_on(OPT_BINS) && primary_bins(H, cd, nv.bounds, bstart, bfaces, bz, bmask, brmask, bins_x, mesh_bins)) {
        if (bfaces.empty()) { bfaces.push_back(0); bz.push_back(0.0f); }
        k.S.bin_start = (cptr<int32_t>)bstart.data();
        k.S.bin_faces = (cptr<int32_t>)bfaces.data();
        k.S.bin_zmin = (cptr<float>)bz.data();
        k.S.bin_objmask = (cptr<uint32_t>)bmask.data();
        k.S.bin_rootmask = (cptr<uint32_t>)brmask.data();
        k.S.mesh_bins = mesh_bins;
        k.S.bins_x = bins_x;
        k.S.bins_on = 1;
    }
    std::vector<float> noise;
    const size_t nsamp = (size_t)cd->n_dof * cd->n_aa;
    if (cd->jitter == RTX_JITTER_REPLAY) noise.assign(cd->noise, cd->noise + 3 * (size_t)cd->ncols * cd->height * nsamp);
    k.xs = (cptr<float>)cd->xs; k.ys = (cptr<float>)cd->ys; k.dof_o = (cptr<float>)cd->dof_origins;
    k.aa_o = (cptr<float>)cd->aa_origins; k.times = (cptr<float>)times.data(); k.noise = (cptr<float>)noise.data();
    Heavy hv;
    hv.bind(H, k, bstart);
    const int64_t npix = (int64_t)nrows * k.ncols;
    uint64_t tot[RTX_COUNTERS] = {};
#pragma omp parallel num_threads(threads > 0 ? threads : 1)
    {
        uint64_t loc[RTX_COUNTERS] = {};
#pragma omp for schedule(dynamic, 64)
        for (int64_t p = 0; p < npix; ++p) {
            Tally tl = {};
            float frames[kMaxDepth * 4];
            float hst[kMaxHLevels * 9];
            const FrameStack fs{frames, 1};
            const HStack hs{hst, 1};
            const int32_t rr = (int32_t)(p / k.ncols), cc = (int32_t)(p % k.ncols);
            pixel_any(H, k, fb, row0, rr, cc, tl, fs, hs, k.jitter != RTX_JITTER_OFF, row0 + (rr & ~7));
            for (int q = 0; q < kMaxDepth; ++q) loc[q] += tl.cast[q];
            loc[RTX_CNT_SHADOW] += tl.shadow;
            loc[RTX_CNT_SHADE] += tl.shade;
            loc[RTX_CNT_TRI] += tl.tri;
        }
#pragma omp critical
        for (int q = 0; q < RTX_COUNTERS; ++q) tot[q] += loc[q];
    }
    if (counters)
        for (int q = 0; q < RTX_COUNTERS; ++q) counters[q] = tot[q];
    return RTX_OK;
}

// The packed image rows rows[0..nrows) (row 0 = top), as one rank renders its share of a
// frame (rtx_render's contiguous block or rtx_render_groups' interleaved 8-row groups).
extern "C" int rtx_hostemu_render_rows(const rtx_scene_desc* sd, const rtx_camera_desc* cd, const int32_t* rows,
                                       int32_t nrows, float* fb, int threads) {
    HostScene H;
    int rc = convert_scene(sd, H);
    if (rc) return rc;
    KParams k;
    if ((rc = convert_camera(cd, k))) return rc;
    for (int32_t r = 0; r < nrows; ++r)
        if (rows[r] < 0 || rows[r] >= cd->height) return fail(RTX_ERR_INVALID, "bad rows");
    bind_view(H, k.S);
    Grids lg;
    lg.bind(H, k.S);
    std::vector<float> times(cd->n_times);
    for (int i = 0; i < cd->n_times; ++i) times[i] = (float)cd->times[i];
    const auto mm = std::minmax_element(times.begin(), times.end());
    Nodes nv;
    nv.bind(H, k.S, *mm.first, *mm.second);
    DirGrids dg;
    dg.bind(H, k.S, *mm.first, *mm.second, camera_origin_bound(cd));
    std::vector<int32_t> bstart, bfaces;
    std::vector<float> bz;
    std::vector<uint32_t> bmask, brmask;
    int32_t bins_x = 0, mesh_bins = 0;
    if (opt_on(OPT_BINS) && primary_bins(H, cd, nv.bounds, bstart, bfaces, bz, bmask, brmask, bins_x, mesh_bins)) {
        if (bfaces.empty()) { bfaces.push_back(0); bz.push_back(0.0f); }
        k.S.bin_start = (cptr<int32_t>)bstart.data();
        k.S.bin_faces = (cptr<int32_t>)bfaces.data();
        k.S.bin_zmin = (cptr<float>)bz.data();
        k.S.bin_objmask = (cptr<uint32_t>)bmask.data();
        k.S.bin_rootmask = (cptr<uint32_t>)brmask.data();
        k.S.mesh_bins = mesh_bins;
        k.S.bins_x = bins_x;
        k.S.bins_on = 1;
    }
    std::vector<float> noise;
    const size_t nsamp = (size_t)cd->n_dof * cd->n_aa;
    if (cd->jitter == RTX_JITTER_REPLAY) noise.assign(cd->noise, cd->noise + 3 * (size_t)cd->ncols * cd->height * nsamp);
    k.xs = (cptr<float>)cd->xs; k.ys = (cptr<float>)cd->ys; k.dof_o = (cptr<float>)cd->dof_origins;
    k.aa_o = (cptr<float>)cd->aa_origins; k.times = (cptr<float>)times.data(); k.noise = (cptr<float>)noise.data();
    Heavy hv;
    hv.bind(H, k, bstart);
    const int64_t npix = (int64_t)nrows * k.ncols;
#pragma omp parallel for num_threads(threads > 0 ? threads : 1) schedule(dynamic, 64)
    for (int64_t p = 0; p < npix; ++p) {
        Tally tl = {};
        float frames[kMaxDepth * 4];
        float hst[kMaxHLevels * 9];
        const FrameStack fs{frames, 1};
        const HStack hs{hst, 1};
        const int32_t rr = (int32_t)(p / k.ncols), cc = (int32_t)(p % k.ncols);
        // render_pixel's image row is row0 + rr
        pixel_any(H, k, fb, rows[rr] - rr, rr, cc, tl, fs, hs, k.jitter != RTX_JITTER_OFF, rows[rr & ~7]);
    }
    return RTX_OK;
}

extern "C" int rtx_hostemu_intersect(const rtx_scene_desc* sd, int64_t n, const float* ro, const float* rd, double time,
                                     double* t_out, int32_t* obj_out, int32_t* mat_out, float* n_out, float* p_out) {
    HostScene H;
    int rc = convert_scene(sd, H);
    if (rc) return rc;
    SceneView v{};
    bind_view(H, v);
    Nodes nv;
    nv.bind(H, v, (float)time, (float)time);
    for (int64_t i = 0; i < n; ++i) {
        const f3 o = mk(ro[i], ro[n + i], ro[2 * n + i]);
        const f3 d = mk(rd[i], rd[n + i], rd[2 * n + i]);
        Tally tl = {};
        float hst[kMaxHLevels * 9];
        const HStack hs{hst, 1};
        HHit hh;
        const float tm = (float)time;
        Hit h = H.has_mesh ? closest_hit<true, true, false>(v, o, d, tm, tl, hs, hh)
                           : closest_hit<false, true, false>(v, o, d, tm, tl, hs, hh);
        int32_t mat = -1;
        f3 nn = mk(0, 0, 0), pp = mk(0, 0, 0);
        const bool hit = h.obj != -1;
        if (hit) {
            Surface sf = H.has_mesh ? resolve_hit<true, true>(v, h, hh, o, d, tm) : resolve_hit<false, true>(v, h, hh, o, d, tm);
            mat = sf.mat; nn = sf.normal; pp = sf.position;
        }
        t_out[i] = !hit ? (double)INFINITY : h.obj == kHierHit ? hh.t64 : hit_t64(v, h.obj, h.sub, o, d, tm);
        obj_out[i] = !hit ? -1 : h.obj == kHierHit ? h.sub : v.objs[h.obj].oid;
        mat_out[i] = mat;
        n_out[i] = nn.x; n_out[n + i] = nn.y; n_out[2 * n + i] = nn.z;
        p_out[i] = pp.x; p_out[n + i] = pp.y; p_out[2 * n + i] = pp.z;
    }
    return RTX_OK;
}

extern "C" int rtx_hostemu_occluded(const rtx_scene_desc* sd, int64_t n, const float* ro, const float* rd,
                                    const double* tmax, double time, uint8_t* occ) {
    HostScene H;
    int rc = convert_scene(sd, H);
    if (rc) return rc;
    SceneView v{};
    bind_view(H, v);
    Nodes nv;
    nv.bind(H, v, (float)time, (float)time);
    for (int64_t i = 0; i < n; ++i) {
        const f3 o = mk(ro[i], ro[n + i], ro[2 * n + i]);
        const f3 d = mk(rd[i], rd[n + i], rd[2 * n + i]);
        Tally tl = {};
        float hst[kMaxHLevels * 9];
        const HStack hs{hst, 1};
        bool r = H.has_mesh ? occluded<true, true, false>(v, o, d, tmax[i], (float)time, tl, hs)
                            : occluded<false, true, false>(v, o, d, tmax[i], (float)time, tl, hs);
        occ[i] = r ? 1 : 0;
    }
    return RTX_OK;
}

// Shadow rays from points o to point light `light` (d = L - o in fp32, t_max 1, as
// regular_lighting casts them): with grids = 1 through its light grid (if it has one),
// with grids = 0 through the BVH walk. Returns -1 if grids = 1 and the light has no grid.
extern "C" int rtx_hostemu_occluded_light(const rtx_scene_desc* sd, int64_t n, const float* ro, int32_t light,
                                          int32_t grids, uint8_t* occ, int32_t* cells) {
    HostScene H;
    int rc = convert_scene(sd, H);
    if (rc) return rc;
    if (light < 0 || light >= (int32_t)H.lights.size() || H.lights[light].type != LIGHT_POINT)
        return fail(RTX_ERR_INVALID, "not a point light");
    SceneView v{};
    bind_view(H, v);
    Grids lg;
    if (grids) {
        lg.bind(H, v);
        if (!v.lgrid_on || lg.grids[light].G == 0) return -1;
    }
    Nodes nv;
    nv.bind(H, v, 0.0f, 0.0f);
    const DLight& L = H.lights[light];
    for (int64_t i = 0; i < n; ++i) {
        const f3 o = mk(ro[i], ro[n + i], ro[2 * n + i]);
        const f3 d = sub(ld3(L.vec), o);  // regular_lighting's sdir
        Tally tl = {};
        float hst[kMaxHLevels * 9];
        const HStack hs{hst, 1};
        const bool r = H.has_mesh ? occluded<true, true, false>(v, o, d, 1.0, 0.0f, tl, hs, nullptr, grids ? light : -1)
                                  : occluded<false, true, false>(v, o, d, 1.0, 0.0f, tl, hs, nullptr, grids ? light : -1);
        occ[i] = r ? 1 : 0;
        if (cells) cells[i] = grids ? lgrid_cell(v.lgrid[light], d) : -3;
    }
    return RTX_OK;
}

// The spheres and boxes directional light `light`'s shadow rays from points ro may meet,
// by its shadow grid (rtx_trace.h dir_shadow_mask; rtx_api.hip dir_shadow_grids): bits per
// point (sphere/box bits, root bits), ~0 where everything is tested. Returns -1 if the
// light has no grid. The grid is built for time 0.
extern "C" int rtx_hostemu_dir_shadow_mask(const rtx_scene_desc* sd, int64_t n, const float* ro, int32_t light,
                                           uint32_t* mask) {
    HostScene H;
    int rc = convert_scene(sd, H);
    if (rc) return rc;
    if (light < 0 || light >= (int32_t)H.lights.size()) return fail(RTX_ERR_INVALID, "bad light");
    SceneView v{};
    bind_view(H, v);
    DirGrids dg;
    dg.bind(H, v, 0.0f, 0.0f);
    if (!v.dsg_on || dg.grids[light].G == 0) return -1;
    for (int64_t i = 0; i < n; ++i) {
        const DSCell c = dir_shadow_mask(v, light, mk(ro[i], ro[n + i], ro[2 * n + i]));
        mask[2 * i] = c.obj;
        mask[2 * i + 1] = c.root;
    }
    return RTX_OK;
}

// The boxes (bits 16-31) whose own shadow test a camera ray's hit on them skips, for
// directional light `light` and this camera (DSGrid::self_boxes); -1: no grid.
extern "C" int64_t rtx_hostemu_dsgrid_self(const rtx_scene_desc* sd, const rtx_camera_desc* cd, int32_t light) {
    HostScene H;
    if (convert_scene(sd, H)) return -1;
    std::vector<float> tms(cd->n_times);
    for (int i = 0; i < cd->n_times; ++i) tms[i] = (float)cd->times[i];
    const auto tmm = std::minmax_element(tms.begin(), tms.end());
    SceneView v{};
    bind_view(H, v);
    DirGrids dg;
    dg.bind(H, v, *tmm.first, *tmm.second, camera_origin_bound(cd));
    if (!v.dsg_on || light < 0 || light >= (int32_t)dg.grids.size() || dg.grids[light].G == 0) return -1;
    return (int64_t)dg.grids[light].self_boxes;
}

// The planes' self-test limits rtx_camera_set builds for this camera (plane_self_limits):
// out[light * 4 + plane], -1 where none.
extern "C" int rtx_hostemu_plane_self(const rtx_scene_desc* sd, const rtx_camera_desc* cd, float* out) {
    HostScene H;
    if (int rc = convert_scene(sd, H)) return rc;
    const std::vector<float> lim = plane_self_limits(H, camera_origin_bound(cd));
    std::copy(lim.begin(), lim.end(), out);
    return RTX_OK;
}

// Light grid statistics (tests and tuning): per light G, list entries, the longest list
// and the non-empty cells; zeros for a light without a grid.
extern "C" int rtx_hostemu_lgrid_stats(const rtx_scene_desc* sd, int64_t* out) {
    HostScene H;
    int rc = convert_scene(sd, H);
    if (rc) return rc;
    std::vector<DLGrid> grids;
    std::vector<int32_t> start, faces;
    std::vector<float> d2;
    light_grids(H, grids, start, faces, d2);
    for (size_t li = 0; li < grids.size(); ++li) {
        const DLGrid& g = grids[li];
        int64_t* o = out + 4 * li;
        o[0] = g.G; o[1] = o[2] = o[3] = 0;
        if (!g.G) continue;
        for (int64_t c = 0; c < (int64_t)g.G * g.G; ++c) {
            const int64_t len = start[g.start_off + c + 1] - start[g.start_off + c];
            o[1] += len;
            o[2] = std::max(o[2], len);
            o[3] += len > 0;
        }
    }
    return RTX_OK;
}

// The device's Philox4x32-10 (rtx_trace.h philox4x32) on one counter and key: ctr is
// overwritten with the output block.
extern "C" void rtx_hostemu_philox(uint32_t* ctr, uint32_t k0, uint32_t k1) { philox4x32(ctr, k0, k1); }

// The production jitter uniforms (rtx_kernels.h jitter_block / jitter_rnd) of the strip
// col0 .. col0 + ncols - 1, in the replay table's layout [column][reference row][dof][aa][3].
extern "C" void rtx_hostemu_jitter(uint64_t seed, int32_t col0, int32_t ncols, int32_t height, int32_t n_dof,
                                   int32_t n_aa, float* out) {
    KParams k{};
    k.col0 = col0;
    k.seed_lo = (uint32_t)seed;
    k.seed_hi = (uint32_t)(seed >> 32);
    int64_t i = 0;
    for (int32_t cc = 0; cc < ncols; ++cc)
        for (int32_t j = 0; j < height; ++j)
            for (int32_t s = 0; s < n_dof * n_aa; ++s, ++i) {
                uint32_t w[4];
                jitter_block(k, cc, j, s >> 1, w);
                const f3 r = jitter_rnd(w, s & 1);
                out[3 * i] = r.x; out[3 * i + 1] = r.y; out[3 * i + 2] = r.z;
            }
}

extern "C" const char* rtx_hostemu_last_error(void) { return g_last_error.c_str(); }

extern "C" int64_t rtx_hostemu_sizeof(int which) {
    switch (which) {
        case 0: return sizeof(rtx_object);
        case 1: return sizeof(rtx_triangle);
        case 2: return sizeof(rtx_material);
        case 3: return sizeof(rtx_light);
        case 4: return sizeof(rtx_scene_desc);
        case 5: return sizeof(rtx_camera_desc);
        case 6: return sizeof(rtx_texture);
    }
    return -1;
}

// The scene-record prelude of the scene-specialized kernels (rtx_api.hip
// jit_baked_records) for a scene, so tests and tools/jit_isa.sh can inspect it offline.
// Returns the string's length; writes at most cap bytes (NUL-terminated) into out.
extern "C" int64_t rtx_hostemu_jit_baked(const rtx_scene_desc* sd, char* out, int64_t cap) {
    HostScene H;
    if (convert_scene(sd, H)) return -1;
    const std::string s = jit_baked_records(H.objs, H.mats, H.lights);
    if (out && cap > 0) {
        const size_t n = std::min((size_t)cap - 1, s.size());
        memcpy(out, s.data(), n);
        out[n] = '\0';
    }
    return (int64_t)s.size();
}

// `x ** hardness` as the shading code evaluates it (rtx_trace.h spec_pow, integer
// hardness), cast to fp32 as regular_lighting does, for n inputs.
extern "C" void rtx_hostemu_spec_pow(const float* x, int64_t n, int32_t hardness, float* out, int threads) {
    DMat m{};
    m.hard_is_int = 1;
    m.hard_int = hardness;
    m.hardness = hardness;
    int bits = 0;
    while (bits < 31 && (hardness >> bits)) ++bits;
#pragma omp parallel for num_threads(threads > 0 ? threads : 1) schedule(static)
    for (int64_t i = 0; i < n; ++i) out[i] = (float)spec_pow((double)x[i], m, bits);
}

// The scene-specialized kernel librtx.so would build for this scene and camera on gfx950
// (rtx_api.hip jit_spec), as text: "name\n" + one option per line + "\n" + the hiprtc
// source. Returns the text's length (-1: the generic kernel runs, -2: bad input); writes
// at most cap bytes (NUL-terminated). tools/jit_offline.py compiles it without a GPU.
extern "C" int64_t rtx_hostemu_jit_spec(const rtx_scene_desc* sd, const rtx_camera_desc* cd, int32_t cnt, int32_t out8,
                                        char* out, int64_t cap) {
    HostScene H;
    if (convert_scene(sd, H)) return -2;
    KParams k;
    if (convert_camera(cd, k)) return -2;
    bind_view(H, k.S);
    k.S.n_objs_all = (int32_t)H.objs.size();
    k.S.n_mats = (int32_t)H.mats.size();
    k.S.n_tris = (int32_t)H.tris.size();
    k.S.n_leaves = (int32_t)H.leaves.size();
    Grids lg;
    lg.bind(H, k.S);
    std::vector<float> tms(cd->n_times);
    for (int i = 0; i < cd->n_times; ++i) tms[i] = (float)cd->times[i];
    const auto tmm = std::minmax_element(tms.begin(), tms.end());
    DirGrids dg;
    dg.bind(H, k.S, *tmm.first, *tmm.second, camera_origin_bound(cd));
    std::vector<int32_t> bstart, bfaces;
    std::vector<float> bz;
    std::vector<uint32_t> bmask, brmask;
    int32_t bins_x = 0, mesh_bins = 0;
    std::vector<DBound> nodeb;
    if (!H.nodes.empty()) nodeb = compute_bounds(H.nodes, H.objs, H.tris, *tmm.first, *tmm.second);
    if (opt_on(OPT_BINS) && primary_bins(H, cd, nodeb, bstart, bfaces, bz, bmask, brmask, bins_x, mesh_bins)) {
        k.S.bins_on = 1;
        k.S.mesh_bins = mesh_bins;
    }
    const int spp = k.n_dof * k.n_aa * k.n_times;
    const bool spp_mode = use_spp_mode(spp, H.has_ext);
    JitSpec sp;
    if (!jit_spec("gfx950", k.S, k, scene_traits(H), H.has_mesh, H.has_secondary, H.has_ext, cnt != 0,
                  k.jitter != RTX_JITTER_OFF, spp_mode, out8 != 0, jit_baked_records(H.objs, H.mats, H.lights), sp))
        return -1;
    std::string s = sp.name + "\n";
    for (const auto& o : sp.opts) s += o + "\n";
    s += "\n" + sp.src;
    if (out && cap > 0) {
        const size_t n = std::min((size_t)cap - 1, s.size());
        memcpy(out, s.data(), n);
        out[n] = '\0';
    }
    return (int64_t)s.size();
}

// The specialized split pass (rtx_api.hip jit_split_spec: pass 0 trace, 1 shadow) librtx.so
// would build for this scene on gfx950, as rtx_hostemu_jit_spec's text; -1: the scene's
// trees do not qualify (jit_csg_tables). *cost: csg_cost of its trees (-1 without any).
extern "C" int64_t rtx_hostemu_jit_split(const rtx_scene_desc* sd, int32_t pass, int32_t cnt, int32_t jit, char* out,
                                         int64_t cap, int64_t* cost) {
    HostScene H;
    if (convert_scene(sd, H)) return -2;
    if (cost) *cost = H.nodes.empty() ? -1 : csg_cost(H.nodes);
    std::string tables = jit_csg_tables(H.nodes);
    if (tables.empty()) return -1;
    if (opt(OPT_JIT_CSG) >= 2.0)  // (the boxes of motion time 0)
        tables += jit_csg_baked(compute_bounds(H.nodes, H.objs, H.tris, 0.0, 0.0), H.objs, opt(OPT_JIT_CSG) >= 3.0 ? 3 : 2);
    // (without the camera's counts, jit_fixed_opts: render_split adds them per camera)
    const JitSpec sp = jit_split_spec("gfx950", tables, H.has_mesh, H.has_secondary, cnt != 0, jit != 0, pass,
                                      ((int)opt(OPT_CSG_RAYS) >> pass) & 1, std::vector<std::string>());
    std::string s = sp.name + "\n";
    for (const auto& o : sp.opts) s += o + "\n";
    s += "\n" + sp.src;
    if (out && cap > 0) {
        const size_t n = std::min((size_t)cap - 1, s.size());
        memcpy(out, s.data(), n);
        out[n] = '\0';
    }
    return (int64_t)s.size();
}

// The split hierarchy passes (rtx_split.h trace_sample / shadow_mask / shade_sample) on
// the host, chunked like rtx_api.hip render_split (split_plan with `budget` bytes and
// `ratio` deeper records per sample), over image rows [row0, row0 + nrows). Deeper records
// are appended by concurrent threads, so their order varies from run to run; the frame
// must not. Blocks whose chains found the pool full are rendered again per pixel
// (render_pixel: the one-kernel form's sums), as the device's redo launch does.
template <bool MESH, bool SEC, bool JIT>
static void split_frame(const KParams& k, const Launch& L0, int64_t npix, int spp, int64_t budget, double ratio,
                        float* fb, uint64_t* tot, int threads, int64_t* redone) {
    const int ppb = spp_pixels_per_block(spp, kBlock<true>);
    const SplitPlan pl = split_plan(npix, spp, ppb, SEC ? ratio : 0.0, budget);
    const int64_t chunk = pl.chunk, cap = pl.cap;
    std::vector<uint32_t> words((size_t)(cap * kSpArrays));
    std::vector<uint32_t> redo_list((size_t)((chunk + ppb - 1) / ppb)), redo_flag(redo_list.size(), 0u);
    unsigned int count = 0;
    uint32_t redo_n = 0;
    for (int64_t p0 = 0; p0 < npix; p0 += chunk) {
        const int64_t np = std::min(chunk, npix - p0), nq = np * spp;
        Launch L = L0;
        L.pix0 = (int32_t)p0;
        count = 0;
        redo_n = 0;
        const SplitBuf sb{words.data(), &count, &redo_n, redo_list.data(), redo_flag.data(), nq, cap};
#pragma omp parallel num_threads(threads > 0 ? threads : 1)
        {
            uint64_t loc[RTX_COUNTERS] = {};
            float hst[kMaxHLevels * 9];
            const HStack hs{hst, 1};
#pragma omp for schedule(dynamic, 64)
            for (int64_t q = 0; q < nq; ++q) {
                Tally tl = {};
                auto alloc = [&](bool hit) -> int64_t {
                    if (!hit) return -1;
                    const int64_t slot = sb.nsamp + (int64_t)__atomic_fetch_add(sb.count, 1u, __ATOMIC_RELAXED);
                    return slot < sb.cap ? slot : -2;
                };
                trace_sample<MESH, SEC, true, JIT>(k, L, sb, q, tl, hs, alloc);
                for (int c = 0; c < kMaxDepth; ++c) loc[c] += tl.cast[c];
                loc[RTX_CNT_TRI] += tl.tri;
            }
            const int64_t n = std::min(sb.cap, sb.nsamp + (int64_t)__atomic_load_n(sb.count, __ATOMIC_RELAXED));
#pragma omp for schedule(dynamic, 64)
            for (int64_t r = 0; r < n; ++r) {
                const uint32_t meta = sb.u(kSpMeta)[r];
                if (!(meta & kSpHit)) continue;
                Tally tl = {};
                const f3 pos = mk(sb.f(kSpPx)[r], sb.f(kSpPy)[r], sb.f(kSpPz)[r]);
                sb.u(kSpOcc)[r] = shadow_mask<MESH, true>(k.S, pos, k.times[(meta >> 2) & (kSpMaxTimes - 1)], tl, hs);
                loc[RTX_CNT_SHADOW] += tl.shadow;
                loc[RTX_CNT_SHADE] += tl.shade;
                loc[RTX_CNT_TRI] += tl.tri;
            }
            float fst[kShadeFrames * 3];
            uint16_t fsm[kShadeFrames];
            const ShadeStack fsc{fst, fsm, 1};
#pragma omp for schedule(dynamic, 16)
            for (int64_t p = 0; p < np; ++p) {
                f3 colour = mk(0.0f, 0.0f, 0.0f);
                for (int s = 0; s < spp; ++s) colour = add(colour, shade_sample<MESH, SEC>(k, L, sb, p * spp + s, fsc));
                const int64_t o = 3 * (p0 + p);
                fb[o] = sample_mean(k, colour.x);
                fb[o + 1] = sample_mean(k, colour.y);
                fb[o + 2] = sample_mean(k, colour.z);
            }
#pragma omp critical
            for (int c = 0; c < RTX_COUNTERS; ++c) tot[c] += loc[c];
        }
        // the redo blocks (their tallies are not counted: the device's counting renders
        // reserve every level, so they never redo)
        for (uint32_t i = 0; i < redo_n; ++i) {
            const int64_t b = redo_list[i];
            redo_flag[(size_t)b] = 0u;
            ++*redone;
            float fst[kMaxDepth * kFrameWords];
            const FrameStack fs{fst, 1};
            float hst[kMaxHLevels * 9];
            const HStack hs{hst, 1};
            for (int64_t p = p0 + b * ppb; p < std::min(p0 + (b + 1) * ppb, p0 + np); ++p) {
                Tally tl = {};
                const int32_t rr = (int32_t)(p / k.ncols), cc = (int32_t)(p - (int64_t)rr * k.ncols);
                render_pixel<MESH, SEC, true, false, JIT>(k, fb, image_row(L, rr) - rr, rr, cc, tl, fs, hs, -1);
            }
        }
    }
}

extern "C" int rtx_hostemu_render_split(const rtx_scene_desc* sd, const rtx_camera_desc* cd, int32_t row0,
                                        int32_t nrows, float* fb, uint64_t* counters, int threads,
                                        int64_t budget, double ratio, int64_t* redone) {
    HostScene H;
    int rc = convert_scene(sd, H);
    if (rc) return rc;
    KParams k;
    if ((rc = convert_camera(cd, k))) return rc;
    if (row0 < 0 || nrows < 0 || row0 + nrows > cd->height) return fail(RTX_ERR_INVALID, "bad rows");
    if (!H.has_ext) return fail(RTX_ERR_INVALID, "the split passes serve hierarchy/texture scenes");
    bind_view(H, k.S);
    Grids lg;
    lg.bind(H, k.S);
    std::vector<float> times(cd->n_times);
    for (int i = 0; i < cd->n_times; ++i) times[i] = (float)cd->times[i];
    const auto mm = std::minmax_element(times.begin(), times.end());
    Nodes nv;
    nv.bind(H, k.S, *mm.first, *mm.second);
    DirGrids dg;
    dg.bind(H, k.S, *mm.first, *mm.second, camera_origin_bound(cd));
    std::vector<int32_t> bstart, bfaces;
    std::vector<float> bz;
    std::vector<uint32_t> bmask, brmask;
    int32_t bins_x = 0, mesh_bins = 0;
    if (opt_on(OPT_BINS) && primary_bins(H, cd, nv.bounds, bstart, bfaces, bz, bmask, brmask, bins_x, mesh_bins)) {
        if (bfaces.empty()) { bfaces.push_back(0); bz.push_back(0.0f); }
        k.S.bin_start = (cptr<int32_t>)bstart.data();
        k.S.bin_faces = (cptr<int32_t>)bfaces.data();
        k.S.bin_zmin = (cptr<float>)bz.data();
        k.S.bin_objmask = (cptr<uint32_t>)bmask.data();
        k.S.bin_rootmask = (cptr<uint32_t>)brmask.data();
        k.S.mesh_bins = mesh_bins;
        k.S.bins_x = bins_x;
        k.S.bins_on = 1;
    }
    std::vector<float> noise;
    const size_t nsamp = (size_t)cd->n_dof * cd->n_aa;
    if (cd->jitter == RTX_JITTER_REPLAY) noise.assign(cd->noise, cd->noise + 3 * (size_t)cd->ncols * cd->height * nsamp);
    k.xs = (cptr<float>)cd->xs; k.ys = (cptr<float>)cd->ys; k.dof_o = (cptr<float>)cd->dof_origins;
    k.aa_o = (cptr<float>)cd->aa_origins; k.times = (cptr<float>)times.data(); k.noise = (cptr<float>)noise.data();
    Launch L{};
    L.row0 = row0;
    L.nrows = nrows;
    const int spp = k.n_dof * k.n_aa * k.n_times;
    uint64_t tot[RTX_COUNTERS] = {};
    const int64_t npix = (int64_t)nrows * k.ncols;
    const bool jit = k.jitter != RTX_JITTER_OFF;
    const int sel = (H.has_mesh ? 4 : 0) | (H.has_secondary ? 2 : 0) | (jit ? 1 : 0);
    switch (sel) {
        case 0: split_frame<false, false, false>(k, L, npix, spp, budget, ratio, fb, tot, threads, redone); break;
        case 1: split_frame<false, false, true>(k, L, npix, spp, budget, ratio, fb, tot, threads, redone); break;
        case 2: split_frame<false, true, false>(k, L, npix, spp, budget, ratio, fb, tot, threads, redone); break;
        case 3: split_frame<false, true, true>(k, L, npix, spp, budget, ratio, fb, tot, threads, redone); break;
        case 4: split_frame<true, false, false>(k, L, npix, spp, budget, ratio, fb, tot, threads, redone); break;
        case 5: split_frame<true, false, true>(k, L, npix, spp, budget, ratio, fb, tot, threads, redone); break;
        case 6: split_frame<true, true, false>(k, L, npix, spp, budget, ratio, fb, tot, threads, redone); break;
        case 7: split_frame<true, true, true>(k, L, npix, spp, budget, ratio, fb, tot, threads, redone); break;
    }
    if (counters)
        for (int q = 0; q < RTX_COUNTERS; ++q) counters[q] = tot[q];
    return RTX_OK;
}

// The primary-ray bins rtx_camera_set builds for a camera (rtx_api.hip primary_bins): per
// 8x8 tile its sphere/box mask and its number of candidate mesh faces. Returns the number
// of bins (0: the camera has none).
extern "C" int64_t rtx_hostemu_bins(const rtx_scene_desc* sd, const rtx_camera_desc* cd, uint32_t* mask,
                                    int32_t* nfaces, uint32_t* rmask, int64_t cap) {
    HostScene H;
    if (convert_scene(sd, H)) return -1;
    std::vector<int32_t> bstart, bfaces;
    std::vector<float> bz;
    std::vector<uint32_t> bmask, brmask;
    int32_t bins_x = 0, mesh_bins = 0;
    std::vector<float> tms(cd->n_times);
    for (int i = 0; i < cd->n_times; ++i) tms[i] = (float)cd->times[i];
    const auto tmm = std::minmax_element(tms.begin(), tms.end());
    std::vector<DBound> nodeb;
    if (!H.nodes.empty()) nodeb = compute_bounds(H.nodes, H.objs, H.tris, *tmm.first, *tmm.second);
    if (!primary_bins(H, cd, nodeb, bstart, bfaces, bz, bmask, brmask, bins_x, mesh_bins)) return 0;
    const int64_t n = (int64_t)bmask.size();
    for (int64_t b = 0; b < n && b < cap; ++b) {
        mask[b] = bmask[b];
        nfaces[b] = mesh_bins && b + 1 < (int64_t)bstart.size() ? bstart[b + 1] - bstart[b] : 0;
        if (rmask) rmask[b] = brmask[b];
    }
    return n;
}

// Host cost of rtx_camera_set's steps (ms, best of `reps`): [0] hierarchy bounds, [1] the
// directional lights' shadow grids, [2] their self-test marks, [3] plane self limits,
// [4] primary-ray bins. (tools: the per-camera setup budget.)
extern "C" int rtx_hostemu_camera_cost(const rtx_scene_desc* sd, const rtx_camera_desc* cd, int reps, double* ms) {
    HostScene H;
    if (int rc = convert_scene(sd, H)) return rc;
    std::vector<float> tms(cd->n_times);
    for (int i = 0; i < cd->n_times; ++i) tms[i] = (float)cd->times[i];
    const auto tmm = std::minmax_element(tms.begin(), tms.end());
    const double omax = camera_origin_bound(cd);
    for (int q = 0; q < 5; ++q) ms[q] = INFINITY;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto dt = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    for (int r = 0; r < reps; ++r) {
        auto t0 = now();
        std::vector<DBound> nodeb;
        if (!H.nodes.empty()) nodeb = compute_bounds(H.nodes, H.objs, H.tris, *tmm.first, *tmm.second);
        auto t1 = now();
        std::vector<DSGrid> grids;
        std::vector<DSCell> cells;
        dir_shadow_grids(H, nodeb, *tmm.first, *tmm.second, grids, cells);
        auto t2 = now();
        dir_self_boxes(H, grids, omax);
        auto t3 = now();
        std::vector<float> lim = plane_self_limits(H, omax);
        auto t4 = now();
        std::vector<int32_t> bstart, bfaces;
        std::vector<float> bz;
        std::vector<uint32_t> bmask, brmask;
        int32_t bins_x = 0, mesh_bins = 0;
        primary_bins(H, cd, nodeb, bstart, bfaces, bz, bmask, brmask, bins_x, mesh_bins);
        auto t5 = now();
        ms[0] = std::min(ms[0], dt(t0, t1));
        ms[1] = std::min(ms[1], dt(t1, t2));
        ms[2] = std::min(ms[2], dt(t2, t3));
        ms[3] = std::min(ms[3], dt(t3, t4));
        ms[4] = std::min(ms[4], dt(t4, t5));
    }
    return RTX_OK;
}
