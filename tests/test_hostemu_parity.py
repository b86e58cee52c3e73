"""The device source of librtx.so, compiled for the host (tests/native/rtx_hostemu.hip),
against the oracle. This checks kernel logic in the GPU-less container; the same
comparisons run on the MI355X in test_gpu_parity.py."""
import numpy as np
import pytest

import hostemu
from common import assert_parity, oracle_render, product_scene
from common import OPTS

CASES = [
    ("TwoSpheresPlane", (160, 120), {}),
    ("TwoSpheresPlane", (97, 61), {"AA": {"jitter": False, "samples": 3}}),
    ("MirrorRefraction", (180, 102), {}),
    ("TorusMesh", (128, 128), {}),
    ("TorusMesh", (64, 64), {"flat_shaded": False}),
    ("MotionBlur", (75, 64), {}),
    ("DepthOfField", (40, 30), {"AA": {"jitter": False, "samples": 2}}),
    ("NovelScene1", (128, 64), {"AA": {"jitter": False, "samples": 1}}),     # CSG hierarchies + textures
    ("NovelScene2", (64, 32), {"AA": {"jitter": False, "samples": 1}}),      # + motion blur, DOF
]


@pytest.mark.parametrize("name,res,edits", CASES)
def test_hostemu_bit_exact(name, res, edits):
    sc = product_scene(name, res, **edits)
    img, cnt = hostemu.render(sc)
    ref, tl = oracle_render(name, res, tallies=True, **edits)
    s = assert_parity(img, ref, name)
    assert s["frac_diff"] == 0.0, s
    assert list(cnt[:10]) == tl[:10]
    assert cnt[10] == tl[11] and cnt[11] == tl[12]


def test_hostemu_jitter_replay():
    edits = {"AA": {"jitter": True, "samples": 2}}
    res = (32, 24)
    noise = np.random.RandomState(7).rand(32 * 24 * 2 * 32 * 3)
    sc = product_scene("DepthOfField", res, **edits)
    sc.jitter_noise = noise
    img, _ = hostemu.render(sc)
    ref = oracle_render("DepthOfField", res, noise=noise, **edits)
    assert assert_parity(img, ref)["frac_diff"] == 0.0


@pytest.mark.parametrize("tasks", [2, 3, 7])
def test_hostemu_strips(tasks):
    res = (61, 23)
    sc = product_scene("MirrorRefraction", res)
    for k in range(tasks):
        img, _ = hostemu.render(sc, k, tasks)
        ref = oracle_render("MirrorRefraction", res, subimage=k, tasks=tasks)
        assert assert_parity(img, ref)["frac_diff"] == 0.0


def _rays(rng, n, center, spread=4.0):
    o = (center + rng.uniform(-spread, spread, (n, 3))).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    return o, d


@pytest.mark.parametrize("name", ["TwoSpheresPlane", "MirrorRefraction", "TorusMesh", "DepthOfField", "MotionBlur"])
def test_hostemu_geometry_kat(name):
    """Closest hit / shadow any-hit of random rays vs the oracle (Geometry ABI KATs)."""
    from oracle import oracle as O
    rng = np.random.RandomState(3)
    o, d = _rays(rng, 4000, np.array([0, 1, 0]))
    sc = product_scene(name, (8, 8))
    dd, base = O.load_bundle(name)
    osc = O.OracleScene(dd, base)
    for time in (0.0, 0.75):
        got = hostemu.intersect(sc, o, d, time)
        t, ob, _, m, nn, pp = osc.closest(time, o, d)
        assert np.array_equal(got["obj"], ob)
        hit = ob >= 0
        assert np.array_equal(got["t"][hit], t[hit])
        assert np.array_equal(got["mat"], m)
        assert np.array_equal(got["normal"][hit], nn[hit])
        assert np.array_equal(got["position"][hit], pp[hit])
        for tmax in (1.0, np.inf):
            assert np.array_equal(hostemu.occluded(sc, o, d, tmax, time), osc.shadow(time, o, d, tmax).astype(bool))


@pytest.mark.parametrize("seed", range(3))
def test_hostemu_mesh_bv_stress(seed):
    """Rays inside / on / grazing the torus's bounding box (its fp32 decision and fp64
    fallback) vs the oracle, exactly."""
    import os
    from oracle import oracle as O
    from scenegen import bv_stress_rays, obj_bounds
    lo, hi = obj_bounds(os.path.join(os.path.dirname(__file__), "..", "assets", "torus_mesh.obj"))
    o, d = bv_stress_rays(lo, hi, 4000, seed)
    sc = product_scene("TorusMesh", (8, 8))
    dd, base = O.load_bundle("TorusMesh")
    osc = O.OracleScene(dd, base)
    got = hostemu.intersect(sc, o, d, 0.0)
    t, ob, _, m, nn, pp = osc.closest(0.0, o, d)
    assert np.array_equal(got["obj"], ob)
    hit = ob >= 0
    assert np.array_equal(got["t"][hit], t[hit])
    for tmax in (1.0, np.inf):
        assert np.array_equal(hostemu.occluded(sc, o, d, tmax, 0.0), osc.shadow(0.0, o, d, tmax).astype(bool))


@pytest.mark.parametrize("seed", range(2))
def test_hostemu_box_stress(seed):
    """Rays inside / on / grazing / aimed at the edges and corners of DepthOfField's boxes
    (the fp32 slab decision and its fp64 fallback) vs the oracle, exactly."""
    from oracle import oracle as O
    from scenegen import scene_box_stress_rays
    dd, base = O.load_bundle("DepthOfField")
    o, d = scene_box_stress_rays(dd, 3000, seed)
    sc = product_scene("DepthOfField", (8, 8))
    osc = O.OracleScene(dd, base)
    got = hostemu.intersect(sc, o, d, 0.0)
    t, ob, _, m, nn, pp = osc.closest(0.0, o, d)
    assert np.array_equal(got["obj"], ob)
    hit = ob >= 0
    assert np.array_equal(got["t"][hit], t[hit])
    assert np.array_equal(got["normal"][hit], nn[hit])
    for tmax in (1.0, np.inf):
        assert np.array_equal(hostemu.occluded(sc, o, d, tmax, 0.0), osc.shadow(0.0, o, d, tmax).astype(bool))


@pytest.mark.parametrize("seed", range(12))
def test_hostemu_random_scenes(seed):
    from common import oracle_render_dict, product_scene_dict
    from scenegen import random_scene
    d = random_scene(seed, mesh=(seed % 3 == 0))
    img, cnt = hostemu.render(product_scene_dict(d))
    ref, tl = oracle_render_dict(d, tallies=True)
    s = assert_parity(img, ref, "seed %d" % seed)
    assert s["frac_diff"] == 0.0, s
    assert list(cnt[:10]) == tl[:10] and cnt[10] == tl[11]


def test_hostemu_ties_follow_scene_order():
    from common import oracle_render_dict, product_scene_dict
    from scenegen import tie_scene
    d = tie_scene()
    img, _ = hostemu.render(product_scene_dict(d))
    ref = oracle_render_dict(d)
    assert assert_parity(img, ref)["frac_diff"] == 0.0
    # the red/blue coincident spheres: s1 (blue) is first in scene order
    assert (ref[..., 2] > ref[..., 0]).any()


@pytest.mark.parametrize("seed", range(16))
def test_hostemu_random_hierarchy_scenes(seed):
    """Random CSG trees (every node type, nesting, transforms, fallback materials, speeds,
    `ref` copies, textured planes/boxes) vs the oracle: bit-exact image and ray tallies."""
    from common import oracle_render_dict, product_scene_dict
    from scenegen import random_hier_scene
    d = random_hier_scene(seed, mesh=(seed % 4 == 0))
    img, cnt = hostemu.render(product_scene_dict(d))
    ref, tl = oracle_render_dict(d, tallies=True)
    s = assert_parity(img, ref, "seed %d" % seed)
    assert s["frac_diff"] == 0.0, s
    assert list(cnt[:10]) == tl[:10] and cnt[10] == tl[11]


@pytest.mark.parametrize("seed", [None, 3, 8])
def test_hostemu_hierarchy_geometry_kat(seed):
    """Batched closest hit / shadow rays through hierarchies vs the oracle."""
    from oracle import oracle as O
    from common import product_scene_dict
    from scenegen import random_hier_scene
    import os
    rng = np.random.RandomState(5)
    if seed is None:
        dd, base = O.load_bundle("NovelScene1")
        o, d = _rays(rng, 3000, np.array([0, 1, 0]), spread=3.0)
        sc = product_scene("NovelScene1", (8, 8))
    else:
        dd = random_hier_scene(seed)
        base = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets")
        o, d = _rays(rng, 3000, np.array([0, 0.5, 0]), spread=2.5)
        sc = product_scene_dict(dd)
    osc = O.OracleScene(dd, base)
    for time in (0.0, 0.5):
        got = hostemu.intersect(sc, o, d, time)
        t, ob, _, m, nn, pp = osc.closest(time, o, d)
        assert np.array_equal(got["obj"], ob)
        hit = ob >= 0
        assert hit.mean() > 0.1
        assert np.array_equal(got["t"][hit], t[hit])
        assert np.array_equal(got["mat"], m)
        assert np.array_equal(got["normal"][hit], nn[hit])
        assert np.array_equal(got["position"][hit], pp[hit])
        for tmax in (1.0, np.inf):
            assert np.array_equal(hostemu.occluded(sc, o, d, tmax, time), osc.shadow(time, o, d, tmax).astype(bool))


@pytest.fixture(scope="module")
def blob5(tmp_path_factory):
    from scenegen import blob_obj
    p = str(tmp_path_factory.mktemp("mesh") / "blob5.obj")
    blob_obj(p, level=5)  # 20,480 faces
    return p


@pytest.mark.parametrize("flat", [False, True])
def test_hostemu_large_mesh_bvh(blob5, flat):
    """Mesh BVH on a 20k-face mesh: bit-exact image and ray tallies."""
    from common import oracle_render_dict, product_scene_dict
    from scenegen import blob_scene
    d = blob_scene(blob5, (40, 40), flat)
    img, cnt = hostemu.render(product_scene_dict(d))
    ref, tl = oracle_render_dict(d, tallies=True)
    assert assert_parity(img, ref)["frac_diff"] == 0.0
    assert list(cnt[:10]) == tl[:10] and cnt[10] == tl[11]


def test_hostemu_large_mesh_kat(blob5):
    from oracle import oracle as O
    from common import product_scene_dict
    from scenegen import blob_scene
    import os
    d = blob_scene(blob5)
    rng = np.random.RandomState(9)
    o, dd = _rays(rng, 1500, np.array([0, 0, 0]), spread=2.0)
    sc = product_scene_dict(d)
    osc = O.OracleScene(d, os.path.dirname(blob5))
    got = hostemu.intersect(sc, o, dd, 0.0)
    t, ob, _, m, nn, pp = osc.closest(0.0, o, dd)
    hit = ob >= 0
    assert np.array_equal(got["obj"], ob) and np.array_equal(got["t"][hit], t[hit])
    assert np.array_equal(got["normal"][hit], nn[hit]) and np.array_equal(got["position"][hit], pp[hit])
    for tmax in (1.0, np.inf):
        assert np.array_equal(hostemu.occluded(sc, o, dd, tmax, 0.0), osc.shadow(0.0, o, dd, tmax).astype(bool))


@pytest.mark.parametrize("seed", range(24))
def test_hostemu_primary_bins_equal_walk(seed, monkeypatch):
    """The primary-ray bins (objects and faces a tile's primary rays may hit) change no
    pixel: binned == full walk == oracle, for whole frames and column strips."""
    from common import oracle_render_dict, product_scene_dict
    from scenegen import bins_scene
    d = bins_scene(seed)
    sc = product_scene_dict(d)
    img, _ = hostemu.render(sc)
    monkeypatch.setattr(OPTS, "bins", "0")
    walk, _ = hostemu.render(sc)
    assert np.array_equal(img, walk)
    monkeypatch.setattr(OPTS, "bins", "1")
    assert_parity(img, oracle_render_dict(d), "bins seed %d" % seed)
    for k in range(3):
        strip, _ = hostemu.render(sc, k, 3)
        assert np.array_equal(strip, oracle_render_dict(d, k, 3)), k


def _mesh_probe_points(tris, light, rng, n):
    """Points that stress a light grid: on faces (interior, edges, vertices), just above
    and below them, around the mesh, near and beyond the light, and far away."""
    v = tris[:, :3].astype(np.float64)
    f = rng.randint(len(v), size=n)
    b = rng.dirichlet([1, 1, 1], size=n)
    b[: n // 4, rng.randint(3)] = 0.0  # on an edge
    b[: n // 4] /= b[: n // 4].sum(1, keepdims=True)
    b[n // 4: n // 3] = np.eye(3)[rng.randint(3, size=n // 3 - n // 4)]  # on a vertex
    on = np.einsum("nk,nkd->nd", b, v[f])
    nrm = np.cross(v[f, 1] - v[f, 0], v[f, 2] - v[f, 0])
    nrm /= np.maximum(np.linalg.norm(nrm, axis=1, keepdims=True), 1e-30)
    off = on + nrm * rng.choice([-1e-3, -1e-5, 1e-5, 1e-3, 0.05], size=(n, 1))
    lo, hi = v.reshape(-1, 3).min(0), v.reshape(-1, 3).max(0)
    ctr, ext = (lo + hi) / 2, (hi - lo).max()
    around = ctr + rng.uniform(-2, 2, (n, 3)) * ext
    L = np.asarray(light, np.float64)
    near_l = L + rng.normal(size=(n, 3)) * rng.choice([1e-3, 0.1, 1.0], size=(n, 1))
    beyond = L + (L - ctr) * rng.uniform(0.05, 3.0, (n, 1)) + rng.normal(size=(n, 3)) * 0.3
    far = ctr + rng.normal(size=(n, 3)) * rng.choice([10.0, 100.0, 1e4], size=(n, 1))
    plane = np.c_[rng.uniform(-30, 30, n), np.full(n, -1.0), rng.uniform(-30, 30, n)]
    return np.concatenate([on, off, around, near_l, beyond, far, plane]).astype(np.float32)


def _grid_scenes(blob_path):
    from scenegen import blob_scene
    from common import product_scene_dict
    from rtx.io import bundled_scene_dict
    out = [("TorusMesh", bundled_scene_dict("TorusMesh", resolution=(32, 32)))]
    d = blob_scene(blob_path, (32, 32))
    out.append(("blob", d))
    rng = np.random.RandomState(5)
    for k in range(4):  # the torus moved and scaled, lights close, far, above, below, inside
        e = bundled_scene_dict("TorusMesh", resolution=(32, 32))
        for g in e["objects"]:
            if g["type"] == "mesh":
                g["scale"] = float(rng.uniform(0.3, 3.0))
                g["position"] = np.round(rng.uniform(-2, 2, 3), 3).tolist()
        e["lights"] = [{"name": "l%d" % i, "type": "point", "colour": [1, 1, 1], "power": 1.0,
                        "position": np.round(rng.uniform(-1, 1, 3) * s, 3).tolist()}
                       for i, s in enumerate((1.0, 4.0, 12.0, 60.0))]
        out.append(("torus%d" % k, e))
    return [(n, product_scene_dict(d)) for n, d in out]


def test_hostemu_light_grids_equal_walk(blob5):
    """The light grids (shadow rays of point lights test only the mesh faces listed in the
    cell of their direction from the light) change no shadow decision: grid == BVH walk
    for points on, just off and around the faces, near and beyond the light, far away and
    on the ground plane, for TorusMesh, the 20k-face blob and moved/scaled tori with
    lights near, far and inside the mesh's bounding sphere (those get no grid)."""
    from rtx import _native as N
    from rtx import records as R
    used = 0
    for name, sc in _grid_scenes(blob5):
        mesh = [g for g in sc.objects if R.kind(g) == N.RTX_MESH][0]
        tris = R.mesh_triangles(mesh)
        for li, lt in enumerate(sc.lights):
            rng = np.random.RandomState(li + 17)
            pts = _mesh_probe_points(tris, R.vec(lt.vector), rng, 3000)
            g = hostemu.occluded_light(sc, pts, li, True)
            if g is None:
                continue
            w, _ = hostemu.occluded_light(sc, pts, li, False)
            occ, cells = g
            assert np.array_equal(occ, w), (name, li, int((occ != w).sum()))
            used += 1
            assert (cells >= 0).sum() > 100 and occ.sum() > 50, (name, li)
    assert used >= 10, used


@pytest.mark.parametrize("flat", [False, True])
def test_hostemu_light_grids_frames(blob5, flat, monkeypatch):
    """Whole frames with and without the light grids: identical, and equal to the oracle."""
    from common import oracle_render_dict, product_scene_dict
    from scenegen import blob_scene
    from rtx.io import bundled_scene_dict
    for d in (bundled_scene_dict("TorusMesh", resolution=(48, 48)), blob_scene(blob5, (40, 40), flat)):
        sc = product_scene_dict(d)
        img, _ = hostemu.render(sc)
        monkeypatch.setattr(OPTS, "lgrid", "0")
        walk, _ = hostemu.render(sc)
        monkeypatch.setattr(OPTS, "lgrid", "1")
        assert np.array_equal(img, walk)
        assert_parity(img, oracle_render_dict(d), "light grids")


def _sphere_shadow_stress_rays(centers, radii, n, rng):
    """Shadow rays whose quadratic roots sit on the decision boundaries of
    Sphere.shadow_intersect (simple_geometry.py:48-72): origins on and near the surface
    (a root at ~0), roots at 1e-3 and at t_max = 1 (+-1e-7 relative), tangent and
    near-tangent lines, long and short directions."""
    os_, ds_ = [], []
    for c, r in zip(centers, radii):
        c = np.asarray(c, np.float64)
        for k in range(n):
            u = rng.normal(size=3); u /= np.linalg.norm(u)
            v = rng.normal(size=3); v -= v.dot(u) * u; v /= np.linalg.norm(v)
            kind = k % 5
            scale = 10.0 ** rng.uniform(-1, 1)
            if kind == 0:    # origin on / near the surface
                o = c + u * r * (1 + rng.choice([0, 1e-7, -1e-7, 1e-4, -1e-4]))
                d = rng.normal(size=3) * scale
            elif kind == 1:  # a root at t = 1e-3 (entry) or exit
                d = -u * scale
                t0 = 1e-3 * (1 + rng.choice([0, 1e-7, -1e-7, 1e-6, -1e-6]))
                o = c + u * r - d * t0 if rng.rand() < 0.5 else c - u * r - d * t0
            elif kind == 2:  # a root at t = t_max = 1
                d = -u * scale
                t0 = 1.0 + rng.choice([0, 1e-7, -1e-7, 1e-6, -1e-6])
                o = c + u * r - d * t0 if rng.rand() < 0.5 else c - u * r - d * t0
            elif kind == 3:  # tangent and near-tangent lines
                p = c + u * r * (1 + rng.choice([0, 1e-7, -1e-7, 1e-5, -1e-5]))
                d = v * scale
                o = p - d * rng.uniform(-0.5, 1.5)
            else:            # from far away through the sphere
                o = c + u * r * rng.uniform(2, 50)
                d = (c + v * r * rng.uniform(0, 1.2) - o) * rng.uniform(0.2, 2.0)
            os_.append(o); ds_.append(d)
    return np.asarray(os_, np.float32), np.asarray(ds_, np.float32)


@pytest.mark.parametrize("name", ["TwoSpheresPlane", "MirrorRefraction"])
def test_hostemu_sphere_shadow_stress(name):
    """Sphere shadow decisions vs the oracle at the 1e-3 and t_max boundaries: the fp64
    roots, and with a build of -DRTX_SHADOW_F32=1 the fp32 decision with error bounds
    (sphere_shadow_f32; a build with zero margins fails this test)."""
    from oracle import oracle as O
    from rtx import _native as N
    from rtx import records as R
    sc = product_scene(name, (8, 8))
    sph = [g for g in sc.objects if R.kind(g) == N.RTX_SPHERE]
    rng = np.random.RandomState(11)
    o, d = _sphere_shadow_stress_rays([R.vec(g.center) for g in sph], [float(g.radius) for g in sph], 1500, rng)
    dd, base = O.load_bundle(name)
    osc = O.OracleScene(dd, base)
    for tmax in (1.0, np.inf, 0.7, 1e-3 * (1 + 1e-6)):
        assert np.array_equal(hostemu.occluded(sc, o, d, tmax, 0.0), osc.shadow(0.0, o, d, tmax).astype(bool)), tmax


def test_hostemu_plane_shadow_stress():
    """Plane shadow decisions vs the oracle where the plane's t sits on the 1e-4 and
    t_max boundaries (+-1e-7 relative) -- the approximate-reciprocal filter must defer to
    the exact quotient there (rtx_trace.h occluded, RTX_PLANE_SHADOW_RCP)."""
    from oracle import oracle as O
    from rtx import _native as N
    from rtx import records as R
    sc = product_scene("TwoSpheresPlane", (8, 8))
    pl = [g for g in sc.objects if R.kind(g) == N.RTX_PLANE][0]
    p0, n = R.vec(pl.point).astype(np.float64), R.vec(pl.normal).astype(np.float64)
    rng = np.random.RandomState(5)
    os_, ds_ = [], []
    for k in range(6000):
        d = rng.normal(size=3) * 10.0 ** rng.uniform(-1, 1)
        if abs(d.dot(n)) < 1e-3:
            continue
        q = p0 + rng.uniform(-20, 20, 3); q -= (q - p0).dot(n) * n / n.dot(n)
        t0 = {0: 1e-4, 1: 1.0, 2: 0.7}[k % 3] * (1 + rng.choice([0, 1e-7, -1e-7, 1e-6, -1e-6, 1e-3]))
        os_.append(q - d * t0); ds_.append(d)
    o, d = np.asarray(os_, np.float32), np.asarray(ds_, np.float32)
    dd, base = O.load_bundle("TwoSpheresPlane")
    osc = O.OracleScene(dd, base)
    for tmax in (1.0, np.inf, 0.7):
        assert np.array_equal(hostemu.occluded(sc, o, d, tmax, 0.0), osc.shadow(0.0, o, d, tmax).astype(bool)), tmax


@pytest.mark.parametrize("seed", range(4))
def test_hostemu_primary_bins_wide_frame(seed, monkeypatch):
    """Bins at 7680 pixels across: a tile's objects come from projecting through the camera's
    own fp32 pixel tables (rtx_api.hip primary_bins), not from a spacing estimate whose
    error grows with the column index -- binned == walk == oracle on the first and last of
    eight column strips, with tiny spheres strung along the frame's width."""
    from common import oracle_render_dict, product_scene_dict
    from scenegen import bins_scene
    d = bins_scene(seed, res=(7680, 16))
    cam = np.array(d["camera"]["position"])
    look = np.array(d["camera"]["lookAt"])
    fwd = (look - cam) / np.linalg.norm(look - cam)
    side = np.cross(fwd, [0.0, 1.0, 0.0])
    side /= np.linalg.norm(side)
    for k, s in enumerate(np.linspace(-1.0, 1.0, 9)):
        c = cam + fwd * 20.0 + side * s * 20.0 * np.tan(np.radians(d["camera"]["fov"] / 2)) * 1.2
        d["objects"].append({"name": "tiny%d" % k, "type": "sphere", "radius": 0.02,
                             "position": np.round(c, 4).tolist(), "materials": [k % 4]})
    sc = product_scene_dict(d)
    for k in (0, 7):
        img, _ = hostemu.render(sc, k, 8)
        monkeypatch.setattr(OPTS, "bins", "0")
        walk, _ = hostemu.render(product_scene_dict(d), k, 8)
        monkeypatch.setattr(OPTS, "bins", "1")
        assert np.array_equal(img, walk), k
        assert_parity(img, oracle_render_dict(d, k, 8), "wide bins seed %d strip %d" % (seed, k))


def _lens_noise(sc, subimage=0, tasks=1):
    """The oracle's jitter stream for a product scene: Philox (oracle/philox.py) or none."""
    if not sc.jitter:
        return None
    from oracle import philox as PH
    from rtx.scene import strip_columns
    col0, ncols = strip_columns(sc.vc.width, subimage, tasks)
    return PH.jitter_noise(sc.seed, col0, ncols, sc.vc.height, sc.vc.dof_samples, sc.samples)


@pytest.mark.parametrize("seed", range(24))
def test_hostemu_lens_bins_equal_walk(seed, monkeypatch):
    """Lens cameras' thick primary-ray bins (rtx_api.hip primary_bins: DOF origins, AA
    spreads and jitter bounded around the pinhole) change no pixel: binned == walk, and
    == the oracle (with the restated Philox stream) on every fourth scene."""
    from common import oracle_render_dict, product_scene_dict
    from scenegen import bins_scene
    d = bins_scene(seed, res=(33, 19), lens=True)
    sc = product_scene_dict(d)
    img, _ = hostemu.render(sc)
    monkeypatch.setattr(OPTS, "bins", "0")
    walk, _ = hostemu.render(sc)
    monkeypatch.setattr(OPTS, "bins", "1")
    assert np.array_equal(img, walk)
    if seed % 4 == 0:
        assert_parity(img, oracle_render_dict(d, noise=_lens_noise(sc)), "lens bins seed %d" % seed)


def _lens_ray_scene(seed, pinhole=False):
    """bins_scene(lens=True) without a mesh (lens cameras keep no face bins), motion, or
    a sphere around the lens (it would take every ray); pinhole=True: the same camera
    with no aperture, AA spread or jitter."""
    from scenegen import bins_scene
    d = bins_scene(seed, res=(160, 96), lens=True)
    cam = np.array(d["camera"]["position"])
    d["objects"] = [o for o in d["objects"] if o["type"] != "mesh" and not (
        o["type"] == "sphere" and np.linalg.norm(np.array(o["position"]) - cam) < o["radius"] + d["DOF"]["aperture"])]
    d.pop("motion", None)
    for o in d["objects"]:
        o.pop("speed", None)
    if pinhole:
        d["DOF"] = {"aperture": 0.0, "focal_length": d["DOF"]["focal_length"], "samples": 1}
        d["AA"] = {"jitter": False, "samples": 1}
    return d


def _lens_ray_misses(d, mask, rmask=None):
    """Primary sample rays of scene d's lens camera (the DOF origin's focal direction from
    the jittered AA origin, scene.py:54-65, set up in fp32 like the device) whose closest
    hit is a sphere or box (rmask given: or a hierarchy root) missing from their tile's
    mask: (misses, rays that hit one)."""
    from common import product_scene_dict
    sc = product_scene_dict(d)
    cd, t = sc.camera_desc()
    W, H, nd, na = cd.ncols, cd.height, sc.vc.dof_samples, sc.samples
    f32 = np.float32
    u, v, w = (np.asarray(x, f32) for x in (sc.vc.u, sc.vc.v, sc.vc.w))
    pos = np.asarray(sc.vc.position, f32)
    xs, ys = np.asarray(t["xs"], f32), np.asarray(t["ys"], f32)
    cc, jj = np.meshgrid(np.arange(W), np.arange(H), indexing="ij")  # [W][H], the jitter table's order
    base = xs[cc][..., None] * u + ys[jj][..., None] * v - w * f32(sc.vc.d)
    bdir = base / np.linalg.norm(base, axis=-1, keepdims=True).astype(f32)
    focal = pos + bdir * f32(sc.vc.focal_length)
    dof = np.asarray(t["dof"], f32).reshape(nd, 3)
    aa = np.asarray(t["aa"], f32).reshape(nd, na, 3)
    if sc.jitter:
        rnd = hostemu.jitter(sc.seed, 0, W, H, nd, na).reshape(W, H, nd, na, 3)
        jit = rnd / np.linalg.norm(rnd, axis=-1, keepdims=True).astype(f32) * f32(t["jscale"])
    else:
        jit = np.zeros((W, H, nd, na, 3), f32)
    dd = focal[:, :, None, :] - dof[None, None]                     # [W][H][nd][3]
    dd = dd / np.linalg.norm(dd, axis=-1, keepdims=True).astype(f32)
    o = (aa[None, None] + jit).reshape(-1, 3)
    dr = np.broadcast_to(dd[:, :, :, None, :], (W, H, nd, na, 3)).reshape(-1, 3)
    hit = hostemu.intersect(sc, o, dr)["obj"]
    kinds = [g["type"] for g in d["objects"]]
    pc = np.broadcast_to(cc[:, :, None, None], (W, H, nd, na)).ravel()
    prow = (H - 1 - np.broadcast_to(jj[:, :, None, None], (W, H, nd, na))).ravel()
    misses = tested = 0
    for i, k in enumerate(kinds):
        if k in ("sphere", "box"):
            m, bt = mask, (0 if k == "sphere" else 16) + sum(1 for q in kinds[:i] if q == k)
        elif k == "node" and rmask is not None:
            m, bt = rmask, sum(1 for q in kinds[:i] if q == "node")
        else:
            continue
        sel = hit == i
        tested += int(sel.sum())
        misses += int((((m[prow[sel] >> 3, pc[sel] >> 3] >> np.uint32(bt)) & 1) == 0).sum())
    return misses, tested


@pytest.mark.parametrize("seed", range(16))
def test_lens_bins_hold_every_sample_ray(seed):
    """The thick bins' bound, ray by ray: every primary sample ray of a lens camera whose
    closest hit is a sphere or box finds that object in its tile's mask. 160 x 96 pixels,
    every DOF x AA sample (up to 24 per pixel)."""
    from common import product_scene_dict
    d = _lens_ray_scene(seed)
    b = hostemu.bins(product_scene_dict(d))
    if b is None:  # an aperture too wide for the focal length: no bins (seed 0)
        assert d["DOF"]["aperture"] > 0.05 * d["DOF"]["focal_length"], d["DOF"]
        return
    misses, tested = _lens_ray_misses(d, b[0])
    assert misses == 0, (misses, tested)


@pytest.mark.parametrize("seed", range(8))
def test_root_bins_hold_every_sample_ray(seed):
    """Primary-ray bins of hierarchy roots (their hit boxes) and of moving objects (swept
    over the frame's times), ray by ray: every primary sample ray of a random CSG scene --
    pinhole or lens camera, AA jitter -- whose closest hit is a root, sphere or box finds
    it in its tile's masks."""
    from common import product_scene_dict
    from scenegen import random_hier_scene
    d = random_hier_scene(seed, res=(64, 48))
    d.pop("motion", None)  # rays at time 0
    d["objects"] = [o for o in d["objects"] if "ref" not in o]  # (objects map to scene positions)
    if seed % 2:
        d["DOF"] = {"aperture": 0.15, "focal_length": 5.0, "samples": 3}
        d["AA"] = {"jitter": True, "samples": 2}
    b = hostemu.bins(product_scene_dict(d), roots=True)
    assert b is not None
    misses, tested = _lens_ray_misses(d, b[0], b[2])
    assert misses == 0, (misses, tested)


@pytest.mark.parametrize("seed", range(2))
def test_hostemu_many_roots_bins_and_grids(seed, monkeypatch):
    """40 hierarchy roots and 20 flat spheres -- beyond the 32 root bits and 16 sphere bits
    of the bins and shadow-grid cells: bins and grids on == both off == the oracle (with
    the restated Philox stream), one-kernel and split forms."""
    from common import oracle_render_dict, product_scene_dict
    from scenegen import many_roots_scene
    d = many_roots_scene(seed)
    sc = product_scene_dict(d)
    assert hostemu.bins(sc, roots=True) is not None
    img, _ = hostemu.render(sc)
    split, _ = hostemu.render_split(sc)
    monkeypatch.setattr(OPTS, "bins", "0")
    monkeypatch.setattr(OPTS, "dsgrid", "0")
    walk, _ = hostemu.render(product_scene_dict(d))
    assert np.array_equal(img, walk) and np.array_equal(split, walk)
    assert_parity(img, oracle_render_dict(d, noise=_lens_noise(sc)), "many roots seed %d" % seed)


def test_lens_ray_check_is_sensitive():
    """The ray check above fails the pinhole bins (no lens growth) of the same scenes:
    lens rays do leave the pinhole footprint, so the growth is what holds them."""
    from common import product_scene_dict
    bad = 0
    for seed in range(16):
        pin = hostemu.bins(product_scene_dict(_lens_ray_scene(seed, pinhole=True)))
        bad += _lens_ray_misses(_lens_ray_scene(seed), pin[0])[0] > 0
    assert bad >= 2, bad


def _shadow_probe_points(d, rng, n_obj=400):
    """Points that stress a directional shadow grid: on and just off each sphere's and box's
    surface, upstream of them along every light (shadow rays grazing the silhouettes), on
    the floor, scattered, and far away (beyond the grid's pmax)."""
    pts = []
    dirs = [np.asarray(l["direction"], np.float64) for l in d["lights"] if l["type"] == "directional"]
    for o in d["objects"]:
        if o["type"] == "sphere":
            c, rad = np.asarray(o["position"], np.float64), o["radius"]
            n = rng.normal(size=(n_obj, 3))
            n /= np.linalg.norm(n, axis=1, keepdims=True)
            surf = c + n * rad * (1.0 + rng.choice([-1e-3, 0.0, 1e-6, 1e-3, 0.05], (n_obj, 1)))
        elif o["type"] == "box":
            if "min" in o:
                mn, mx = np.minimum(o["min"], o["max"]), np.maximum(o["min"], o["max"])
            else:
                c, sz = np.asarray(o["position"]), np.asarray(o["size"])
                mn, mx = c - sz / 2, c + sz / 2
            surf = rng.uniform(mn, mx, (n_obj, 3))
            ax = rng.randint(3, size=n_obj)
            side = rng.rand(n_obj) < 0.5
            surf[np.arange(n_obj), ax] = np.where(side, mn[ax], mx[ax]) + rng.choice([-1e-3, 0.0, 1e-3], n_obj)
        else:
            continue
        pts.append(surf)
        for dv in dirs:  # upstream of the surface: the ray from there grazes or crosses it
            u = -dv / np.linalg.norm(dv)
            pts.append(surf - u * rng.uniform(0.001, 12.0, (n_obj, 1)))
    pts.append(np.c_[rng.uniform(-10, 10, (2000, 1)), np.full((2000, 1), -1.0), rng.uniform(-10, 10, (2000, 1))])
    pts.append(rng.uniform(-12, 12, (3000, 3)))
    pts.append(rng.uniform(-300, 300, (500, 3)))
    return np.concatenate(pts).astype(np.float32)


def _check_dir_shadow_grid(d, p, what):
    """Wherever one sphere, box or hierarchy root of scene d alone occludes a directional
    light's shadow ray from a point of p (the device's own test, at time 0), the light's
    grid lists it for that point. Returns the number of occluded (ray, object) pairs."""
    import copy
    from common import product_scene_dict
    sc = product_scene_dict(d)
    sd = sc.scene_desc()
    kinds = [o["type"] for o in d["objects"]]
    checked = 0
    for li, l in enumerate(d["lights"]):
        if l["type"] != "directional":
            continue
        mask = hostemu.dir_shadow_mask(sc, p, li)
        assert mask is not None
        dvec = -np.asarray(sd.lights[li].vector[:3], np.float32)  # the light's negvec, as the device casts it
        for i, o in enumerate(d["objects"]):
            if o["type"] in ("sphere", "box"):
                word, bt = 0, (0 if o["type"] == "sphere" else 16) + sum(1 for q in kinds[:i] if q == o["type"])
            elif o["type"] == "node":
                word, bt = 1, sum(1 for q in kinds[:i] if q == "node")
            else:
                continue
            has = ((mask[:, word] >> np.uint32(bt)) & 1).astype(bool)
            one = copy.deepcopy(d)
            one["objects"] = [copy.deepcopy(o)]
            one.pop("motion", None)
            occ = hostemu.occluded(product_scene_dict(one), p, np.broadcast_to(dvec, p.shape), np.inf, 0.0)
            assert not (occ & ~has).any(), (what, li, i, int((occ & ~has).sum()), int(occ.sum()))
            checked += int(occ.sum())
    return checked


@pytest.mark.parametrize("seed", range(16))
def test_hostemu_dir_shadow_grids_hold_every_ray(seed, monkeypatch):
    """Directional shadow grids, ray by ray, on spheres and boxes (static and moving; a
    grid for every scene, however few its spheres)."""
    monkeypatch.setattr(OPTS, "dsgrid_min", "1")
    from scenegen import shadow_scene
    d = shadow_scene(seed)
    p = _shadow_probe_points(d, np.random.RandomState(seed))
    assert _check_dir_shadow_grid(d, p, "seed %d" % seed) > 0


@pytest.mark.parametrize("seed", range(12))
def test_hostemu_dir_shadow_grids_hold_every_ray_hierarchies(seed, monkeypatch):
    """Directional shadow grids, ray by ray, on hierarchy roots (their shadow boxes):
    random CSG trees under diagonal, vertical and random directional lights."""
    from scenegen import random_hier_scene
    monkeypatch.setattr(OPTS, "dsgrid_min", "1")
    d = random_hier_scene(seed)
    d["objects"] = [o for o in d["objects"] if "ref" not in o]  # (a copy needs its source in the scene)
    d["lights"] = [{"name": "d%d" % k, "type": "directional", "direction": v, "colour": [1.0, 1.0, 1.0], "power": 0.5}
                   for k, v in enumerate([[1.0, -1.0, -1.0], [0.0, -1.0, 0.0], [-0.3, 0.2, 0.9]])]
    rng = np.random.RandomState(seed)
    near = rng.uniform(-3.5, 3.5, (6000, 3))
    p = [near, rng.uniform(-12, 12, (2000, 3))]
    for l in d["lights"]:
        u = -np.asarray(l["direction"]) / np.linalg.norm(l["direction"])
        p.append(near - u * rng.uniform(0.001, 8.0, (len(near), 1)))
    assert _check_dir_shadow_grid(d, np.concatenate(p).astype(np.float32), "hier seed %d" % seed) > 0


@pytest.mark.parametrize("seed", list(range(8)) + ["dof"])
def test_hostemu_box_self_shadow_never_passes(seed):
    """The skipped self tests (DSGrid.self_boxes): rays from the camera's sample origins
    aimed at random points of each marked box -- faces, edges, corners, grazing -- hit it
    at fp32 points from which that box alone never occludes the light's shadow ray (the
    device's own test); the marks hold."""
    import copy
    from common import product_scene_dict
    from rtx.io import bundled_scene_dict
    from scenegen import shadow_scene
    if seed == "dof":
        d = bundled_scene_dict("DepthOfField", resolution=(64, 48))
        d["AA"] = {"jitter": True, "samples": 2}
    else:
        d = shadow_scene(seed)
    sc = product_scene_dict(d)
    sd = sc.scene_desc()
    cd, t = sc.camera_desc()
    rng = np.random.RandomState(11)
    aa = np.asarray(t["aa"], np.float64).reshape(-1, 3)
    boxes = [i for i, o in enumerate(d["objects"]) if o["type"] == "box"]
    marked = 0
    for li, l in enumerate(d["lights"]):
        if l["type"] != "directional":
            continue
        bits = hostemu.dsgrid_self(sc, li)
        if not bits:
            continue
        dvec = -np.asarray(sd.lights[li].vector[:3], np.float32)
        for k, i in enumerate(boxes):
            if not (bits >> (16 + k)) & 1:
                continue
            o = d["objects"][i]
            if "min" in o:
                mn, mx = np.minimum(o["min"], o["max"]), np.maximum(o["min"], o["max"])
            else:
                mn = np.asarray(o["position"]) - np.asarray(o["size"]) / 2
                mx = np.asarray(o["position"]) + np.asarray(o["size"]) / 2
            n = 6000
            tgt = rng.uniform(mn, mx, (n, 3))
            ax = rng.randint(3, size=n)
            tgt[np.arange(n), ax] = np.where(rng.rand(n) < 0.5, mn[ax], mx[ax])  # on a face
            edge = rng.rand(n) < 0.3
            ax2 = (ax + 1) % 3
            tgt[edge, ax2[edge]] = np.where(rng.rand(edge.sum()) < 0.5, mn[ax2[edge]], mx[ax2[edge]])
            org = aa[rng.randint(len(aa), size=n)] + rng.normal(size=(n, 3)) * 0.3 * float(t["jscale"])
            dr = tgt - org
            dr /= np.linalg.norm(dr, axis=1, keepdims=True)
            hit = hostemu.intersect(sc, org.astype(np.float32), dr.astype(np.float32))
            on = hit["obj"] == i
            one = copy.deepcopy(d)
            one["objects"] = [copy.deepcopy(o)]
            occ = hostemu.occluded(product_scene_dict(one), hit["position"][on], np.broadcast_to(dvec, (int(on.sum()), 3)),
                                   np.inf, 0.0)
            assert not occ.any(), (seed, li, k, int(on.sum()), int(occ.sum()))
            marked += int(on.sum())  # (a box inside another object takes no hits)
    assert marked > 1000 or seed not in ("dof", 1)


def test_hostemu_box_self_shadow_grazing_light_not_marked():
    """Under a grazing light (direction y = 1e-5) a box's own shadow test does pass for
    some camera hits on its top face (fp32 points just above it): such boxes must not be
    marked, and are not."""
    import copy
    from common import product_scene_dict
    from scenegen import shadow_scene
    d = shadow_scene(1)
    d["lights"] = [{"name": "g", "type": "directional", "direction": [1.0, 1e-5, 0.3], "colour": [1.0, 1.0, 1.0],
                    "power": 0.7}]
    sc = product_scene_dict(d)
    assert hostemu.dsgrid_self(sc, 0) == 0
    cd, t = sc.camera_desc()
    aa = np.asarray(t["aa"], np.float64).reshape(-1, 3)
    rng = np.random.RandomState(1)
    dvec = -np.asarray(sc.scene_desc().lights[0].vector[:3], np.float32)
    self_occ = 0
    for i, o in enumerate(d["objects"]):
        if o["type"] != "box" or "speed" in o:
            continue
        mn = np.minimum(o["min"], o["max"]) if "min" in o else np.asarray(o["position"]) - np.asarray(o["size"]) / 2
        mx = np.maximum(o["min"], o["max"]) if "min" in o else np.asarray(o["position"]) + np.asarray(o["size"]) / 2
        tgt = rng.uniform(mn, mx, (20000, 3))
        tgt[:, 1] = mx[1]
        org = aa[rng.randint(len(aa), size=20000)]
        dr = (tgt - org) / np.linalg.norm(tgt - org, axis=1, keepdims=True)
        hit = hostemu.intersect(sc, org.astype(np.float32), dr.astype(np.float32))
        on = hit["obj"] == i
        one = copy.deepcopy(d)
        one["objects"] = [copy.deepcopy(o)]
        self_occ += int(hostemu.occluded(product_scene_dict(one), hit["position"][on],
                                         np.broadcast_to(dvec, (int(on.sum()), 3)), np.inf, 0.0).sum())
    assert self_occ > 0


@pytest.mark.parametrize("case", ["TwoSpheresPlane", "DepthOfField", "MirrorRefraction", "rand0", "rand1", "rand2",
                                  "rand3", "shadow0", "shadow1", "lowlight"])
def test_hostemu_plane_self_shadow_never_passes(case):
    """The skipped self tests of planes (SceneView::plane_self): camera rays from the
    sample origins hit each plane near and far, head-on and grazing; wherever the hit
    point's max |p_i| is within the light's limit, the plane alone never occludes the
    point's shadow ray toward that light (the device's own test, d and t_max as
    regular_lighting casts them). 'lowlight' puts a point light 3e-4 above the ground
    (above the test's 1e-4 floor on |denom|): no limit there, and self-occluded points do
    exist."""
    import copy
    from common import product_scene_dict
    from rtx.io import bundled_scene_dict
    from scenegen import random_scene, shadow_scene
    if case.startswith("rand"):
        d = random_scene(int(case[4:]))
    elif case.startswith("shadow"):
        d = shadow_scene(int(case[6:]))
    elif case == "lowlight":
        d = random_scene(0)
        d["lights"] = [{"name": "low", "type": "point", "position": [1.0, -1.0 + 3e-4, 0.5],
                        "colour": [1.0, 1.0, 1.0], "power": 1.0}]
        d["objects"] = [o for o in d["objects"] if o["type"] == "plane"][:1]
        d["objects"][0]["position"] = [0.0, -1.0, 0.0]
        d["objects"][0]["normal"] = [0.0, 1.0, 0.0]
    else:
        d = bundled_scene_dict(case, resolution=(64, 48))
    sc = product_scene_dict(d)
    sd = sc.scene_desc()
    lim = hostemu.plane_self(sc)
    cd, t = sc.camera_desc()
    aa = np.asarray(t["aa"], np.float64).reshape(-1, 3)
    rng = np.random.RandomState(3)
    planes = [i for i, o in enumerate(d["objects"]) if o["type"] == "plane"]
    tested = self_occ = 0
    for k, i in enumerate(planes[:4]):
        o = d["objects"][i]
        if "speed" in o:
            continue
        p0, nrm = np.asarray(o["position"], np.float64), np.asarray(o["normal"], np.float64)
        u = np.cross(nrm, [0.3, 0.5, 0.7])
        u /= np.linalg.norm(u)
        v = np.cross(nrm / np.linalg.norm(nrm), u)
        n = 20000
        rad = np.exp(rng.uniform(np.log(0.01), np.log(400.0), n))  # near and far (grazing)
        ang = rng.uniform(0, 2 * np.pi, n)
        tgt = p0 + (np.cos(ang) * rad)[:, None] * u + (np.sin(ang) * rad)[:, None] * v
        org = aa[rng.randint(len(aa), size=n)]
        dr = (tgt - org) / np.linalg.norm(tgt - org, axis=1, keepdims=True)
        hit = hostemu.intersect(sc, org.astype(np.float32), dr.astype(np.float32))
        on = hit["obj"] == i
        P = hit["position"][on]
        m = np.abs(P).max(axis=1)
        one = copy.deepcopy(d)
        one["objects"] = [copy.deepcopy(o)]
        one.pop("motion", None)
        s1 = product_scene_dict(one)
        for li, l in enumerate(d["lights"]):
            if l["type"] == "directional":
                D = np.broadcast_to(-np.asarray(sd.lights[li].vector[:3], np.float32), P.shape)
                tmax = np.inf
            else:
                D = (np.asarray(sd.lights[li].vector[:3], np.float32) - P).astype(np.float32)
                tmax = 1.0
            occ = hostemu.occluded(s1, P, D, tmax, 0.0)
            within = m <= lim[li, k]
            assert not (occ & within).any(), (case, k, li, float(lim[li, k]), int((occ & within).sum()))
            tested += int(within.sum())
            self_occ += int(occ.sum())
    if case == "lowlight":
        assert (lim < 0).all() and self_occ > 0, (lim, self_occ)
    elif case in ("TwoSpheresPlane", "DepthOfField", "MirrorRefraction"):
        assert tested > 1000, tested  # (random scenes may have no limit: lights near a plane)


def test_hostemu_dir_shadow_grids_skip_most_rays(monkeypatch):
    """The grids are tight enough to pay: on DepthOfField (and on MirrorRefraction, whose
    four spheres alone get no grid unless RTX_DSGRID_MIN allows it) most floor points'
    shadow rays test no sphere or box."""
    rng = np.random.RandomState(1)
    p = np.c_[rng.uniform(-6, 6, (4000, 1)), np.zeros((4000, 1)), rng.uniform(-8, 3, (4000, 1))].astype(np.float32)
    assert hostemu.dir_shadow_mask(product_scene("MirrorRefraction", (8, 8)), p, 0) is None
    monkeypatch.setattr(OPTS, "dsgrid_min", "1")
    for name in ("DepthOfField", "MirrorRefraction"):
        m = hostemu.dir_shadow_mask(product_scene(name, (8, 8)), p, 0)
        assert m is not None
        assert (m[:, 0] == 0).mean() > 0.6, (name, float((m[:, 0] == 0).mean()))


@pytest.mark.parametrize("seed", range(12))
def test_hostemu_dir_shadow_grids_equal_walk(seed, monkeypatch):
    """Frames with the directional shadow grids == without (RTX_DSGRID=0) == the oracle."""
    from common import oracle_render_dict, product_scene_dict
    from scenegen import shadow_scene
    monkeypatch.setattr(OPTS, "dsgrid_min", "1")
    d = shadow_scene(seed)
    img, cnt = hostemu.render(product_scene_dict(d))
    monkeypatch.setattr(OPTS, "dsgrid", "0")
    walk, cnt2 = hostemu.render(product_scene_dict(d))
    monkeypatch.setattr(OPTS, "dsgrid", "1")
    assert np.array_equal(img, walk)
    assert np.array_equal(cnt, cnt2)
    assert_parity(img, oracle_render_dict(d), "shadow grids seed %d" % seed)


@pytest.mark.parametrize("name", ["TwoSpheresPlane", "MirrorRefraction", "TorusMesh", "DepthOfField"])
def test_jit_baked_records_are_the_scene_records(name):
    """The prelude of the one-sample scene-specialized kernels (rtx_api.hip
    jit_baked_records) holds exactly the object, material and light records the scene
    uploads: one DObj (56 words), DMat (20) and DLight (20) per record, objects grouped
    by type (planes, spheres, boxes, meshes) and materials' diffuse colours in f32."""
    import re
    sc = product_scene(name, (64, 48))
    src = hostemu.jit_baked(sc)
    assert src.rstrip().endswith("#define RTX_BAKED_RECORDS 1")
    arrays = {m.group(1): [int(w, 16) for w in re.findall(r"0x([0-9a-f]+)u", m.group(2))]
              for m in re.finditer(r"static constexpr unsigned (\w+)\[\] = \{([^}]*)\}", src)}
    objs, mats, lights = arrays["kObjs"], arrays["kMats"], arrays["kLights"]
    assert len(objs) == 56 * len(sc.objects)
    assert len(mats) == 20 * len(sc.materials)
    assert len(lights) == 20 * len(sc.lights)
    kinds = [objs[56 * i] for i in range(len(sc.objects))]  # DObj::type: sphere 0, plane 1, box 2, mesh 3
    assert kinds == sorted(kinds, key=lambda k: [1, 0, 2, 3].index(k))
    want = sorted({"sphere": 0, "plane": 1, "box": 2, "mesh": 3}[o.gtype] for o in sc.objects)
    assert sorted(kinds) == want
    for i, m in enumerate(sc.materials):
        got = np.array(mats[20 * i:20 * i + 3], np.uint32).view(np.float32)
        assert np.array_equal(got, np.asarray(m.diffuse, np.float32)), (i, got, m.diffuse)


SPLIT_CASES = [("NovelScene1", (64, 32), {"AA": {"jitter": False, "samples": 2}}),
               ("NovelScene2", (48, 24), {"AA": {"jitter": False, "samples": 1}})]


@pytest.mark.parametrize("budget", [1 << 31, 2000 * 40])
@pytest.mark.parametrize("name,res,edits", SPLIT_CASES)
def test_hostemu_split_passes_bit_exact(name, res, edits, budget):
    """The hierarchy scenes' three split passes (csrc/rtx_split.h: chains of closest hits,
    then shadow rays per record, then lighting + unwinding + the ordered mean), host build,
    one chunk or many: bit-identical to the oracle, with its ray tallies."""
    sc = product_scene(name, res, **edits)
    img, cnt = hostemu.render_split(sc, budget=budget)
    ref, tl = oracle_render(name, res, tallies=True, **edits)
    assert_parity(img, ref, name)
    assert list(cnt[:10]) == tl[:10]
    assert cnt[10] == tl[11] and cnt[11] == tl[12]


@pytest.mark.parametrize("ratio,budget", [(0.0, 1 << 31), (0.02, 3000 * 40), (0.3, 1 << 31)])
def test_hostemu_split_pool_overflow_redo(ratio, budget):
    """A deeper-record pool smaller than the chains need (rtx_split.h): the hits that find
    it full mark their blocks, which are rendered again in the one-kernel form -- the frame
    is still the oracle's, bit for bit, and blocks were in fact redone."""
    from common import oracle_render_dict, product_scene_dict
    from scenegen import random_hier_scene
    d = random_hier_scene(3, res=(40, 30))
    d["materials"] = [dict(m, type="mirror", tint=m.get("tint", 0.3)) if i % 2 == 0 else m for i, m in enumerate(d["materials"])]
    img, _, redone = hostemu.render_split(product_scene_dict(d), budget=budget, ratio=ratio, with_redone=True)
    assert_parity(img, oracle_render_dict(d), "pool overflow %g" % ratio)
    assert redone > 0


@pytest.mark.parametrize("seed", range(12))
def test_hostemu_split_random_hierarchy_scenes(seed):
    """Random CSG trees (mirrors and refractive materials included) through the split
    passes, in small chunks: bit-exact image and ray tallies against the oracle."""
    from common import oracle_render_dict, product_scene_dict
    from scenegen import random_hier_scene
    d = random_hier_scene(seed, mesh=(seed % 4 == 0))
    img, cnt = hostemu.render_split(product_scene_dict(d), budget=3000 * 40)
    ref, tl = oracle_render_dict(d, tallies=True)
    assert_parity(img, ref, "seed %d" % seed)
    assert list(cnt[:10]) == tl[:10] and cnt[10] == tl[11]
