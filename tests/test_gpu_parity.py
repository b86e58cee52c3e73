"""Parity of the HIP path (librtx.so on the MI355X) against the CPU oracle."""
import numpy as np
import pytest
import torch

from common import assert_parity, compare, oracle_render, product_scene
from common import OPTS

pytestmark = pytest.mark.gpu

CASES = [
    ("TwoSpheresPlane", (160, 120), {}),
    ("TwoSpheresPlane", (97, 61), {"AA": {"jitter": False, "samples": 3}}),
    ("MirrorRefraction", (180, 102), {}),
    ("TorusMesh", (128, 128), {}),
    ("TorusMesh", (64, 64), {"flat_shaded": False}),
    ("MotionBlur", (75, 64), {}),
    ("DepthOfField", (40, 30), {"AA": {"jitter": False, "samples": 2}}),
]


@pytest.fixture(scope="module", autouse=True)
def _device():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    torch.cuda.set_device(0)


@pytest.mark.parametrize("name,res,edits", CASES)
def test_render_matches_oracle(name, res, edits):
    sc = product_scene(name, res, **edits)
    img = sc.render()
    ref = oracle_render(name, res, **edits)
    s = assert_parity(img, ref, name)
    print(name, res, s)


@pytest.mark.parametrize("name", ["TwoSpheresPlane", "MirrorRefraction", "TorusMesh"])
def test_config_size_1080p_matches_oracle(name):
    """BASELINE.json configs 2-4 at their full 1920x1080 size against the oracle. Three
    frames: the first measures the tile schedule of the secondary-ray and mesh scenes, the
    later ones run in its longest-first order (rtx_api.hip tile_schedule) -- same bytes."""
    sc = product_scene(name, (1920, 1080), AA={"jitter": False, "samples": 1})
    ref = oracle_render(name, (1920, 1080), AA={"jitter": False, "samples": 1})
    kernels = []
    for _ in range(3):
        s = assert_parity(sc.render(), ref, name)
        kernels.append(sc.last_kernel)
    print(name, "1080p", s, kernels)
    assert not kernels[0].endswith("+tiles")
    assert kernels[2].endswith("+tiles") == (name != "TwoSpheresPlane"), kernels


@pytest.mark.parametrize("name,res", [("MirrorRefraction", (1000, 600)), ("TorusMesh", (1920, 1080)),
                                      ("TwoSpheresPlane", (333, 257))])
def test_xcd_block_order_equal(name, res, monkeypatch):
    """The XCD-aware block order (rtx_kernels.h xcd_block, option xcd_map) renders the same
    bytes as dispatch order -- sizes whose last round of blocks is incomplete, eager frames
    through the tile schedule's measure/sort/scheduled states -- and a scene whose schedule
    table was laid out under one setting keeps rendering right after the option flips."""
    sc = product_scene(name, res)
    imgs = [sc.render_device().cpu().numpy() for _ in range(3)]
    monkeypatch.setattr(OPTS, "xcd_map", "0")
    imgs.append(sc.render_device().cpu().numpy())  # (the table sorted under xcd_map 1)
    sc0 = product_scene(name, res)
    imgs += [sc0.render_device().cpu().numpy() for _ in range(3)]
    monkeypatch.setattr(OPTS, "xcd_map", "1")
    imgs.append(sc0.render_device().cpu().numpy())  # (the table sorted under xcd_map 0)
    imgs.append(sc0.render_device(row0=40, nrows=77).cpu().numpy())
    for k, a in enumerate(imgs[:-1]):
        assert np.array_equal(a, imgs[0]), (name, k)
    assert np.array_equal(imgs[-1], imgs[0][40:117]), name


def test_counters_match_oracle_tallies():
    for name, res in (("MirrorRefraction", (192, 108)), ("TorusMesh", (96, 54)), ("TwoSpheresPlane", (192, 108))):
        sc = product_scene(name, res)
        cnt = torch.zeros(16, dtype=torch.int64, device="cuda")
        sc.render_device(counters=cnt)
        c = cnt.cpu().numpy()
        _, tl = oracle_render(name, res, tallies=True)
        assert list(c[:10]) == tl[:10] and c[10] == tl[11] and c[11] == tl[12], (name, c, tl)


def test_jitter_replay_matches_oracle():
    edits = {"AA": {"jitter": True, "samples": 2}}
    res = (48, 32)
    noise = np.random.RandomState(11).rand(48 * 32 * 2 * 32 * 3)
    sc = product_scene("DepthOfField", res, **edits)
    sc.jitter_noise = noise
    ref = oracle_render("DepthOfField", res, noise=noise, **edits)
    assert_parity(sc.render(), ref, "DOF replay")


def _philox_noise(sc, col0, ncols):
    from oracle import philox as PH
    return PH.jitter_noise(sc.seed, col0, ncols, sc.vc.height, sc.vc.dof_samples, sc.samples)


def test_philox_config5_kernel_bit_exact():
    """BASELINE config 5 as the bench times it: DepthOfField 3840x2160, AA 2 x DOF 32,
    production (Philox) jitter, the whole frame in one launch of the scene-specialized
    kernel rtx_jit_render_00001 (the replay-mode variant is named *_replay). Columns of
    that framebuffer against the oracle fed with the restated Philox stream
    (oracle/philox.py): bit-identical, 138,240 samples per column."""
    edits = {"AA": {"jitter": True, "samples": 2}}
    res = (3840, 2160)
    sc = product_scene("DepthOfField", res, **edits)
    assert sc.jitter_noise is None
    fb = sc.render_device()  # [H][W][3] fp32, row 0 = top
    torch.cuda.synchronize()
    assert sc.last_kernel == "rtx_jit_render_00001", sc.last_kernel
    for col in (3000, 0, 1921, 3839):
        got = fb[:, col, :].flip(0).double().cpu().numpy()[None]  # (1, H, 3), reference row order
        ref = oracle_render("DepthOfField", res, subimage=col, tasks=3840, noise=_philox_noise(sc, col, 1), **edits)
        assert_parity(got, ref, "DOF 4K Philox column %d" % col)


@pytest.mark.parametrize("res,subimage,tasks", [((64, 48), 0, 1), ((64, 48), 5, 8), ((3840, 2160), 3000, 3840)])
def test_philox_frames_bit_exact(res, subimage, tasks):
    """Philox-mode DepthOfField frames and strips (a 64x48 frame, a strip starting at
    column 40, and config 5's column 3000 rendered as its own 1-column strip) against the
    oracle with the restated stream."""
    edits = {"AA": {"jitter": True, "samples": 2}}
    sc = product_scene("DepthOfField", res, **edits)
    img = sc.render(subimage, tasks)
    assert sc.last_kernel == "rtx_jit_render_00001", sc.last_kernel
    from rtx.scene import strip_columns
    col0, ncols = strip_columns(res[0], subimage, tasks)
    ref = oracle_render("DepthOfField", res, subimage=subimage, tasks=tasks, noise=_philox_noise(sc, col0, ncols), **edits)
    assert_parity(img, ref, "DOF Philox %s strip %d/%d" % (res, subimage, tasks))


def test_philox_jitter_is_deterministic_and_statistically_matches():
    """Production jitter (Philox keyed by pixel and sample) vs the oracle with numpy's
    stream (the reference's unseeded np.random): same distribution."""
    edits = {"AA": {"jitter": True, "samples": 1}}
    res = (128, 128)
    sc = product_scene("DepthOfField", res, **edits)
    a = sc.render()
    b = sc.render()
    assert np.array_equal(a, b)
    ref = oracle_render("DepthOfField", res, noise=np.random.RandomState(5).rand(128 * 128 * 32 * 3), **edits)
    from oracle import oracle as O
    d = O.to_png_array(a).astype(int) - O.to_png_array(ref).astype(int)
    assert np.abs(d).mean() < 0.5 and abs(d.mean()) < 0.1


@pytest.mark.parametrize("tasks", [2, 3, 5])
def test_strip_render_matches_oracle(tasks):
    res = (91, 40)
    sc = product_scene("MirrorRefraction", res)
    for k in range(tasks):
        img = sc.render(k, tasks)
        ref = oracle_render("MirrorRefraction", res, subimage=k, tasks=tasks)
        assert compare(img, ref)["frac_diff"] == 0.0


def test_row_blocks_are_partition_invariant():
    """Rank row blocks (multi-GPU partition) reassemble to the single-launch frame."""
    from rtx.scene import split_rows
    sc = product_scene("MirrorRefraction", (320, 181))
    full = sc.render_device().clone()
    for n in (2, 3, 8):
        parts = []
        for k in range(n):
            r0, nr = split_rows(181, n, k)
            parts.append(sc.render_device(row0=r0, nrows=nr))
        assert torch.equal(torch.cat(parts), full)


def test_rgb8_matches_main_py_conversion():
    from oracle import oracle as O
    sc = product_scene("TwoSpheresPlane", (160, 90))
    img = sc.render()
    assert np.array_equal(sc.render_rgb8(), O.to_png_array(img))


@pytest.mark.parametrize("name", ["TwoSpheresPlane", "MirrorRefraction", "TorusMesh", "DepthOfField", "MotionBlur"])
def test_geometry_kat(name):
    """Closest hit / shadow any-hit of random SoA rays vs the oracle (Geometry ABI)."""
    from oracle import oracle as O
    rng = np.random.RandomState(3)
    n = 20000
    o = (np.array([0, 1, 0]) + rng.uniform(-4, 4, (n, 3))).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    sc = product_scene(name, (8, 8))
    dd, base = O.load_bundle(name)
    osc = O.OracleScene(dd, base)
    for time in (0.0, 0.75):
        got = sc.intersect(o, d, time)
        t, ob, _, m, nn, pp = osc.closest(time, o, d)
        hit = ob >= 0
        assert np.array_equal(got["obj"], ob)
        assert np.array_equal(got["t"][hit], t[hit]) and np.array_equal(got["mat"], m)
        assert np.array_equal(got["normal"][hit], nn[hit]) and np.array_equal(got["position"][hit], pp[hit])
        for tmax in (1.0, np.inf):
            assert np.array_equal(sc.occluded(o, d, tmax, time), osc.shadow(time, o, d, tmax).astype(bool))


@pytest.mark.parametrize("seed", range(3))
def test_mesh_bv_stress_matches_oracle(seed):
    """Rays inside / on / grazing the torus's bounding box vs the oracle, exactly (the
    fp32 decision of BoundingAABB.intersect and its fp64 fallback)."""
    import os
    from oracle import oracle as O
    from scenegen import bv_stress_rays, obj_bounds
    lo, hi = obj_bounds(os.path.join(os.path.dirname(__file__), "..", "assets", "torus_mesh.obj"))
    o, d = bv_stress_rays(lo, hi, 20000, seed)
    sc = product_scene("TorusMesh", (8, 8))
    dd, base = O.load_bundle("TorusMesh")
    osc = O.OracleScene(dd, base)
    got = sc.intersect(o, d, 0.0)
    t, ob, _, m, nn, pp = osc.closest(0.0, o, d)
    assert np.array_equal(got["obj"], ob)
    hit = ob >= 0
    assert np.array_equal(got["t"][hit], t[hit])
    for tmax in (1.0, np.inf):
        assert np.array_equal(sc.occluded(o, d, tmax, 0.0), osc.shadow(0.0, o, d, tmax).astype(bool))


@pytest.mark.parametrize("seed", range(3))
def test_box_stress_matches_oracle(seed):
    """Rays inside / on / grazing / aimed at the edges and corners of DepthOfField's two
    boxes vs the oracle, exactly: the fp32 slab decision (box_slabs_iv), the single fp64
    entry division and the full fp64 fallback of AABB.intersect / shadow_intersect
    (simple_geometry.py:188-294), for closest hits and shadows with t_max 1 and inf."""
    from oracle import oracle as O
    from scenegen import scene_box_stress_rays
    dd, base = O.load_bundle("DepthOfField")
    o, d = scene_box_stress_rays(dd, 10000, seed)
    sc = product_scene("DepthOfField", (8, 8))
    osc = O.OracleScene(dd, base)
    got = sc.intersect(o, d, 0.0)
    t, ob, _, m, nn, pp = osc.closest(0.0, o, d)
    assert np.array_equal(got["obj"], ob)
    hit = ob >= 0
    assert np.array_equal(got["t"][hit], t[hit])
    assert np.array_equal(got["normal"][hit], nn[hit])
    for tmax in (1.0, np.inf):
        assert np.array_equal(sc.occluded(o, d, tmax, 0.0), osc.shadow(0.0, o, d, tmax).astype(bool))


def test_full_size_dof_4k_properties():
    """DepthOfField 3840x2160, AA 2 x DOF 32 (config 5): a 64-row block. Values in [0, 1],
    deterministic, and identical when split into sub-blocks (partition invariance)."""
    sc = product_scene("DepthOfField", (3840, 2160), AA={"jitter": True, "samples": 2})
    a = sc.render_device(row0=1000, nrows=64)
    b = torch.cat([sc.render_device(row0=1000, nrows=32), sc.render_device(row0=1032, nrows=32)])
    assert torch.equal(a, b)
    assert float(a.min()) >= 0.0 and float(a.max()) <= 1.0


@pytest.mark.parametrize("seed", range(24))
def test_random_scenes_match_oracle(seed):
    from common import oracle_render_dict, product_scene_dict
    from scenegen import random_scene
    d = random_scene(seed, res=(64, 48), mesh=(seed % 3 == 0))
    img = product_scene_dict(d).render()
    ref = oracle_render_dict(d)
    assert_parity(img, ref, "seed %d" % seed)


@pytest.mark.parametrize("seed", range(8))
def test_random_static_uniform_hardness_scenes_match_oracle(seed):
    """Random scenes whose facts the specialized kernels pin: no speeds (static scene),
    one integer hardness for every material (pow as a fixed multiplication chain), point
    and directional lights, AA 1 or 4 (pinned sample counts)."""
    from common import oracle_render_dict, product_scene_dict
    from scenegen import random_scene
    d = random_scene(100 + seed, res=(64, 48), mesh=(seed % 4 == 0))
    h = [0, 1, 16, 32, 50, 3, 7, 64][seed]
    for m in d["materials"]:
        m["hardness"] = h
    for o in d["objects"]:
        o.pop("speed", None)
    if seed % 2:
        d["AA"] = {"jitter": False, "samples": 4}
    assert_parity(product_scene_dict(d).render(), oracle_render_dict(d), "static seed %d" % seed)


@pytest.mark.parametrize("seed", range(16))
def test_point_lights_scenes_match_oracle(seed, monkeypatch):
    """Planes and spheres under 2-8 point lights: the specialized kernel tests every
    light's shadow ray at once (rtx_trace.h occluded_points); bit-exact with the oracle,
    and equal to the one-light-at-a-time kernel (RTX_LIGHTS_TOGETHER=0)."""
    from common import OPTS, oracle_render_dict, product_scene_dict
    from scenegen import point_lights_scene
    d = point_lights_scene(seed)
    img = product_scene_dict(d).render()
    assert_parity(img, oracle_render_dict(d), "point lights seed %d" % seed)
    monkeypatch.setattr(OPTS, "jit_flags", "-DRTX_LIGHTS_TOGETHER=0")
    assert np.array_equal(product_scene_dict(d).render(), img)


@pytest.mark.parametrize("mirror", [False, True])
def test_ties_follow_scene_order(mirror):
    """Coincident objects: scene order breaks closest-hit ties (offer()); with a mirror the
    secondary-ray kernel meets them too, through its deferred tie pass (RTX_DEFER_TIES)."""
    from common import oracle_render_dict, product_scene_dict
    from scenegen import tie_scene
    d = tie_scene((80, 60), mirror=mirror)
    sc = product_scene_dict(d)
    assert compare(sc.render(), oracle_render_dict(d))["frac_diff"] == 0.0
    if mirror:
        assert sc.last_kernel.startswith("rtx_jit_render_01"), sc.last_kernel


HIER_CASES = [
    ("NovelScene1", (256, 128), {"AA": {"jitter": False, "samples": 1}}),
    ("NovelScene2", (128, 64), {"AA": {"jitter": False, "samples": 1}}),
]


@pytest.mark.parametrize("name,res,edits", HIER_CASES)
def test_hierarchy_scenes_match_oracle(name, res, edits):
    """CSG hierarchies + textures (+ motion blur, DOF for NovelScene2) vs the oracle."""
    sc = product_scene(name, res, **edits)
    s = assert_parity(sc.render(), oracle_render(name, res, **edits), name)
    assert s["frac_diff"] == 0.0, s


@pytest.mark.parametrize("name,max_mean", [("NovelScene1", 0.1), ("NovelScene2", 0.2)])
def test_novel_scenes_full_size_match_published_render(name, max_mean):
    """The full configs of renders/NovelScene{1,2}.png (2048x1024 AA32, and 1024x512
    AA2 x DOF15 x 16 motion times, both jittered with the reference's unseeded RNG) against
    the published PNGs: Philox jitter vs unseeded numpy, so the comparison is statistical."""
    import os
    from PIL import Image
    from oracle import oracle as O
    sc = product_scene(name)
    png = sc.render_rgb8()
    pub = np.asarray(Image.open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "published",
                                             name + ".png")).convert("RGB"))
    assert png.shape == pub.shape
    d = png.astype(int) - pub.astype(int)
    print(name, "mean|d| %.4f bias %.4f exact %.4f" % (np.abs(d).mean(), d.mean(), (np.abs(d).max(axis=2) == 0).mean()))
    assert np.abs(d).mean() < max_mean and abs(d.mean()) < 0.05
    assert (np.abs(d).max(axis=2) == 0).mean() > 0.93


@pytest.mark.parametrize("seed", range(24))
def test_random_hierarchy_scenes_match_oracle(seed):
    from common import oracle_render_dict, product_scene_dict
    from scenegen import random_hier_scene
    d = random_hier_scene(seed, res=(64, 48), mesh=(seed % 4 == 0))
    s = assert_parity(product_scene_dict(d).render(), oracle_render_dict(d), "hier seed %d" % seed)
    assert s["frac_diff"] == 0.0, s


def test_hierarchy_geometry_kat():
    from oracle import oracle as O
    rng = np.random.RandomState(3)
    n = 20000
    o = (np.array([0, 1, 0]) + rng.uniform(-3, 3, (n, 3))).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    sc = product_scene("NovelScene1", (8, 8))
    dd, base = O.load_bundle("NovelScene1")
    osc = O.OracleScene(dd, base)
    for time in (0.0, 0.5):
        got = sc.intersect(o, d, time)
        t, ob, _, m, nn, pp = osc.closest(time, o, d)
        assert np.array_equal(got["obj"], ob)
        hit = ob >= 0
        assert np.array_equal(got["t"][hit], t[hit]) and np.array_equal(got["mat"], m)
        assert np.array_equal(got["normal"][hit], nn[hit]) and np.array_equal(got["position"][hit], pp[hit])
        for tmax in (1.0, np.inf):
            assert np.array_equal(sc.occluded(o, d, tmax, time), osc.shadow(time, o, d, tmax).astype(bool))


@pytest.mark.parametrize("flat", [False, True])
def test_large_mesh_bvh_matches_oracle(tmp_path, flat):
    """81,920-face mesh (bunny-sized stand-in) through the device BVH."""
    from common import oracle_render_dict, product_scene_dict
    from scenegen import blob_obj, blob_scene
    p = str(tmp_path / "blob6.obj")
    blob_obj(p, level=6)
    d = blob_scene(p, (64, 64), flat)
    s = assert_parity(product_scene_dict(d).render(), oracle_render_dict(d), "blob")
    assert s["frac_diff"] == 0.0, s


def test_heavy_tiles_equal_walk(tmp_path, monkeypatch):
    """Heavy primary-ray tiles (a bin's face list longer than kHeavyChunk faces, tested in
    chunks by k_mesh_chunks before the render kernel, rtx_api.hip heavy_chunks): the
    81,920-face mesh at 1920x1080 and 256x144 and TorusMesh at 64x64 (its bins are heavy
    at that size) with and without them, bit for bit; the small frames also against the
    oracle; groups of 8-row groups too (the pass runs only its launch's tiles)."""
    from common import oracle_render_dict, product_scene_dict
    from scenegen import blob_obj, blob_scene
    from rtx.io import bundled_scene_dict
    p = str(tmp_path / "blob6.obj")
    blob_obj(p, level=6)
    cases = [(blob_scene(p, (1920, 1080)), False), (blob_scene(p, (256, 144)), True),
             (bundled_scene_dict("TorusMesh", resolution=(64, 64)), True)]
    for d, small in cases:
        d = {k: v for k, v in d.items() if k != "__base_dir__"}
        sc = product_scene_dict(d)
        a = sc.render_device().clone()
        assert sc.last_kernel.startswith("rtx_jit_render_1"), sc.last_kernel
        H = a.shape[0]
        from rtx.scene import group_rows
        for k in range(3):
            part = sc.render_device(groups=(k, 3)).clone()
            assert torch.equal(part, a[torch.as_tensor(group_rows(H, 3, k), device="cuda")])
        monkeypatch.setattr(OPTS, "heavy_tiles", "0")
        b = product_scene_dict(d).render_device().clone()
        monkeypatch.setattr(OPTS, "heavy_tiles", "1")
        assert torch.equal(a, b), float((a != b).float().mean())
        if small:
            img = np.ascontiguousarray(np.transpose(a.cpu().numpy()[::-1], (1, 0, 2))).astype(np.float64)
            assert_parity(img, oracle_render_dict(d), "heavy tiles")


def test_device_face_bins_equal_host(tmp_path, monkeypatch):
    """A mesh's primary-ray face bins built on the device (option dev_bins, rtx_bins.hip:
    the host's projection arithmetic, rtx_bins.h, then two radix sorts) render the frames
    of the host-built bins and of no bins at all, bit for bit: the 81,920-face mesh at
    1920x1080 (heavy tiles included) and at a size that is not a multiple of 8, TorusMesh
    at 1080p; the small ones also against the oracle. Each camera is set twice, so the
    scratch is reused, and a camera move re-bins."""
    from common import oracle_render_dict, product_scene_dict
    from scenegen import blob_obj, blob_scene
    from rtx.io import bundled_scene_dict
    p = str(tmp_path / "blob6.obj")
    blob_obj(p, level=6)
    cases = [(blob_scene(p, (1920, 1080)), False), (blob_scene(p, (203, 117)), True),
             (bundled_scene_dict("TorusMesh", resolution=(1920, 1080)), False),
             (bundled_scene_dict("TorusMesh", resolution=(97, 61)), True)]
    for d, small in cases:
        d = {k: v for k, v in d.items() if k != "__base_dir__"}
        frames = {}
        for opt, val in (("dev_bins", "1"), ("dev_bins", "0"), ("bins", "0")):
            monkeypatch.setattr(OPTS, opt, val)
            sc = product_scene_dict(d)
            frames[(opt, val)] = sc.render_device().clone()
            sc.vc.set_camera(sc.vc.position + np.float32(0.05), [0.0, 0.5, 0.0], [0.0, 1.0, 0.0], 40)
            frames[(opt, val, "moved")] = sc.render_device().clone()
            monkeypatch.setattr(OPTS, opt, "1")
        for key in (("dev_bins", "0"), ("bins", "0")):
            assert torch.equal(frames[("dev_bins", "1")], frames[key]), key
            assert torch.equal(frames[("dev_bins", "1", "moved")], frames[key + ("moved",)]), key
        if small:
            a = frames[("dev_bins", "1")]
            img = np.ascontiguousarray(np.transpose(a.cpu().numpy()[::-1], (1, 0, 2))).astype(np.float64)
            assert_parity(img, oracle_render_dict(d), "device face bins")


@pytest.mark.parametrize("name,res,edits", [
    ("TwoSpheresPlane", (160, 90), {}), ("MirrorRefraction", (160, 90), {}), ("TorusMesh", (96, 96), {}),
    ("DepthOfField", (64, 48), {"AA": {"jitter": True, "samples": 2}}),
    ("NovelScene1", (128, 64), {"AA": {"jitter": True, "samples": 2}}),
])
def test_scene_specialized_kernel_equals_generic(name, res, edits, monkeypatch):
    """rtx_render's hiprtc kernel (object/light counts pinned) vs the precompiled generic
    kernel: identical framebuffers and counters, and rtx_last_kernel shows that each side
    really ran the kernel it is meant to (hierarchy/texture scenes specialize only under
    RTX_JIT_EXT=1, which this test sets)."""
    monkeypatch.setattr(OPTS, "jit_ext", "1")
    monkeypatch.setattr(OPTS, "split", "0")  # the generic side: the one-kernel form
    sc = product_scene(name, res, **edits)
    cnt_a = torch.zeros(16, dtype=torch.int64, device="cuda")
    a = sc.render_device(counters=cnt_a).clone()
    assert sc.last_kernel.startswith("rtx_jit_render_"), sc.last_kernel
    monkeypatch.setattr(OPTS, "jit", "0")
    cnt_b = torch.zeros(16, dtype=torch.int64, device="cuda")
    b = sc.render_device(counters=cnt_b).clone()
    assert sc.last_kernel.startswith("k_render"), sc.last_kernel
    assert torch.equal(a, b) and torch.equal(cnt_a, cnt_b)


@pytest.mark.parametrize("name", ["TwoSpheresPlane", "MirrorRefraction", "TorusMesh"])
@pytest.mark.parametrize("opt,value", [("tile_block", "256"), ("jit_ilp", "0"), ("prim_origin", "0")])
def test_codegen_options_render_the_default_bytes(name, opt, value, monkeypatch):
    """The code-generation options off their defaults -- 256-thread
    blocks for the secondary-ray / mesh kernels, no max-ILP scheduling or kernel-argument
    preload, no host-computed primary-ray origin terms -- render the default kernel's bytes
    at the configs' 1920x1080 size (three frames: the tile schedule's measured and sorted
    orders too)."""
    sc = product_scene(name, (1920, 1080), AA={"jitter": False, "samples": 1})
    base = sc.render_device().clone()
    k0 = sc.last_kernel
    monkeypatch.setattr(OPTS, opt, value)
    sc.invalidate()  # (options are read when a camera's kernels are resolved)
    for _ in range(3):
        alt = sc.render_device()
        assert torch.equal(base, alt), (name, opt, k0, sc.last_kernel)
    assert sc.last_kernel.startswith("rtx_jit_render_"), sc.last_kernel


def test_default_flat_scenes_run_the_specialized_kernel():
    """The production path for flat scenes is the scene-specialized kernel (bench.py reports
    its name); hierarchy/texture scenes run the split passes (csrc/rtx_split.h) specialized
    on their CSG trees (option jit_csg)."""
    for name, prefix in (("TwoSpheresPlane", "rtx_jit_render_00000"), ("TorusMesh", "rtx_jit_render_10000"),
                         ("MirrorRefraction", "rtx_jit_render_01000"), ("NovelScene1", "rtx_jit_split_")):
        sc = product_scene(name, (64, 32))
        sc.render_device()
        assert sc.last_kernel.startswith(prefix), (name, sc.last_kernel)


def test_camera_changes_rerender():
    """Moving the camera / changing samples after a render re-uploads the tables (the
    reference reads the camera on every render), and invalidate() re-reads the objects:
    a scene that rendered before each change equals a fresh scene built with it."""
    def moved(sc):
        sc.vc.set_camera([1.0, 2.5, 6.0], [0.0, 0.5, 0.0], [0.0, 1.0, 0.0], 40)
        return sc
    sc = product_scene("TwoSpheresPlane", (96, 72))
    first = sc.render()
    img = moved(sc).render()
    assert not np.array_equal(img, first)
    assert np.array_equal(img, moved(product_scene("TwoSpheresPlane", (96, 72))).render())
    sc.samples = 3
    fresh = moved(product_scene("TwoSpheresPlane", (96, 72)))
    fresh.samples = 3
    assert np.array_equal(sc.render(), fresh.render())
    k = next(i for i, o in enumerate(sc.objects) if hasattr(o, "radius"))
    for s in (sc, fresh):
        s.objects[k].center = s.objects[k].center + np.float32(0.25)
    fresh.invalidate()
    sc.invalidate()
    assert np.array_equal(sc.render(), fresh.render())


def test_edits_between_renders_match_oracle():
    """a sphere centre, a material's diffuse colour, a light's power, a
    plane's checker material and an appended object are edited between renders -- in
    place, with no invalidate() -- and every render equals the oracle of the edited scene
    JSON (the reference reads the objects, materials and lights on every render,
    provided/scene.py:86-88, :148, :161-164). Both the fp32 frame (render) and the fused
    uint8 path (render_rgb8) re-upload."""
    from common import oracle_render_dict, product_scene_dict
    from rtx.geometry import Sphere
    from rtx.io import bundled_scene_dict
    d = bundled_scene_dict("TwoSpheresPlane", resolution=(96, 72))
    d.pop("__base_dir__", None)
    sc = product_scene_dict(d)
    assert_parity(sc.render(), oracle_render_dict(d), "before edits")
    k = next(i for i, o in enumerate(d["objects"]) if o["type"] == "sphere")
    steps = [
        ("sphere centre", lambda: sc.objects[k].center.__setitem__(1, np.float32(0.75)),
         lambda: d["objects"][k]["position"].__setitem__(1, 0.75)),
        ("material diffuse", lambda: sc.materials[1].diffuse.__setitem__(slice(None), (0.25, 0.5, 0.125)),
         lambda: d["materials"][1].__setitem__("diffuse", [0.25, 0.5, 0.125])),
        ("light power", lambda: setattr(sc.lights[0], "power", 0.25),
         lambda: d["lights"][0].__setitem__("power", 0.25)),
        ("checker material", lambda: sc.objects[0].materials.__setitem__(1, sc.materials[0]),
         lambda: d["objects"][0]["materials"].__setitem__(1, 0)),
        ("appended sphere", lambda: sc.objects.append(Sphere("s2", "sphere", [sc.materials[3]],
                                                             np.array([1.5, 0.4, 0.5], np.float32), 0.4, None)),
         lambda: d["objects"].append({"materials": [3], "name": "s2", "position": [1.5, 0.4, 0.5], "radius": 0.4,
                                      "type": "sphere"})),
    ]
    prev = sc.render()
    for what, edit_product, edit_json in steps:
        gen = sc._gen
        edit_product()
        edit_json()
        ref = oracle_render_dict(d)
        img = sc.render()
        assert_parity(img, ref, what)
        assert not np.array_equal(img, prev), what  # the edit shows
        assert sc._gen != gen, what                 # one re-upload
        assert np.array_equal(sc.render_rgb8(), (np.rot90(ref, k=1, axes=(0, 1)) * 255).astype(np.uint8)), what
        prev = img
    assert isinstance(sc.objects[k], Sphere)


SPP_CASES = CASES + [
    ("NovelScene1", (96, 48), {"AA": {"jitter": False, "samples": 2}}),
    ("NovelScene2", (64, 32), {"AA": {"jitter": False, "samples": 1}}),
]


@pytest.mark.parametrize("name,res,edits", SPP_CASES)
def test_sample_parallel_mapping_matches_oracle(name, res, edits, monkeypatch):
    """The sample-parallel mapping (render_body_spp, forced for every sample count, 1 to
    NovelScene2's 240) vs the oracle: exact, i.e. the owner lanes' in-order LDS sums equal
    the reference's per-pixel accumulation."""
    monkeypatch.setattr(OPTS, "spp", "1")
    monkeypatch.setattr(OPTS, "split", "0")  # hierarchy scenes: the one-kernel form's mapping
    sc = product_scene(name, res, **edits)
    W, H = res
    fb = torch.full((H, W, 3), float("nan"), dtype=torch.float32, device="cuda")  # every pixel must be written
    sc.render_device(out=fb)
    img = np.ascontiguousarray(np.transpose(fb.cpu().numpy()[::-1], (1, 0, 2))).astype(np.float64)
    assert np.isfinite(img).all(), "pixels left unwritten"
    s = assert_parity(img, oracle_render(name, res, **edits), name)
    assert s["frac_diff"] == 0.0, s


@pytest.mark.parametrize("name,res,edits,rows", [
    ("DepthOfField", (3840, 2160), {"AA": {"jitter": True, "samples": 2}}, (1000, 40)),
    ("DepthOfField", (97, 61), {"AA": {"jitter": True, "samples": 3}}, (0, 61)),
    ("MotionBlur", (75, 64), {}, (0, 64)),
    ("NovelScene1", (256, 128), {"AA": {"jitter": True, "samples": 2}}, (0, 128)),
    ("NovelScene2", (128, 64), {}, (17, 20)),
    ("TwoSpheresPlane", (160, 90), {"AA": {"jitter": True, "samples": 5}}, (3, 80)),
])
def test_sample_parallel_equals_pixel_mapping(name, res, edits, rows, monkeypatch):
    """Both mappings on the production (Philox) jitter: identical framebuffers (bitwise)
    and ray counters, on row blocks that start mid-frame."""
    monkeypatch.setattr(OPTS, "split", "0")  # hierarchy scenes: the one-kernel form's two mappings
    sc = product_scene(name, res, **edits)
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setattr(OPTS, "spp", mode)
        cnt = torch.zeros(16, dtype=torch.int64, device="cuda")
        fb = torch.full((rows[1], res[0], 3), float("nan"), dtype=torch.float32, device="cuda")
        out[mode] = (sc.render_device(row0=rows[0], nrows=rows[1], out=fb, counters=cnt), cnt)
    assert torch.equal(out["0"][0], out["1"][0])
    assert torch.equal(out["0"][1], out["1"][1])


@pytest.mark.parametrize("name,res,edits", [
    ("MirrorRefraction", (160, 181), {}),
    ("DepthOfField", (96, 77), {"AA": {"jitter": True, "samples": 2}}),
    ("NovelScene1", (64, 45), {"AA": {"jitter": True, "samples": 2}}),
    ("TorusMesh", (64, 64), {}),
])
def test_interleaved_row_groups_equal_full_frame(name, res, edits):
    """rtx_render_groups (multi-GPU load balance): each rank's packed 8-row groups are
    exactly the full frame's rows group_rows(H, n, k), for tile and sample-parallel kernels."""
    from rtx.scene import group_rows
    sc = product_scene(name, res, **edits)
    full = sc.render_device().clone()
    H = res[1]
    for n in (2, 3, 8):
        for k in range(n):
            rows = group_rows(H, n, k)
            fb = torch.full((len(rows), res[0], 3), float("nan"), dtype=torch.float32, device="cuda")
            got = sc.render_device(groups=(k, n), out=fb)
            assert torch.equal(got, full[torch.as_tensor(rows, device="cuda")]), (n, k)


@pytest.mark.parametrize("name,res,edits", [
    ("TwoSpheresPlane", (160, 90), {}), ("MirrorRefraction", (97, 61), {}), ("TorusMesh", (96, 96), {}),
    ("DepthOfField", (64, 48), {"AA": {"jitter": True, "samples": 2}}),
    ("NovelScene1", (64, 32), {"AA": {"jitter": True, "samples": 2}}),
])
def test_fused_rgb8_equals_render_then_convert(name, res, edits):
    """rtx_render_rgb8 / rtx_render_groups_rgb8 (main.py's uint8 conversion fused into the
    scene-specialized kernel; hierarchy/texture scenes stage through fp32 + k_to_rgb8) give
    the bytes of rtx_render followed by rtx_fb_to_rgb8, for row blocks and row groups."""
    from rtx.scene import fb_to_rgb8, group_rows
    sc = product_scene(name, res, **edits)
    W, H = res
    full = sc.render_device().clone()
    want = fb_to_rgb8(full)
    got = sc.render_device(rgb8=True)
    assert got.dtype == torch.uint8 and torch.equal(got, want)
    flat = name != "NovelScene1"
    kern = sc.last_kernel.replace("+tiles", "")  # (the measured tile schedule's mark)
    assert kern.endswith("_rgb8") if flat else kern.endswith("+k_to_rgb8"), sc.last_kernel
    part = torch.full((20, W, 3), 7, dtype=torch.uint8, device="cuda")
    assert torch.equal(sc.render_device(row0=H - 20, nrows=20, out=part), want[H - 20:])
    for n in (2, 3):
        for k in range(n):
            rows = torch.as_tensor(group_rows(H, n, k), device="cuda")
            assert torch.equal(sc.render_device(groups=(k, n), rgb8=True), want[rows]), (n, k)
    assert np.array_equal(sc.render_rgb8(), want.cpu().numpy())


def test_rgb8_conversion_unaligned_and_tails():
    """rtx_fb_to_rgb8's vector kernel (16-byte fp32 loads) and its unaligned / tail paths."""
    import ctypes as C
    from rtx import _native as N
    g = torch.Generator(device="cpu").manual_seed(3)
    base = torch.rand(3 * 1001 + 1, generator=g, dtype=torch.float32)
    base[:7] = torch.tensor([0.0, 1.0, 0.999999, 1.0 / 255, 2.0 / 255, 0.5, 254.5 / 255])
    for off, n in ((0, 3003), (1, 3000), (0, 3001), (2, 7)):
        src = base[off:off + n].contiguous() if off == 0 else base.cuda()[off:off + n]
        fb = src.cuda() if not src.is_cuda else src
        out = torch.empty(n, dtype=torch.uint8, device="cuda")
        N.call("rtx_fb_to_rgb8", C.c_void_p(fb.data_ptr()), C.c_void_p(out.data_ptr()), n,
               C.c_void_p(torch.cuda.current_stream().cuda_stream))
        want = (fb.cpu().numpy().astype(np.float64) * 255.0).astype(np.uint8)
        assert np.array_equal(out.cpu().numpy(), want), (off, n)


@pytest.mark.parametrize("seed", range(16))
def test_primary_bins_equal_walk(seed, monkeypatch):
    """Primary-ray bins (a tile's primary rays test only the objects / faces its bin lists)
    change no pixel: binned == full walk == oracle, whole frames, 8-row groups and row
    blocks that start off the 8-row grid (which walk everything)."""
    from common import oracle_render_dict, product_scene_dict
    from scenegen import bins_scene
    d = bins_scene(seed, res=(97, 61))
    on = product_scene_dict(d)
    a = on.render_device().clone()
    monkeypatch.setattr(OPTS, "bins", "0")
    off = product_scene_dict(d)  # RTX_BINS is read when the camera is uploaded
    b = off.render_device().clone()
    monkeypatch.setattr(OPTS, "bins", "1")
    assert torch.equal(a, b)
    img = np.ascontiguousarray(np.transpose(a.cpu().numpy()[::-1], (1, 0, 2))).astype(np.float64)
    assert_parity(img, oracle_render_dict(d), "bins seed %d" % seed)
    from rtx.scene import group_rows
    for n in (3,):
        for k in range(n):
            rows = torch.as_tensor(group_rows(61, n, k), device="cuda")
            assert torch.equal(on.render_device(groups=(k, n)), a[rows])
    assert torch.equal(on.render_device(row0=13, nrows=30), a[13:43])


@pytest.mark.parametrize("seed", range(16))
def test_lens_bins_equal_walk(seed, monkeypatch):
    """Lens cameras' thick primary-ray bins (rtx_api.hip primary_bins: DOF samples, AA
    spreads, Philox jitter) change no pixel: binned == walk on 160x96 frames, == the oracle
    (restated Philox stream) on every fourth."""
    from common import oracle_render_dict, product_scene_dict
    from scenegen import bins_scene
    d = bins_scene(seed, res=(160, 96), lens=True)
    on = product_scene_dict(d)
    a = on.render_device().clone()
    monkeypatch.setattr(OPTS, "bins", "0")
    b = product_scene_dict(d).render_device().clone()
    monkeypatch.setattr(OPTS, "bins", "1")
    assert torch.equal(a, b)
    if seed % 4 == 0:
        img = np.ascontiguousarray(np.transpose(a.cpu().numpy()[::-1], (1, 0, 2))).astype(np.float64)
        noise = _philox_noise(on, 0, 160) if on.jitter else None
        assert_parity(img, oracle_render_dict(d, noise=noise), "lens bins seed %d" % seed)


def test_lens_bins_config5_full_frame(monkeypatch):
    """BASELINE config 5 (DepthOfField 3840x2160, AA 2 x DOF 32, Philox jitter) with its
    thick bins and without (RTX_LENS_BINS=0): the same 8.3 M pixels, bit for bit."""
    edits = {"AA": {"jitter": True, "samples": 2}}
    res = (3840, 2160)
    a = product_scene("DepthOfField", res, **edits).render_device().clone()
    monkeypatch.setattr(OPTS, "lens_bins", "0")
    b = product_scene("DepthOfField", res, **edits).render_device().clone()
    torch.cuda.synchronize()
    assert torch.equal(a, b), float((a != b).float().mean())


@pytest.mark.parametrize("seed", range(12))
def test_dir_shadow_grids_equal_walk(seed, monkeypatch):
    """Directional lights' shadow grids (a shadow ray tests only the spheres and boxes its
    origin's cell lists; rtx_api.hip dir_shadow_grids) change no pixel: grid == every
    object (RTX_DSGRID=0) == oracle, 160x120 frames."""
    from common import oracle_render_dict, product_scene_dict
    from scenegen import shadow_scene
    monkeypatch.setattr(OPTS, "dsgrid_min", "1")  # a grid for every scene, however few its spheres
    d = shadow_scene(seed, res=(160, 120))
    a = product_scene_dict(d).render_device().clone()
    monkeypatch.setattr(OPTS, "dsgrid", "0")
    b = product_scene_dict(d).render_device().clone()
    monkeypatch.setattr(OPTS, "dsgrid", "1")
    assert torch.equal(a, b)
    img = np.ascontiguousarray(np.transpose(a.cpu().numpy()[::-1], (1, 0, 2))).astype(np.float64)
    assert_parity(img, oracle_render_dict(d), "shadow grids seed %d" % seed)


@pytest.mark.parametrize("name,res,edits", [("DepthOfField", (3840, 2160), {"AA": {"jitter": True, "samples": 2}}),
                                            ("MirrorRefraction", (1920, 1080), {})])
def test_dir_shadow_grids_full_frames(name, res, edits, monkeypatch):
    """The BASELINE configs with directional lights, with their shadow grids and without:
    the same frames, bit for bit (MirrorRefraction's four spheres get a grid only when
    RTX_DSGRID_MIN allows it)."""
    monkeypatch.setattr(OPTS, "dsgrid_min", "1")
    a = product_scene(name, res, **edits).render_device().clone()
    monkeypatch.setattr(OPTS, "dsgrid", "0")
    b = product_scene(name, res, **edits).render_device().clone()
    torch.cuda.synchronize()
    assert torch.equal(a, b), float((a != b).float().mean())


@pytest.mark.parametrize("name,res,edits", [("DepthOfField", (3840, 2160), {"AA": {"jitter": True, "samples": 2}}),
                                            ("TwoSpheresPlane", (1920, 1080), {}), ("TorusMesh", (1920, 1080), {})])
def test_self_skip_full_frames(name, res, edits, monkeypatch):
    """The plane and box self-test skips (a camera ray's hit skips its own
    object's shadow test where a rounding bound proves it cannot pass) on and off (option
    self_skip): the same BASELINE-config frames, bit for bit."""
    a = product_scene(name, res, **edits).render_device().clone()
    monkeypatch.setattr(OPTS, "self_skip", "0")
    b = product_scene(name, res, **edits).render_device().clone()
    torch.cuda.synchronize()
    assert torch.equal(a, b), float((a != b).float().mean())


@pytest.mark.parametrize("case", ["blob", "blob_walk", "random0", "random3", "random6", "bins0", "bins5", "bins8"])
def test_wave_cooperative_mesh_matches_oracle(case, tmp_path, monkeypatch):
    """The wave-cooperative mesh variant (experiment -DRTX_WCOOP=1, off by default; DESIGN
    §6e) is exact too: RTX_WCOOP_MIN=1 puts every mesh on it -- the 81,920-face blob with
    its primary-ray bins and with the BVH walk, and random scenes whose reflected and
    refracted rays reach the meshes from a subset of a wave's lanes, ragged tiles included."""
    from common import oracle_render_dict, product_scene_dict
    from scenegen import blob_obj, blob_scene, bins_scene, random_scene
    monkeypatch.setattr(OPTS, "jit_flags", "-DRTX_WCOOP=1 -DRTX_WCOOP_MIN=1")
    if case.startswith("blob"):
        p = str(tmp_path / "blob6.obj")
        blob_obj(p, level=6)
        d = blob_scene(p, (64, 64))
        if case == "blob_walk":
            monkeypatch.setattr(OPTS, "bins", "0")
    elif case.startswith("bins"):
        d = bins_scene(int(case[4:]), res=(97, 61))
    else:
        d = random_scene(int(case[6:]), res=(64, 48), mesh=True)
    sc = product_scene_dict(d)
    img = sc.render()
    assert sc.last_kernel.startswith("rtx_jit_render_1"), sc.last_kernel
    assert_parity(img, oracle_render_dict(d), case)


@pytest.mark.parametrize("case", ["TorusMesh", "blob", "random0", "random3", "bins5", "bins8"])
def test_light_grids_equal_walk(case, tmp_path, monkeypatch):
    """Light grids (a point light's shadow rays test only the mesh faces listed in the cell
    of their direction from the light; rtx_api.hip light_grids) change no pixel: grid ==
    BVH walk (RTX_LGRID=0) == oracle."""
    from common import oracle_render_dict, product_scene_dict
    from scenegen import blob_obj, blob_scene, bins_scene, random_scene
    from rtx.io import bundled_scene_dict
    if case == "TorusMesh":
        d = bundled_scene_dict("TorusMesh", resolution=(160, 120))
    elif case == "blob":
        p = str(tmp_path / "blob6.obj")
        blob_obj(p, level=6)
        d = blob_scene(p, (64, 64))
    elif case.startswith("bins"):
        d = bins_scene(int(case[4:]), res=(97, 61))
    else:
        d = random_scene(int(case[6:]), res=(64, 48), mesh=True)
    a = product_scene_dict(d).render_device().clone()
    monkeypatch.setattr(OPTS, "lgrid", "0")
    b = product_scene_dict(d).render_device().clone()
    assert torch.equal(a, b)
    img = np.ascontiguousarray(np.transpose(a.cpu().numpy()[::-1], (1, 0, 2))).astype(np.float64)
    assert_parity(img, oracle_render_dict(d), case)


@pytest.mark.gpu
@pytest.mark.parametrize("name,res,edits", [("TwoSpheresPlane", (120, 67), {}), ("MirrorRefraction", (64, 40), {}),
                                            ("TorusMesh", (48, 48), {}), ("NovelScene1", (64, 32), {"AA": {"jitter": False, "samples": 2}})])
@pytest.mark.parametrize("jit", ["1", "0"])
def test_render_frames_equals_per_frame_renders(name, res, edits, jit, monkeypatch):
    """rtx_render_frames (one launch, gridDim.y = frames) writes into every slot exactly
    what rtx_render / rtx_render_rgb8 write for the same rows, for the specialized and the
    generic kernels; the slots' padding rows stay untouched."""
    monkeypatch.setattr(OPTS, "jit", jit)
    sc = product_scene(name, res, **edits)
    H, W = res[1], res[0]
    for dtype in (torch.uint8, torch.float32):
        for row0, nrows in ((0, H), (8, H // 3), (3, H // 2 - 1)):
            want = sc.render_device(row0=row0, nrows=nrows, out=torch.empty((nrows, W, 3), dtype=dtype, device="cuda"))
            out = torch.full((3, nrows + 5, W, 3), 7, dtype=dtype, device="cuda")
            sc.render_frames(out, row0=row0, nrows=nrows)
            kern = sc.last_kernel
            for f in range(3):
                assert torch.equal(out[f, :nrows], want), (dtype, row0, nrows, f, kern)
                assert bool((out[f, nrows:] == 7).all())
            assert kern.startswith("rtx_jit_render_") == (jit == "1" and name != "NovelScene1"), kern
        for k, n in ((0, 1), (1, 3), (2, 3)):  # interleaved 8-row groups (rtx_render_groups_frames)
            want = sc.render_device(groups=(k, n), rgb8=dtype == torch.uint8)
            if dtype == torch.float32:
                want = sc.render_device(groups=(k, n))
            out = torch.full((2, want.shape[0] + 3, W, 3), 7, dtype=dtype, device="cuda")
            sc.render_frames(out, groups=(k, n))
            for f in range(2):
                assert torch.equal(out[f, :want.shape[0]], want), (dtype, k, n, f, sc.last_kernel)
                assert bool((out[f, want.shape[0]:] == 7).all())
    # overlapping frames (stride below one frame's bytes) are refused
    import ctypes as C
    from rtx import _native as N
    buf = torch.empty((8, W, 3), dtype=torch.uint8, device="cuda")
    with pytest.raises(N.RtxError):
        N.call("rtx_render_frames", sc._native.h, 0, 4, C.c_void_p(buf.data_ptr()), 1, 2, 4 * W * 3 - 1, None,
               C.c_void_p(torch.cuda.current_stream().cuda_stream))


@pytest.mark.parametrize("seed", range(2))
def test_primary_bins_wide_frame(seed, monkeypatch):
    """Primary-ray bins at 7680 pixels across (the tables, not a spacing estimate, map a
    projected point to its column): binned == walk == oracle on the last column strip."""
    from common import oracle_render_dict, product_scene_dict
    from scenegen import bins_scene
    d = bins_scene(seed, res=(7680, 16))
    a = product_scene_dict(d).render(7, 8)
    monkeypatch.setattr(OPTS, "bins", "0")
    b = product_scene_dict(d).render(7, 8)
    monkeypatch.setattr(OPTS, "bins", "1")
    assert np.array_equal(a, b)
    assert_parity(a, oracle_render_dict(d, 7, 8), "wide bins seed %d" % seed)
