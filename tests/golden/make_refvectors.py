"""Generate tests/golden/refvectors/*.npz: golden input/output vectors produced by the
REFERENCE's own code (provided/scene.py, provided/geometry/*.py), imported as-is.

Runs only in the build container (the reference does not travel to the GPU box): it puts
the test-only PyGLM / libigl stand-ins of tests/refshim first on sys.path (PyGLM and
libigl are not installed in this image; the stand-ins restate GLM 0.9.9's generic code),
then /root/reference/provided, and works from /root/reference (the scene JSON asset paths
are CWD-relative).

Two kinds of fixture:

- render cases (``render_<name>.npz``): ``Scene.render(subimage, tasks)`` of a scene
  dictionary (stored as JSON in the fixture, with asset paths relative to assets/).
  Jittered cases seed ``np.random.seed(seed)`` first and wrap ``np.random.rand`` to count
  the draws (scene.py:63-65); the fixture keeps the seed, the count and a digest of the
  stream, which ``np.random.RandomState(seed).rand(count)`` regenerates. Ray tallies are
  counted by wrapping ``Scene.cast_ray`` (per recursion depth) and
  ``Scene._compute_regular_lighting`` (shade points; one shadow ray per light).
- known-answer vectors (``kat_<name>.npz``): for every top-level object of a scene,
  ``obj.intersect(ray)`` (every hit: time, normal, position, material),
  ``obj.shadow_intersect(ray, t_max)`` and ``obj.is_inside(p)`` on seeded rays and
  points, plus the scene's closest hit ``min(intersections, key=time)`` (scene.py:86-94)
  and any-hit occlusion (scene.py:161-164).

usage: python tests/golden/make_refvectors.py [--jobs 8] [case ...]
"""
import argparse
import contextlib
import copy
import hashlib
import io
import json
import os
import sys
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
TESTS = os.path.dirname(HERE)
REPO = os.path.dirname(TESTS)
REF = "/root/reference"
OUT = os.path.join(HERE, "refvectors")
sys.path.insert(0, TESTS)


# ------------------------------------------------------------------ the cases
def _bundle(name, **edits):
    with open(os.path.join(REPO, "assets", "scenes.json")) as f:
        d = json.load(f)[name]
    d.update(copy.deepcopy(edits))
    return d


def box_stress_scene(res=(64, 48)):
    """Boxes in every role the reference gives them (simple_geometry.py:179-355): diffuse,
    mirror and refractive boxes (refraction with eta > 1 leaving a non-sphere), a moving
    box, a box given by corners with min > max on one axis, textured boxes (every face's
    get_diffuse branch), a box enclosing a point light, coincident faces (tie break), a
    box the camera sits inside and a sphere inside a box."""
    mats = [{"name": "red", "ID": 0, "diffuse": [0.9, 0.2, 0.2], "specular": [0.6, 0.6, 0.6], "hardness": 24},
            {"name": "floor_a", "ID": 1, "diffuse": [0.8, 0.8, 0.8], "specular": [0.1, 0.1, 0.1], "hardness": 4},
            {"name": "floor_b", "ID": 2, "diffuse": [0.2, 0.3, 0.4], "specular": [0.1, 0.1, 0.1]},
            {"name": "mirror", "ID": 3, "type": "mirror", "diffuse": [0.1, 0.1, 0.1], "specular": [1, 1, 1],
             "tint": 0.2},
            {"name": "glass", "ID": 4, "type": "refractive", "diffuse": [0.2, 0.4, 0.2], "specular": [0.9, 0.9, 0.9],
             "hardness": 64, "tint": 0.3, "refr_index": 1.5},
            {"name": "blue", "ID": 5, "diffuse": [0.1, 0.2, 0.9], "specular": [0.3, 0.3, 0.3], "hardness": 0}]
    objs = [{"name": "floor", "type": "plane", "normal": [0.0, 1.0, 0.0], "position": [0.0, -1.0, 0.0],
             "materials": [1, 2]},
            {"name": "glassbox", "type": "box", "position": [-1.2, 0.0, 0.5], "size": [1.0, 2.0, 0.8], "materials": [4]},
            {"name": "mirrorbox", "type": "box", "min": [0.8, -1.0, -2.5], "max": [2.6, 1.6, -2.2], "materials": [3]},
            {"name": "movingbox", "type": "box", "position": [1.3, -0.4, 0.6], "size": [0.7, 0.7, 0.7],
             "speed": [0.2, 0.3, 0.0], "materials": [0]},
            {"name": "swapped", "type": "box", "min": [-2.8, -1.0, -1.5], "max": [-2.0, 0.2, -2.3], "materials": [5]},
            {"name": "tex1", "type": "box", "position": [0.0, -0.5, -1.0], "size": [1.0, 1.0, 1.0],
             "texture": "textures/axes.png", "materials": [0]},
            {"name": "tex2", "type": "box", "min": [2.0, -1.0, 0.8], "max": [3.0, 0.0, 1.8],
             "texture": "textures/brick.jpg", "materials": [5]},
            {"name": "twin", "type": "box", "position": [0.0, -0.5, -1.0], "size": [1.0, 1.0, 1.0], "materials": [5]},
            {"name": "lamp", "type": "box", "position": [-2.0, 3.0, 2.0], "size": [0.6, 0.6, 0.6], "materials": [0]},
            {"name": "ball", "type": "sphere", "position": [-1.2, 0.1, 0.5], "radius": 0.3, "materials": [0]},
            {"name": "far", "type": "box", "position": [0.0, 0.0, -12.0], "size": [30.0, 14.0, 0.5], "materials": [2]}]
    lights = [{"name": "sun", "type": "directional", "direction": [-0.4, -1.0, -0.5], "colour": [1.0, 0.95, 0.9],
               "power": 0.7},
              {"name": "lamp", "type": "point", "position": [-2.0, 3.0, 2.0], "colour": [1.0, 1.0, 1.0], "power": 1.0},
              {"name": "fill", "type": "point", "position": [3.0, 2.0, 4.0], "colour": [0.5, 0.6, 0.9], "power": 0.8}]
    return {"resolution": list(res), "AA": {"jitter": False, "samples": 2}, "ambient": [0.08, 0.08, 0.08],
            "camera": {"position": [0.5, 1.5, 5.5], "lookAt": [0.0, 0.0, -0.5], "up": [0.0, 1.0, 0.0], "fov": 55.0},
            "motion": {"time": 1.0, "samples": 2, "final": 1},
            "materials": mats, "objects": objs, "lights": lights}


def inside_box_scene(res=(32, 24)):
    """The camera inside a box (AABB.intersect rejects start < 0, simple_geometry.py:226):
    the enclosing box is invisible from inside; a refractive box is seen through."""
    d = box_stress_scene(res)
    d["objects"].append({"name": "room", "type": "box", "position": [0.5, 1.5, 5.5], "size": [2.0, 2.0, 2.0],
                         "materials": [0]})
    d["AA"] = {"jitter": False, "samples": 1}
    d.pop("motion")
    return d


def render_cases():
    from scenegen import random_hier_scene, random_scene
    cases = {
        # BASELINE config 5's scene with its AA2 x DOF32 jitter (seeded, replayed)
        "dof_aa2_jitter": dict(scene=_bundle("DepthOfField", resolution=[40, 30], AA={"jitter": True, "samples": 2}),
                               seed=5),
        "dof_strip": dict(scene=_bundle("DepthOfField", resolution=[96, 64], AA={"jitter": True, "samples": 1}),
                          seed=11, subimage=5, tasks=8),
        # BASELINE config 1: TwoSpheresPlane 256x256 1 spp on the reference's CPU path
        "tsp256_config1": dict(scene=_bundle("TwoSpheresPlane", resolution=[256, 256],
                                             AA={"jitter": False, "samples": 1})),
        # BASELINE configs 2-5 at their stated sizes: column strips (np.array_split) of the
        # full frames, the columns crossing the objects
        "config2_tsp1080_cols": dict(scene=_bundle("TwoSpheresPlane", resolution=[1920, 1080],
                                                   AA={"jitter": False, "samples": 1}), subimage=37, tasks=96),
        "config3_tm1080_cols": dict(scene=_bundle("TorusMesh", resolution=[1920, 1080],
                                                  AA={"jitter": False, "samples": 1}), subimage=125, tasks=240),
        "config4_mr1080_cols": dict(scene=_bundle("MirrorRefraction", resolution=[1920, 1080],
                                                  AA={"jitter": False, "samples": 1}), subimage=52, tasks=96),
        "config5_dof4k_col": dict(scene=_bundle("DepthOfField", resolution=[3840, 2160],
                                                AA={"jitter": True, "samples": 2}), seed=29, subimage=3000, tasks=3840),
        "tsp_aa3_jitter": dict(scene=_bundle("TwoSpheresPlane", resolution=[48, 36],
                                             AA={"jitter": True, "samples": 3}), seed=7),
        "motionblur": dict(scene=_bundle("MotionBlur", resolution=[48, 40])),
        "mirror_refraction_jitter": dict(scene=_bundle("MirrorRefraction", resolution=[64, 36],
                                                       AA={"jitter": True, "samples": 2}), seed=13),
        "box_stress": dict(scene=box_stress_scene()),
        "box_inside": dict(scene=inside_box_scene()),
        # NovelScene1/2: hierarchies (CSG), `ref` copies, fallback materials, textures
        "novel1": dict(scene=_bundle("NovelScene1", resolution=[128, 64], AA={"jitter": True, "samples": 2}), seed=17),
        "novel1_strip": dict(scene=_bundle("NovelScene1", resolution=[512, 256], AA={"jitter": False, "samples": 1}),
                             subimage=20, tasks=64),
        "novel2": dict(scene=_bundle("NovelScene2", resolution=[48, 24], AA={"jitter": True, "samples": 2},
                                     DOF={"aperture": 0.1, "focal_length": 10.0, "samples": 3},
                                     motion={"final": 1, "samples": 3, "time": 1.0}), seed=19),
        "torus_smooth_aa2": dict(scene=_bundle("TorusMesh", resolution=[32, 32], AA={"jitter": True, "samples": 2}),
                                 seed=23, smooth=True),
    }
    for k in range(8):
        cases["hier_rand%d" % k] = dict(scene=random_hier_scene(k, res=(32, 24), mesh=(k % 4 == 3)))
    for k in range(4):
        cases["rand%d" % k] = dict(scene=random_scene(100 + k, res=(32, 24), mesh=(k % 2 == 1)))
    for c in cases.values():
        if c.pop("smooth", False):
            for g in c["scene"]["objects"]:
                if g["type"] == "mesh":
                    g["flat_shaded"] = False
    return cases


def kat_cases():
    from scenegen import random_hier_scene
    return {
        "dof": dict(scene=_bundle("DepthOfField"), n=3000, times=(0.0,)),
        "box_stress": dict(scene=box_stress_scene(), n=2500, times=(0.0, 0.5, 1.0)),
        "novel1": dict(scene=_bundle("NovelScene1"), n=1500, times=(0.0,)),
        "novel2": dict(scene=_bundle("NovelScene2"), n=1200, times=(0.0, 0.6)),
        "hier_rand0": dict(scene=random_hier_scene(0), n=1500, times=(0.0, 0.5)),
        "hier_rand1": dict(scene=random_hier_scene(1), n=1500, times=(0.0,)),
        "hier_rand3": dict(scene=random_hier_scene(3, mesh=True), n=800, times=(0.0,)),
        "torus": dict(scene=_bundle("TorusMesh"), n=1500, times=(0.0,)),
    }


# ------------------------------------------------------------------ reference harness
_ref = {}


def _init_reference():
    """Import the reference as-is (stand-ins first), once per worker process."""
    if _ref:
        return _ref
    os.environ["TQDM_DISABLE"] = "1"
    sys.path[:0] = [os.path.join(TESTS, "refshim"), os.path.join(REF, "provided")]
    os.chdir(REF)
    import numpy.random  # noqa: F401
    import geometry
    import scene as ref_scene
    import scene_parser
    _ref.update(scene_parser=scene_parser, scene=ref_scene, geometry=geometry)
    return _ref


def _to_reference_paths(d):
    """Asset paths as the reference resolves them from /root/reference."""
    d = copy.deepcopy(d)

    def fix(objs):
        for g in objs:
            if g.get("type") == "mesh" and g.get("filepath") == "torus_mesh.obj":
                g["filepath"] = "meshes/torus.obj"
            fix(g.get("children", []))
    fix(d.get("objects", []))
    return d


def _load(d):
    r = _init_reference()
    with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as t:
        json.dump(_to_reference_paths(d), t)
    try:
        with contextlib.redirect_stdout(io.StringIO()):  # the parser prints its defaults
            return r["scene_parser"].load_scene(t.name)
    finally:
        os.unlink(t.name)


def _run_render(name, case):
    r = _init_reference()
    sc = _load(case["scene"])
    Scene = r["scene"].Scene
    tallies = np.zeros(13, np.int64)
    orig_cast, orig_light = Scene.cast_ray, Scene._compute_regular_lighting

    def cast_ray(self, ray, max_recursion=10, in_shape=False):
        if max_recursion > 0:
            tallies[10 - max_recursion] += 1
        return orig_cast(self, ray, max_recursion, in_shape)

    def lighting(self, ray, intersection):
        tallies[12] += 1
        tallies[11] += len(self.lights)
        return orig_light(self, ray, intersection)

    draws = []
    orig_rand = np.random.rand

    def rand(*a):
        v = orig_rand(*a)
        draws.append(v)
        return v

    seed = case.get("seed")
    Scene.cast_ray, Scene._compute_regular_lighting = cast_ray, lighting
    np.random.rand = rand
    try:
        if seed is not None:
            np.random.seed(seed)
        t0 = time.time()
        img = sc.render(case.get("subimage", 0), case.get("tasks", 1))
        dt = time.time() - t0
    finally:
        Scene.cast_ray, Scene._compute_regular_lighting = orig_cast, orig_light
        np.random.rand = orig_rand
    stream = np.asarray(draws, np.float64)
    if seed is not None:
        assert np.array_equal(stream, np.random.RandomState(seed).rand(stream.size)), "np.random stream not replayable"
    out = dict(scene_json=json.dumps(case["scene"], sort_keys=True), image=np.asarray(img, np.float64),
               subimage=case.get("subimage", 0), tasks=case.get("tasks", 1), tallies=tallies,
               noise_seed=-1 if seed is None else seed, noise_count=stream.size,
               noise_digest=hashlib.sha256(stream.tobytes()).hexdigest())
    np.savez_compressed(os.path.join(OUT, "render_%s.npz" % name), **out)
    return "render_%s %s %.1fs" % (name, img.shape, dt)


def _kat_rays(d, n, rng):
    """Seeded rays and points around the scene: camera rays toward the look-at region,
    random origins and directions (some axis components exactly 0), rays aimed at the
    faces, edges and corners of every top-level box, and rays aimed at every node."""
    from scenegen import bv_stress_rays
    cam = np.array(d["camera"]["position"], np.float64)
    look = np.array(d["camera"]["lookAt"], np.float64)
    k = n // 3
    tgt = look + rng.uniform(-3, 3, (k, 3))
    o1, d1 = np.repeat(cam[None], k, 0), tgt - cam
    o2 = look + rng.uniform(-4, 4, (k, 3))
    d2 = rng.normal(size=(k, 3))
    d2[rng.rand(k, 3) < 0.1] = 0.0
    d2[np.all(d2 == 0, axis=1), 0] = 1.0
    os_, ds_ = [o1, o2], [d1, d2]
    boxes = [g for g in d["objects"] if g["type"] == "box"]
    nodes = [g for g in d["objects"] if g["type"] == "node"]
    rest = n - 2 * k
    per = max(1, rest // max(1, len(boxes) + len(nodes)))
    for i, b in enumerate(boxes):
        if "size" in b:
            c, s = np.float32(b.get("position", [0, 0, 0])), np.float32(b["size"])
            lo, hi = c - s / np.float32(2), c + s / np.float32(2)
        else:
            lo, hi = np.float32(b["min"]), np.float32(b["max"])
        o, dd = bv_stress_rays(np.minimum(lo, hi), np.maximum(lo, hi), per, int(rng.randint(1 << 30)))
        os_.append(o)
        ds_.append(dd)
    for g in nodes:
        p = np.array(g.get("position", [0, 0, 0]), np.float64)
        t = p + rng.uniform(-1.5, 1.5, (per, 3))
        o = t + rng.normal(size=(per, 3)) * rng.uniform(1, 8, (per, 1))
        os_.append(o)
        ds_.append(t - o)
    o = np.concatenate(os_).astype(np.float32)
    dd = np.concatenate(ds_).astype(np.float32)
    tmax = np.where(rng.rand(len(o)) < 0.4, 1.0, np.where(rng.rand(len(o)) < 0.5, np.inf, rng.uniform(0, 4, len(o))))
    return o, dd, tmax


def _run_kat(name, case):
    _init_reference()
    import glm
    d = case["scene"]
    sc = _load(d)
    rng = np.random.RandomState(1234 + sum(map(ord, name)))
    o, dd, tmax = _kat_rays(d, case["n"], rng)
    mats = sc.materials

    def mat_index(m):
        """Index in Scene.materials; `ref` copies of a hierarchy carry deep copies of the
        materials (scene_parser.py:199), found by their ID."""
        for i, x in enumerate(mats):
            if x is m:
                return i
        for i, x in enumerate(mats):
            if m is not None and x.ID == m.ID:
                return i
        return -1
    out = dict(scene_json=json.dumps(d, sort_keys=True), o=o, d=dd, tmax=tmax,
               times=np.asarray(case["times"], np.float64), nobj=len(sc.objects))
    t0 = time.time()
    for ti, tm in enumerate(case["times"]):
        sc.current_time = tm
        for g in sc.objects:
            g.set_scene(sc)
        hits = [[] for _ in sc.objects]          # per object, per ray: list of hits
        all_hits = []
        pts = []
        for i in range(len(o)):
            ray = _ray(o[i], dd[i])
            per_ray = []
            for k, g in enumerate(sc.objects):
                hs = g.intersect(ray)
                hits[k].append(hs)
                per_ray += [(h, k) for h in hs]
            all_hits.append(per_ray)
            for h, _ in per_ray[:2]:
                pts.append(np.asarray(h.position.a, np.float32))
        pts = np.array(pts + [np.asarray(x, np.float32) for x in
                              (np.array(d["camera"]["lookAt"]) + rng.uniform(-3, 3, (len(o), 3)))], np.float32)
        for k, g in enumerate(sc.objects):
            off, ht, hn, hp, hm = [0], [], [], [], []
            for hs in hits[k]:
                for h in hs:
                    ht.append(float(h.time))
                    hn.append(np.asarray(h.normal.a, np.float32))
                    hp.append(np.asarray(h.position.a, np.float32))
                    hm.append(mat_index(h.mat))
                off.append(len(ht))
            out["t%d_obj%d_off" % (ti, k)] = np.asarray(off, np.int64)
            out["t%d_obj%d_t" % (ti, k)] = np.asarray(ht, np.float64)
            out["t%d_obj%d_normal" % (ti, k)] = np.asarray(hn, np.float32).reshape(-1, 3)
            out["t%d_obj%d_position" % (ti, k)] = np.asarray(hp, np.float32).reshape(-1, 3)
            out["t%d_obj%d_mat" % (ti, k)] = np.asarray(hm, np.int32)
            out["t%d_obj%d_shadow" % (ti, k)] = np.array(
                [bool(g.shadow_intersect(_ray(o[i], dd[i]), float(tmax[i]))) for i in range(len(o))])
            out["t%d_obj%d_inside" % (ti, k)] = np.array([bool(g.is_inside(glm.vec3(*p))) for p in pts])
        # the scene: min(intersections, key=time) over objects in order; any-hit shadow
        ct, co, cm = np.full(len(o), np.inf), np.full(len(o), -1, np.int32), np.full(len(o), -1, np.int32)
        cn, cp = np.zeros((len(o), 3), np.float32), np.zeros((len(o), 3), np.float32)
        for i, per_ray in enumerate(all_hits):
            if per_ray:
                h, k = min(per_ray, key=lambda x: x[0].time)
                ct[i], co[i], cm[i] = h.time, k, mat_index(h.mat)
                cn[i], cp[i] = h.normal.a, h.position.a
        out["t%d_closest_t" % ti], out["t%d_closest_obj" % ti], out["t%d_closest_mat" % ti] = ct, co, cm
        out["t%d_closest_normal" % ti], out["t%d_closest_position" % ti] = cn, cp
        out["t%d_occluded" % ti] = np.array([any(out["t%d_obj%d_shadow" % (ti, k)][i] for k in range(len(sc.objects)))
                                             for i in range(len(o))])
        out["t%d_points" % ti] = pts
    np.savez_compressed(os.path.join(OUT, "kat_%s.npz" % name), **out)
    return "kat_%s %d rays %.1fs" % (name, len(o), time.time() - t0)


def _ray(o, d):
    import glm
    import helperclasses as hc
    return hc.Ray(glm.vec3(*[float(x) for x in o]), glm.vec3(*[float(x) for x in d]))


def _job(args):
    kind, name, case = args
    try:
        with contextlib.redirect_stdout(io.StringIO()):  # "Ray direction is zero" (simple_geometry.py:26-27)
            return (_run_render if kind == "render" else _run_kat)(name, case)
    except Exception as e:  # report and keep the other cases going
        import traceback
        return "FAILED %s_%s: %r\n%s" % (kind, name, e, traceback.format_exc())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=8)
    ap.add_argument("cases", nargs="*")
    a = ap.parse_args()
    os.makedirs(OUT, exist_ok=True)
    jobs = [("render", k, v) for k, v in render_cases().items()] + [("kat", k, v) for k, v in kat_cases().items()]
    if a.cases:
        jobs = [j for j in jobs if "%s_%s" % (j[0], j[1]) in a.cases]
    from multiprocessing import Pool
    with Pool(a.jobs) as pool:
        for msg in pool.imap_unordered(_job, jobs):
            print(msg, flush=True)


if __name__ == "__main__":
    main()
