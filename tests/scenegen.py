"""Random scene dictionaries (reference JSON schema) for parity fuzzing."""
import numpy as np


def random_scene(seed, res=(48, 36), mesh=False):
    rng = np.random.RandomState(seed)
    r = lambda lo, hi, n=None: np.round(rng.uniform(lo, hi, n), 3).tolist()  # noqa: E731
    mats = []
    for i in range(5):
        t = rng.choice(["diffuse", "diffuse", "mirror", "refractive"])
        m = {"name": "m%d" % i, "ID": 10 + i, "type": str(t), "diffuse": r(0, 1, 3), "specular": r(0, 1, 3)}
        h = rng.choice([0, 1, 16, 32, 50, 7.5])
        m["hardness"] = float(h) if h == 7.5 else int(h)
        if t != "diffuse":
            m["tint"] = float(rng.choice([0.0, 0.3, 0.5]))
        if t == "refractive":
            m["refr_index"] = float(rng.choice([1.2, 1.458, 1.8]))
        mats.append(m)
    ids = [m["ID"] for m in mats]
    objs = [{"name": "ground", "type": "plane", "normal": [0.0, 1.0, 0.0], "position": [0.0, float(r(-1.2, -0.8)), 0.0],
             "materials": [int(rng.choice(ids)), int(rng.choice(ids))]}]
    if rng.rand() < 0.5:
        objs.append({"name": "wall", "type": "plane", "normal": r(-1, 1, 3), "position": r(-3, 3, 3),
                     "materials": [int(rng.choice(ids))]})
    for k in range(rng.randint(1, 4)):
        o = {"name": "s%d" % k, "type": "sphere", "radius": float(r(0.3, 1.2)), "position": r(-2, 2, 3),
             "materials": [int(rng.choice(ids))]}
        if rng.rand() < 0.3:
            o["speed"] = r(-0.5, 0.5, 3)
        objs.append(o)
    for k in range(rng.randint(0, 3)):
        o = {"name": "b%d" % k, "type": "box", "position": r(-2, 2, 3), "size": r(0.3, 1.5, 3),
             "materials": [int(rng.choice(ids))]}
        if rng.rand() < 0.4:  # given by corners, some axes with min > max (NovelScene2's trails)
            c, sz = np.array(o.pop("position")), np.array(o.pop("size"))
            mn, mx = c - sz / 2, c + sz / 2
            sw = rng.rand(3) < 0.4
            mn[sw], mx[sw] = mx[sw].copy(), mn[sw].copy()
            o["min"], o["max"] = np.round(mn, 3).tolist(), np.round(mx, 3).tolist()
        if rng.rand() < 0.3:
            o["speed"] = r(-0.5, 0.5, 3)
        objs.append(o)
    if mesh:
        objs.append({"name": "torus", "type": "mesh", "filepath": "torus_mesh.obj", "scale": float(r(0.5, 1.2)),
                     "position": r(-1, 1, 3), "materials": [int(rng.choice(ids))],
                     "flat_shaded": bool(rng.rand() < 0.5)})
    order = rng.permutation(len(objs))
    objs = [objs[i] for i in order]
    lights = [{"name": "p", "type": "point", "position": r(-5, 5, 3), "colour": r(0.3, 1, 3), "power": float(r(0.3, 1.5))}]
    if rng.rand() < 0.7:
        lights.append({"name": "d", "type": "directional", "direction": r(-1, 1, 3), "colour": r(0.3, 1, 3), "power": 1.0})
    sc = {"resolution": list(res), "AA": {"jitter": False, "samples": int(rng.choice([1, 2, 3]))},
          "ambient": r(0, 0.2, 3),
          "camera": {"position": [float(r(-1, 1)), float(r(1, 3)), float(r(5, 7))], "lookAt": [0.0, 0.5, 0.0],
                     "up": [0.0, 1.0, 0.0], "fov": float(r(40, 60))},
          "materials": mats, "objects": objs, "lights": lights}
    if rng.rand() < 0.3:
        sc["DOF"] = {"focal_length": float(r(3, 6)), "aperture": float(r(0.05, 0.2)), "samples": 3}
    if rng.rand() < 0.3:
        sc["motion"] = {"time": 1.0, "samples": 3, "final": 1}
    return sc


def point_lights_scene(seed, res=(64, 48)):
    """Flat scenes of planes and spheres under two to eight point lights only -- the
    specialized kernels' all-lights-at-once shadow test (rtx_trace.h occluded_points):
    lights above and below the ground, inside and next to spheres, on a wall's plane
    (grazing shadow rays), mirrors and refraction so secondary hits shade too."""
    rng = np.random.RandomState(9000 + seed)
    r = lambda lo, hi, n=None: np.round(rng.uniform(lo, hi, n), 3).tolist()  # noqa: E731
    mats = [{"name": "m%d" % i, "ID": i, "diffuse": r(0, 1, 3), "specular": r(0, 1, 3),
             "hardness": int(rng.choice([0, 16, 50])), "type": t, "tint": 0.3, "refr_index": 1.3}
            for i, t in enumerate(["diffuse", "diffuse", "mirror", "refractive"])]
    objs = [{"name": "ground", "type": "plane", "normal": [0.0, 1.0, 0.0], "position": [0.0, -1.0, 0.0],
             "materials": [0, 1]}]
    for k in range(rng.randint(0, 4)):
        objs.append({"name": "w%d" % k, "type": "plane", "normal": r(-1, 1, 3), "position": r(-4, 4, 3),
                     "materials": [int(rng.randint(4))]})
    spheres = []
    for k in range(rng.randint(1, 7)):
        o = {"name": "s%d" % k, "type": "sphere", "radius": float(r(0.1, 1.2)), "position": r(-2.5, 2.5, 3),
             "materials": [int(rng.randint(4))]}
        if rng.rand() < 0.2:
            o["speed"] = r(-0.5, 0.5, 3)
        spheres.append(o)
        objs.append(o)
    lights = []
    for i in range(rng.randint(2, 9)):
        u = rng.rand()
        if u < 0.15:  # inside a sphere
            pos = list(spheres[int(rng.randint(len(spheres)))]["position"])
        elif u < 0.3:  # under the ground
            pos = [float(r(-3, 3)), float(r(-4, -1.5)), float(r(-3, 3))]
        elif u < 0.4:  # on the ground's plane: grazing shadow rays
            pos = [float(r(-3, 3)), -1.0, float(r(-3, 3))]
        else:
            pos = r(-6, 6, 3)
        lights.append({"name": "p%d" % i, "type": "point", "position": pos, "colour": r(0.2, 1, 3),
                       "power": float(r(0.2, 1.0))})
    order = rng.permutation(len(objs))
    sc = {"resolution": list(res), "AA": {"jitter": False, "samples": int(rng.choice([1, 2]))},
          "ambient": [0.1, 0.1, 0.1],
          "camera": {"position": [float(r(-2, 2)), float(r(1, 4)), float(r(6, 9))], "lookAt": [0.0, 0.0, 0.0],
                     "up": [0.0, 1.0, 0.0], "fov": float(rng.choice([45.0, 70.0]))},
          "materials": mats, "objects": [objs[i] for i in order], "lights": lights}
    if rng.rand() < 0.25:
        sc["motion"] = {"time": 1.0, "samples": 2, "final": 1}
    return sc


def shadow_scene(seed, res=(40, 30)):
    """Scenes for the directional lights' shadow grids (rtx_api.hip dir_shadow_grids):
    spheres from tiny to large, near and far, boxes (some given by swapped corners), some
    moving, under one to three directional lights -- axis-aligned, diagonal, grazing and
    random directions."""
    rng = np.random.RandomState(7000 + seed)
    r = lambda lo, hi, n=None: np.round(rng.uniform(lo, hi, n), 3).tolist()  # noqa: E731
    mats = [{"name": "m%d" % i, "ID": i, "diffuse": r(0, 1, 3), "specular": r(0, 1, 3), "hardness": 16,
             "type": "mirror" if i == 3 else "diffuse", "tint": 0.3} for i in range(4)]
    objs = [{"name": "ground", "type": "plane", "normal": [0.0, 1.0, 0.0], "position": [0.0, -1.0, 0.0],
             "materials": [0, 1]}]
    for k in range(rng.randint(2, 9)):
        far = rng.rand() < 0.15
        o = {"name": "s%d" % k, "type": "sphere", "radius": float(r(0.02, 0.3) if rng.rand() < 0.3 else r(0.3, 1.5)),
             "position": r(-40, 40, 3) if far else r(-4, 4, 3), "materials": [int(rng.randint(4))]}
        if rng.rand() < 0.15:
            o["speed"] = r(-0.5, 0.5, 3)
        objs.append(o)
    for k in range(rng.randint(0, 5)):
        o = {"name": "b%d" % k, "type": "box", "position": r(-4, 4, 3), "size": r(0.1, 2.5, 3),
             "materials": [int(rng.randint(4))]}
        if rng.rand() < 0.3:
            c, sz = np.array(o.pop("position")), np.array(o.pop("size"))
            mn, mx = c - sz / 2, c + sz / 2
            sw = rng.rand(3) < 0.4
            mn[sw], mx[sw] = mx[sw].copy(), mn[sw].copy()
            o["min"], o["max"] = np.round(mn, 3).tolist(), np.round(mx, 3).tolist()
        if rng.rand() < 0.15:
            o["speed"] = r(-0.5, 0.5, 3)
        objs.append(o)
    dirs = [[0.0, -1.0, 0.0], [1.0, -1.0, -1.0], [-1.0, 0.0, -1.0], [1.0, -0.01, 0.3], r(-1, 1, 3), r(-1, 1, 3)]
    lights = [{"name": "d%d" % i, "type": "directional", "direction": dirs[int(j)], "colour": r(0.3, 1, 3),
               "power": 0.7} for i, j in enumerate(rng.choice(len(dirs), rng.randint(1, 4), replace=False))]
    if rng.rand() < 0.3:
        lights.append({"name": "p", "type": "point", "position": r(-5, 5, 3), "colour": r(0.3, 1, 3), "power": 1.0})
    sc = {"resolution": list(res), "AA": {"jitter": False, "samples": 1}, "ambient": [0.1, 0.1, 0.1],
          "camera": {"position": [float(r(-2, 2)), float(r(2, 5)), float(r(7, 10))], "lookAt": [0.0, 0.0, 0.0],
                     "up": [0.0, 1.0, 0.0], "fov": float(rng.choice([45.0, 70.0, 100.0]))},
          "materials": mats, "objects": objs, "lights": lights}
    if rng.rand() < 0.3:
        sc["motion"] = {"time": 1.0, "samples": 2, "final": 1}
    return sc


def many_roots_scene(seed, res=(48, 32), n_roots=40, n_spheres=20):
    """More hierarchy roots than the 32 bits of a bin or shadow-grid cell, and more spheres
    than the 16 a mask holds: the ones beyond are tested by every ray. A lens camera with
    AA jitter, a directional and a point light."""
    rng = np.random.RandomState(9000 + seed)
    r = lambda lo, hi, n=None: np.round(rng.uniform(lo, hi, n), 3).tolist()  # noqa: E731
    mats = [{"name": "m%d" % i, "ID": i, "diffuse": r(0, 1, 3), "specular": r(0, 1, 3), "hardness": 16}
            for i in range(3)]
    objs = [{"name": "ground", "type": "plane", "normal": [0.0, 1.0, 0.0], "position": [0.0, -1.0, 0.0],
             "materials": [0, 1]}]
    for k in range(n_roots):
        kids = [{"name": "c%d_%d" % (k, j), "type": "sphere", "radius": float(r(0.1, 0.35)),
                 "position": r(-0.3, 0.3, 3)} for j in range(2)]
        if rng.rand() < 0.3:
            kids.append({"name": "cb%d" % k, "type": "box", "size": r(0.2, 0.5, 3), "position": r(-0.2, 0.2, 3)})
        n = {"name": "n%d" % k, "type": "node", "hierarchy_type": str(rng.choice(["union", "intersection"])),
             "position": r(-5, 5, 3), "materials": [int(rng.randint(3))], "children": kids}
        if rng.rand() < 0.2:
            n["speed"] = r(-0.3, 0.3, 3)
        objs.append(n)
    for k in range(n_spheres):
        objs.append({"name": "s%d" % k, "type": "sphere", "radius": float(r(0.1, 0.5)), "position": r(-5, 5, 3),
                     "materials": [int(rng.randint(3))]})
    order = rng.permutation(len(objs))
    return {"resolution": list(res), "AA": {"jitter": True, "samples": 2}, "ambient": [0.1, 0.1, 0.1],
            "DOF": {"aperture": 0.1, "focal_length": 8.0, "samples": 2},
            "camera": {"position": [0.0, 4.0, 12.0], "lookAt": [0.0, 0.0, 0.0], "up": [0.0, 1.0, 0.0], "fov": 60.0},
            "materials": mats, "objects": [objs[i] for i in order],
            "lights": [{"name": "d", "type": "directional", "direction": [1.0, -1.0, -0.5], "colour": [1.0, 1.0, 1.0],
                        "power": 0.7},
                       {"name": "p", "type": "point", "position": [3.0, 6.0, 4.0], "colour": [1.0, 1.0, 1.0], "power": 0.5}]}


def tie_scene(res=(40, 30), mirror=False):
    """Coincident geometry: the first object in scene order must win closest-hit ties.
    mirror: a mirror sphere that reflects the tied objects (secondary rays meet the ties
    too, and the scene runs the secondary-ray kernels)."""
    sc = _tie_scene(res)
    if mirror:
        sc["materials"].append({"name": "m", "ID": 3, "type": "mirror", "diffuse": [0.2, 0.2, 0.2], "tint": 0.2})
        sc["objects"].append({"name": "mirror", "type": "sphere", "radius": 0.8, "position": [0.0, 1.2, -2.0],
                              "materials": [3]})
    return sc


def _tie_scene(res):
    return {"resolution": list(res), "ambient": [0.1, 0.1, 0.1],
            "camera": {"position": [0.0, 3.0, 6.0], "lookAt": [0.0, 0.0, 0.0], "up": [0.0, 1.0, 0.0], "fov": 50.0},
            "materials": [{"name": "a", "ID": 0, "diffuse": [1, 0, 0], "specular": [0.5, 0.5, 0.5], "hardness": 16},
                          {"name": "b", "ID": 1, "diffuse": [0, 0, 1], "specular": [0.5, 0.5, 0.5], "hardness": 16},
                          {"name": "c", "ID": 2, "diffuse": [0, 1, 0]}],
            "objects": [{"name": "s1", "type": "sphere", "radius": 1.0, "position": [-1.5, 1.0, 0.0], "materials": [1]},
                        {"name": "ground", "type": "plane", "normal": [0, 1, 0], "position": [0, 0, 0], "materials": [2]},
                        {"name": "s0", "type": "sphere", "radius": 1.0, "position": [-1.5, 1.0, 0.0], "materials": [0]},
                        {"name": "box", "type": "box", "min": [0.5, -1.0, -1.0], "max": [2.5, 0.0, 1.0], "materials": [0]},
                        {"name": "box2", "type": "box", "min": [0.5, -1.0, -1.0], "max": [2.5, 0.0, 1.0], "materials": [1]}],
            "lights": [{"name": "l", "type": "point", "position": [2, 5, 3], "colour": [1, 1, 1], "power": 1.0}]}


def random_hier_scene(seed, res=(48, 36), mesh=False):
    """Random hierarchy (CSG) scenes: nested union / intersection / difference / unknown
    nodes with translate-rotate-scale, fallback materials, root and child speeds, a `ref`
    copy, difference nodes with a third (ignored) child, and textured planes and boxes."""
    rng = np.random.RandomState(1000 + seed)
    r = lambda lo, hi, n=None: np.round(rng.uniform(lo, hi, n), 3).tolist()  # noqa: E731
    sc = random_scene(seed, res=res, mesh=False)
    ids = [m["ID"] for m in sc["materials"]]
    tex = ["textures/axes.png", "textures/brick.jpg", "textures/ground.png", "textures/wall2.png"]
    counter = [0]

    def name():
        counter[0] += 1
        return "g%d" % counter[0]

    def leaf(depth):
        k = rng.choice(["sphere", "sphere", "box", "box", "plane"] + (["mesh"] if mesh else []))
        g = {"name": name(), "type": str(k), "position": r(-1, 1, 3)}
        if rng.rand() < 0.7:
            g["materials"] = [int(rng.choice(ids))] + ([int(rng.choice(ids))] if rng.rand() < 0.3 else [])
        if k == "sphere":
            g["radius"] = float(r(0.3, 1.2))
        elif k == "box":
            if rng.rand() < 0.5:
                g["size"] = r(0.4, 1.6, 3)
            else:
                lo = np.array(r(-1, 0, 3))
                g["min"], g["max"] = lo.tolist(), (lo + np.array(r(0.4, 1.5, 3))).round(3).tolist()
            if rng.rand() < 0.3:
                g["texture"] = str(rng.choice(tex))
        elif k == "plane":
            g["normal"] = [[0.0, 1.0, 0.0], [1.0, 0.0, 0.0], [0.0, 0.0, 1.0], r(-1, 1, 3)][rng.randint(4)]
            if rng.rand() < 0.5:
                g["texture"] = str(rng.choice(tex))
                if rng.rand() < 0.7:
                    g["texture_scale"] = float(r(1, 40))
        else:
            g.update({"filepath": "torus_mesh.obj", "scale": float(r(0.3, 0.6)), "flat_shaded": bool(rng.rand() < 0.5)})
        if rng.rand() < 0.2:
            g["speed"] = r(-0.5, 0.5, 3)
        return g

    def node(depth):
        ht = str(rng.choice(["union", "intersection", "difference", "difference", "xor"], p=[0.3, 0.25, 0.2, 0.2, 0.05]))
        n = {"name": name(), "type": "node", "hierarchy_type": ht}
        if rng.rand() < 0.2:
            del n["hierarchy_type"]  # default: union
        if rng.rand() < 0.8:
            n["position"] = r(-1.5, 1.5, 3)
        if rng.rand() < 0.6:
            n["rotation"] = [float(rng.choice([0.0, 15.0, 30.0, 45.0, 90.0, -20.0, 7.5])) for _ in range(3)]
        if rng.rand() < 0.6:
            n["scale"] = r(0.5, 1.6, 3)
        nc = rng.randint(2, 4) if ht == "difference" else rng.randint(1, 4)
        n["children"] = [node(depth + 1) if (depth < 3 and rng.rand() < 0.35) else leaf(depth + 1) for _ in range(nc)]
        return n

    roots = []
    for k in range(rng.randint(1, 4)):
        n = node(0)
        n["materials"] = [int(rng.choice(ids))]
        if rng.rand() < 0.3:
            n["speed"] = r(-0.4, 0.4, 3)
        roots.append(n)
    objs = sc["objects"] + roots
    if rng.rand() < 0.6:
        ref = {"name": "copy", "type": "node", "ref": roots[0]["name"], "position": r(-2, 2, 3),
               "materials": [int(rng.choice(ids))]}
        if rng.rand() < 0.5:
            ref["rotation"] = [0.0, float(rng.choice([30.0, 90.0])), 0.0]
        objs.append(ref)
    if rng.rand() < 0.5:  # a textured ground
        objs[0] = dict(objs[0], texture="textures/ground.png", texture_scale=float(r(1, 8)))
    order = rng.permutation(len(objs))
    sc["objects"] = [objs[i] for i in order]
    # leaves without materials need a root that has some (else the reference raises)
    return sc


def blob_obj(path, level=6, seed=0):
    """A closed, bumpy triangle mesh (icosphere subdivided `level` times, 20 * 4^level
    faces, radially displaced by a few smooth waves) written as OBJ: a stand-in of the
    size of the reference's missing bunny.obj (scenes/TorusMesh.json) for the large-mesh
    path. Deterministic in (level, seed)."""
    rng = np.random.RandomState(seed)
    t = (1.0 + 5 ** 0.5) / 2
    V = [[-1, t, 0], [1, t, 0], [-1, -t, 0], [1, -t, 0], [0, -1, t], [0, 1, t], [0, -1, -t], [0, 1, -t],
         [t, 0, -1], [t, 0, 1], [-t, 0, -1], [-t, 0, 1]]
    Fc = [[0, 11, 5], [0, 5, 1], [0, 1, 7], [0, 7, 10], [0, 10, 11], [1, 5, 9], [5, 11, 4], [11, 10, 2],
          [10, 7, 6], [7, 1, 8], [3, 9, 4], [3, 4, 2], [3, 2, 6], [3, 6, 8], [3, 8, 9], [4, 9, 5], [2, 4, 11],
          [6, 2, 10], [8, 6, 7], [9, 8, 1]]
    V = [list(np.array(v) / np.linalg.norm(v)) for v in V]
    for _ in range(level):
        cache = {}
        nf = []

        def mid(a, b):
            key = (min(a, b), max(a, b))
            if key not in cache:
                m = (np.array(V[a]) + np.array(V[b])) / 2
                V.append(list(m / np.linalg.norm(m)))
                cache[key] = len(V) - 1
            return cache[key]
        for a, b, c in Fc:
            ab, bc, ca = mid(a, b), mid(b, c), mid(c, a)
            nf += [[a, ab, ca], [b, bc, ab], [c, ca, bc], [ab, bc, ca]]
        Fc = nf
    V = np.array(V)
    k = rng.normal(size=(6, 3)) * 2.5
    ph = rng.uniform(0, 6.28, 6)
    r = 1.0 + sum(0.06 * np.sin(V @ k[i] + ph[i]) for i in range(6))
    V = V * r[:, None] * np.array([0.9, 0.8, 0.7])
    with open(path, "w") as f:
        for v in V:
            f.write("v %.6f %.6f %.6f\n" % tuple(v))
        for a, b, c in Fc:
            f.write("f %d %d %d\n" % (a + 1, b + 1, c + 1))
    return len(V), len(Fc)


def blob_scene(obj_path, res=(64, 64), flat=False):
    """The reference's scenes/TorusMesh.json (plane + one mesh, three point lights) with
    the mesh file replaced by obj_path."""
    return {"resolution": list(res), "AA": {"jitter": False, "samples": 1}, "ambient": [0.1, 0.1, 0.1],
            "camera": {"position": [0.0, 4.0, 4.0], "lookAt": [0.0, 0.0, 0.0], "up": [0.0, 1.0, 0.0], "fov": 45.0},
            "materials": [{"name": "white", "ID": 0, "diffuse": [0.9, 0.9, 0.9], "specular": [0.1, 0.1, 0.1],
                           "hardness": 8},
                          {"name": "grey", "ID": 1, "diffuse": [0.3, 0.3, 0.3], "specular": [0.1, 0.1, 0.1]},
                          {"name": "clay", "ID": 2, "diffuse": [0.8, 0.5, 0.3], "specular": [0.6, 0.6, 0.6],
                           "hardness": 32}],
            "objects": [{"name": "plane", "type": "plane", "normal": [0.0, 1.0, 0.0], "position": [0.0, -1.0, 0.0],
                         "materials": [1, 0]},
                        {"name": "blob", "type": "mesh", "filepath": obj_path, "scale": 1.0,
                         "position": [0.0, 0.0, 0.0], "materials": [2], "flat_shaded": bool(flat)}],
            "lights": [{"name": "light1", "type": "point", "position": [-3.0, 10.0, 1.0], "colour": [1.0, 1.0, 1.0],
                        "power": 0.5},
                       {"name": "light2", "type": "point", "position": [3.0, 10.0, 1.0], "colour": [1.0, 1.0, 1.0],
                        "power": 0.5},
                       {"name": "light3", "type": "point", "position": [0.0, -5.0, 0.0], "colour": [1.0, 1.0, 1.0],
                        "power": 10.0}]}


def bv_stress_rays(lo, hi, n, seed=0):
    """Rays that stress a mesh's AABB bounding volume (bounding_volumes.py:49-83):
    origins inside, outside and exactly on the faces of the box [lo, hi], directions with
    exact zero components, and rays aimed at the box's edges and corners (start == end up
    to rounding). Returns float32 (n, 3) origins and directions."""
    rng = np.random.RandomState(seed)
    lo = np.asarray(lo, np.float64)
    hi = np.asarray(hi, np.float64)
    span = hi - lo
    k = n // 4
    # 1: origins in the box grown by half its size, random directions, some axes zeroed
    o1 = lo - 0.5 * span + rng.uniform(0, 2, (k, 3)) * span
    d1 = rng.normal(size=(k, 3))
    z = rng.rand(k, 3) < 0.15
    d1[z] = 0.0
    d1[np.all(d1 == 0, axis=1), 1] = 1.0
    # 2: origins exactly on a face of the box
    o2 = lo + rng.uniform(0, 1, (k, 3)) * span
    ax = rng.randint(0, 3, k)
    side = rng.rand(k) < 0.5
    o2[np.arange(k), ax] = np.where(side, lo[ax], hi[ax])
    d2 = rng.normal(size=(k, 3))
    # 3: aimed at points on the box's edges and corners from outside
    m = n - 3 * k
    tgt = lo + rng.uniform(0, 1, (m, 3)) * span
    for i in range(m):
        for a in rng.choice(3, rng.randint(2, 4), replace=False):
            tgt[i, a] = lo[a] if rng.rand() < 0.5 else hi[a]
    d3 = rng.normal(size=(m, 3))
    o3 = tgt - d3 * rng.uniform(1, 6, (m, 1))
    # 4: like 1 with directions of very different magnitudes (unnormalised shadow rays)
    o4 = lo - span + rng.uniform(0, 3, (k, 3)) * span
    d4 = rng.normal(size=(k, 3)) * (10.0 ** rng.uniform(-3, 2, (k, 1)))
    o = np.concatenate([o1, o2, o3, o4]).astype(np.float32)
    d = np.concatenate([d1, d2, d3, d4]).astype(np.float32)
    return o, d


def scene_box_stress_rays(scene_dict, n_per_box, seed=0):
    """bv_stress_rays around every top-level box of a scene dict (corners as AABB.__init__
    computes them in fp32: center -+ size / 2, simple_geometry.py:180-185)."""
    os_, ds_ = [], []
    for k, b in enumerate(x for x in scene_dict["objects"] if x["type"] == "box"):
        c, s = np.float32(b["position"]), np.float32(b["size"])
        o, d = bv_stress_rays(c - s / np.float32(2), c + s / np.float32(2), n_per_box, seed * 7 + k)
        os_.append(o)
        ds_.append(d)
    return np.concatenate(os_), np.concatenate(ds_)


def obj_bounds(path):
    """Vertex bounds (float32) of an OBJ file, as Mesh.__init__ computes them for scale 1
    and no translation (mesh.py:31-36)."""
    v = np.array([[float(x) for x in l.split()[1:4]] for l in open(path) if l.startswith("v ")], np.float32)
    return v.min(axis=0), v.max(axis=0)


def bins_scene(seed, res=(41, 23), lens=False):
    """Scenes that stress the primary-ray bins (rtx_api.hip primary_bins): one sample per
    pixel, no lens or jitter (the pinhole bins), wide and narrow fields of view, spheres and
    boxes around, beside, behind and enclosing the camera, tiny far spheres (the fp32
    discriminant's fuzz), moving objects, and sometimes the torus mesh up close. lens=True:
    the same scenes seen through a lens (DOF samples, apertures up to 1.5, near and far
    focal lengths) with AA samples and jitter (the thick bins)."""
    rng = np.random.RandomState(1000 + seed)
    r = lambda lo, hi, n=None: np.round(rng.uniform(lo, hi, n), 3).tolist()  # noqa: E731
    mats = [{"name": "m%d" % i, "ID": i, "diffuse": r(0, 1, 3), "specular": r(0, 1, 3), "hardness": 16,
             "type": "mirror" if i == 3 else "diffuse", "tint": 0.3} for i in range(4)]
    cam = np.array([r(-2, 2), r(0.5, 3), r(3, 8)])
    look = np.array([r(-1, 1), r(0, 1), r(-1, 1)])
    objs = [{"name": "ground", "type": "plane", "normal": [0.0, 1.0, 0.0], "position": [0.0, -1.0, 0.0],
             "materials": [0, 1]}]
    fwd = (look - cam) / np.linalg.norm(look - cam)
    for k in range(rng.randint(2, 7)):
        kind = rng.randint(5)
        if kind == 0:    # beside / behind the camera
            c = cam + rng.uniform(-3, 3, 3) - fwd * rng.uniform(0, 2)
            rad = float(r(0.2, 1.0))
        elif kind == 1:  # tiny and far
            c = cam + fwd * rng.uniform(30, 80) + rng.uniform(-5, 5, 3)
            rad = float(r(0.01, 0.2))
        elif kind == 2:  # enclosing the camera
            c = cam + rng.uniform(-0.2, 0.2, 3)
            rad = float(r(1.0, 2.0))
        else:            # in view
            c = look + rng.uniform(-2, 2, 3)
            rad = float(r(0.2, 1.2))
        o = {"name": "s%d" % k, "type": "sphere", "radius": rad, "position": np.round(c, 3).tolist(),
             "materials": [int(rng.randint(4))]}
        if rng.rand() < 0.2:
            o["speed"] = r(-0.5, 0.5, 3)
        objs.append(o)
    for k in range(rng.randint(0, 3)):
        c = (cam if rng.rand() < 0.3 else look) + rng.uniform(-2, 2, 3)
        objs.append({"name": "b%d" % k, "type": "box", "position": np.round(c, 3).tolist(), "size": r(0.2, 1.5, 3),
                     "materials": [int(rng.randint(4))]})
    if rng.rand() < 0.5:
        objs.append({"name": "torus", "type": "mesh", "filepath": "torus_mesh.obj", "scale": float(r(0.4, 1.2)),
                     "position": np.round(look + rng.uniform(-1, 1, 3), 3).tolist(), "materials": [2],
                     "flat_shaded": bool(rng.rand() < 0.5)})
    sc = {"resolution": list(res), "AA": {"jitter": False, "samples": 1}, "ambient": [0.1, 0.1, 0.1],
          "camera": {"position": np.round(cam, 3).tolist(), "lookAt": np.round(look, 3).tolist(),
                     "up": [0.0, 1.0, 0.0], "fov": float(rng.choice([15.0, 45.0, 90.0, 120.0]))},
          "materials": mats, "objects": objs,
          "lights": [{"name": "p", "type": "point", "position": [2.0, 6.0, 3.0], "colour": [1.0, 1.0, 1.0],
                      "power": 1.0}]}
    if rng.rand() < 0.3:
        sc["motion"] = {"time": 1.0, "samples": 2, "final": 1}
    if lens:  # the lens cameras' "thick" bins: DOF spread, AA spread, jitter
        lr = np.random.RandomState(5000 + seed)
        sc["DOF"] = {"aperture": float(np.round(lr.choice([0.02, 0.2, 0.6, 1.5]), 3)),
                     "focal_length": float(np.round(lr.uniform(0.5, 12.0), 3)), "samples": int(lr.randint(1, 9))}
        sc["AA"] = {"jitter": bool(lr.rand() < 0.8), "samples": int(lr.randint(1, 4))}
    return sc
