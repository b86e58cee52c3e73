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


def tie_scene(res=(40, 30)):
    """Coincident geometry: the first object in scene order must win closest-hit ties."""
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
