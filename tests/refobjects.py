"""Reference-shaped scene objects rebuilt from tests/golden/refobjects.json (made by
tests/golden/make_refobjects.py from the reference's own parser): instances of classes
named like the reference's (Scene, ViewportCamera, Material, Light, Sphere, Plane, AABB,
Mesh, BoundingAABB, BoundingSphere, Hierarchy) carrying exactly the attributes the
reference's objects carried, with PyGLM-like vectors (tests/refshim/glm.py) and PIL
textures. They have no methods: they are what a maintainer's `Scene.render` would hand
to rtx.Scene.from_reference."""
import functools
import importlib.util
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURE = os.path.join(HERE, "golden", "refobjects.json")
TEXTURES = os.path.join(os.path.dirname(HERE), "assets", "textures")


@functools.lru_cache(None)
def glm():
    spec = importlib.util.spec_from_file_location("refshim_glm", os.path.join(HERE, "refshim", "glm.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@functools.lru_cache(None)
def _class(name, module):
    return type(name, (), {"__module__": module})


def names():
    with open(FIXTURE) as f:
        return list(json.load(f))


def load(name):
    """(reference-shaped Scene object, resolution) of one fixture scene."""
    from PIL import Image
    with open(FIXTURE) as f:
        entry = json.load(f)[name]
    g = glm()
    memo = {}

    def dec(x):
        if isinstance(x, list):
            return [dec(v) for v in x]
        if not isinstance(x, dict):
            return x
        if "__vec__" in x:
            return (g.vec3 if x["__vec__"] == 3 else g.vec4)(*x["v"])
        if "__mat4__" in x:
            return g.mat4._wrap(np.array(x["__mat4__"], np.float32).reshape(4, 4))
        if "__np__" in x:
            return np.dtype(x["__np__"]).type(x["v"])
        if "__nd__" in x:
            return np.array(x["v"], dtype=x["__nd__"]).reshape(x["shape"])
        if "__tuple__" in x:
            return tuple(dec(v) for v in x["__tuple__"])
        if "__ref__" in x:
            return memo[x["__ref__"]]
        if "__image__" in x:
            im = Image.open(os.path.join(TEXTURES, x["__image__"]))
            memo[x["__id__"]] = im
            return im
        o = _class(x["__obj__"], x["__module__"]).__new__(_class(x["__obj__"], x["__module__"]))
        memo[x["__id__"]] = o
        for a, v in x["attrs"].items():
            setattr(o, a, dec(v))
        return o
    return dec(entry["scene"]), tuple(entry["resolution"])
