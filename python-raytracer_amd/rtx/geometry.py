"""Scene geometry descriptions (mirror of provided/geometry/*.py constructors).

These classes keep the reference's constructor signatures and attributes; they hold
*data* only. Their intersect/shadow_intersect behaviour lives on the device
(csrc/rtx_trace.h) and is reached through ``Scene.intersect`` / ``Scene.occluded`` (the
batched Geometry ABI) and ``Scene.render``. ``Mesh`` performs the reference's host
preprocessing (OBJ read, transform, smooth normals, bounding-volume choice) in fp32.
"""
import math
import os

import numpy as np

from . import f32 as F
from .track import TList, Tracked

epsilon = 10 ** (-4)  # geometry/__init__.py:12


class Geometry(Tracked):
    """geometry/__init__.py:38-63. Attribute edits, in-place array writes and changes of
    TList attributes are tracked (rtx.track), so a Scene re-uploads an edited object."""
    shadow_epsilon = 10 ** (-4)

    def __init__(self, name, gtype, materials, speed):
        self.name = name
        self.gtype = gtype
        self.materials = materials
        self.speed = None if speed is None else F.vec3(speed)

    def set_scene(self, scene):
        self.scene = scene

    def __repr__(self):
        return "Geometry(%s, type: %s)" % (self.name, self.gtype)


class Sphere(Geometry):
    """simple_geometry.py:12-83."""
    shadow_epsilon = 10 ** (-3)

    def __init__(self, name, gtype, materials, center, radius, speed):
        super().__init__(name, gtype, materials, speed)
        self.center = F.vec3(center)
        self.radius = radius


class Plane(Geometry):
    """simple_geometry.py:86-176. ``texture`` is the PIL image the parser opened
    (scene_parser.py:222-229); ``texture_scale`` defaults to 1.0 (simple_geometry.py:157-160)."""

    def __init__(self, name, gtype, materials, point, normal, speed):
        super().__init__(name, gtype, materials, speed)
        self.point = F.vec3(point)
        self.normal = F.vec3(normal)
        self.texture = None
        self.texture_scale = 1.0


class AABB(Geometry):
    """simple_geometry.py:179-355: halfside = dimension / 2 (fp32)."""

    def __init__(self, name, gtype, materials, center, dimension, speed):
        super().__init__(name, gtype, materials, speed)
        halfside = F.vec3(dimension) / np.float32(2)
        center = F.vec3(center)
        self.minpos = center - halfside
        self.maxpos = center + halfside
        self.texture = None


def read_obj(path):
    """igl.read_obj for triangle OBJ files (mesh.py:20): vertices (fp64), 0-based faces,
    vertex normals (unused: the reference recomputes them)."""
    V, N, Fc = [], [], []
    with open(path) as f:
        for line in f:
            p = line.split()
            if not p:
                continue
            if p[0] == "v":
                V.append([float(x) for x in p[1:4]])
            elif p[0] == "vn":
                N.append([float(x) for x in p[1:4]])
            elif p[0] == "f":
                idx = [int(x.split("/")[0]) for x in p[1:]]
                if len(idx) != 3:
                    raise ValueError("%s: only triangle faces are supported (got %d vertices)" % (path, len(idx)))
                Fc.append([i - 1 if i > 0 else len(V) + i for i in idx])
    return (np.array(V, dtype=np.float64).reshape(-1, 3), np.array(N, dtype=np.float64).reshape(-1, 3),
            np.array(Fc, dtype=np.int64).reshape(-1, 3))


class Mesh(Geometry):
    """mesh.py:16-70: (v + translate) * scale, area-weighted smooth normals, and the
    bounding volume (AABB if its volume is below the bounding sphere's)."""

    def __init__(self, name, gtype, materials, translate, scale, filepath, flat_shaded=False, speed=None):
        super().__init__(name, gtype, materials, speed)
        V, N, self.faces = read_obj(filepath)
        if len(self.faces) and (self.faces.min() < 0 or self.faces.max() >= len(V)):
            raise ValueError("%s: face index out of range" % filepath)
        self.filepath = filepath
        self.verts = (V.astype(np.float32) + F.vec3(translate)) * np.float32(scale)
        self.norms = N.astype(np.float32)
        self.flat_shaded = bool(flat_shaded)
        if not self.flat_shaded:
            self._compute_normals()

        vs = self.verts
        max_x, min_x = float(vs[:, 0].max()), float(vs[:, 0].min())
        max_y, min_y = float(vs[:, 1].max()), float(vs[:, 1].min())
        max_z, min_z = float(vs[:, 2].max()), float(vs[:, 2].min())
        center = F.vec3((max_x + min_x) / 2, (max_y + min_y) / 2, (max_z + min_z) / 2)
        max_dist = float(F.length(vs - center).max())
        aabb_volume = (max_x - min_x) * (max_y - min_y) * (max_z - min_z)
        sphere_volume = 4 / 3 * math.pi * max_dist ** 3
        if aabb_volume < sphere_volume:
            self.bounding_volume = BoundingAABB(F.vec3(min_x, min_y, min_z), F.vec3(max_x, max_y, max_z), None)
        else:
            self.bounding_volume = BoundingSphere(center, max_dist, None)

    def _compute_normals(self):
        """mesh.py:53-70: normals[face[k]] += normalize(e1 x e2) * area, in face order."""
        v = self.verts
        f = self.faces
        v0, v1, v2 = v[f[:, 0]], v[f[:, 1]], v[f[:, 2]]
        c = F.cross(v1 - v0, v2 - v0)
        normal = F.normalize(c)
        area = (F.length(c).astype(np.float64) / 2).astype(np.float32)
        weighted = normal * area[:, None]
        acc = np.zeros_like(v)
        np.add.at(acc, f.ravel(), np.repeat(weighted, 3, axis=0))  # sequential, in face order
        self.norms = F.normalize(acc)

    def __repr__(self):
        return "Mesh(%s)" % self.name


class BoundingSphere(Tracked):
    """bounding_volumes.py:12-16 (the cull itself runs on the device: mesh_bv)."""

    def __init__(self, center, radius, geometry):
        self.center = F.vec3(center)
        self.radius = radius
        self.geometry = geometry


class BoundingAABB(Tracked):
    """bounding_volumes.py:43-47."""

    def __init__(self, minpos, maxpos, geometry):
        self.minpos = F.vec3(minpos)
        self.maxpos = F.vec3(maxpos)


def resolve_path(path, base_dir):
    """The reference opens asset paths relative to the CWD; fall back to the scene file's
    directory when the CWD-relative path does not exist."""
    if os.path.exists(path) or base_dir is None:
        return path
    alt = os.path.join(base_dir, path)
    return alt if os.path.exists(alt) else path


class Hierarchy(Geometry):
    """hierarchy.py:11-146: a CSG node (union / intersection / difference) with a
    translate-rotate-scale transform. The matrices are built on the device side of the
    ABI from (t, r, s) exactly as make_matrices does (hierarchy.py:30-40)."""

    def __init__(self, name, gtype, materials, hierarchy_type, t, r, s, speed):
        super().__init__(name, gtype, materials, speed)
        self.hierarchy_type = hierarchy_type
        self.children = TList()
        self.make_matrices(t, r, s)

    def make_matrices(self, t, r, s):
        self.t = F.vec3(t)
        self.r = F.vec3(r)
        self.s = F.vec3(s)

    def set_fallback_material(self, materials):
        """hierarchy.py:21-28: leaves get the root's materials appended (nested nodes pass them on)."""
        if len(materials) == 0:
            return
        for child in self.children:
            if isinstance(child, Hierarchy):
                child.set_fallback_material(materials)
            else:
                child.materials += materials

    def set_scene(self, scene):
        self.scene = scene
        for child in self.children:
            child.set_scene(scene)

    def __repr__(self):
        return "Hierarchy(%s, t: %s, r: %s, s: %s, children: %d)" % (self.name, self.t, self.r, self.s,
                                                                      len(self.children))


def open_texture(path, base_dir=None):
    """Image.open(texture) (scene_parser.py:224) as the RGB8 array getpixel((i, j))[:3]
    reads; modes whose getpixel is not an RGB-indexable tuple raise like the reference."""
    from PIL import Image
    im = Image.open(resolve_path(path, base_dir))
    if im.mode not in ("RGB", "RGBA", "RGBX", "CMYK", "RGBa", "YCbCr", "LAB", "HSV"):
        raise TypeError("texture %s: getpixel of mode %s is not indexable as RGB" % (path, im.mode))
    return im
