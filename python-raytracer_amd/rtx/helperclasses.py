"""Value types of the scene description (mirror of provided/helperclasses.py:13-108).

Same class names, constructor arguments and attribute names as the reference, so code
written against the reference's objects keeps working. Vectors are numpy float32 arrays
(PyGLM vec3 semantics); scalars are Python floats.
"""
import math
import weakref

import numpy as np

from . import f32 as F
from .track import Tracked


class Ray:
    """helperclasses.py:13-25 (host-side value; the device traces rays in SoA form)."""

    def __init__(self, o, d):
        self.origin = F.vec3(o)
        self.direction = F.vec3(d)

    def getDistance(self, point):
        return float(F.length(F.vec3(point) - self.origin))

    def getPoint(self, t):
        return self.origin + F.scale(self.direction, t)

    def __repr__(self):
        return "Ray(origin: %s, dir: %s)" % (self.origin, self.direction)


class Material(Tracked):
    """helperclasses.py:28-47 (edits are tracked: rtx.track)."""

    def __init__(self, name, specular, diffuse, hardness, ID, mat_type="diffuse", mat_tint=0.0):
        self.name = name
        self.specular = F.vec3(specular)
        self.diffuse = F.vec3(diffuse)
        self.hardness = hardness
        self.ID = ID
        self.mat_type = mat_type
        self.refr_index = 1.0
        self.tint = mat_tint

    @staticmethod
    def default():
        return Material("default", (0, 0, 0), (0, 0, 0), -1, -1)

    def __repr__(self):
        return "Material(%s, type: %s, specular: %s, diffuse: %s, hardness: %s, ID: %s)" % (
            self.name, self.mat_type, self.specular, self.diffuse, self.hardness, self.ID)


class Light(Tracked):
    """helperclasses.py:50-59 (edits are tracked: rtx.track)."""

    def __init__(self, ltype, name, colour, vector, power):
        self.type = ltype
        self.name = name
        self.colour = F.vec3(colour)
        self.vector = F.vec3(vector)
        self.power = power

    def __repr__(self):
        return "Light(%s, type: %s, colour: %s, vector: %s, power: %s)" % (
            self.name, self.type, self.colour, self.vector, self.power)


class AAInterval:
    """helperclasses.py:62-66 (the device restates it in rtx_trace.h box_slabs)."""

    def __init__(self, t1, t2, label=None):
        self.start = min(t1, t2)
        self.end = max(t1, t2)
        self.label = label


class _Times(list):
    """ViewportCamera.motion_times: a list that counts its owner's version up on every
    in-place change (it still compares equal to a plain list)."""

    def __init__(self, values, owner):
        super().__init__(values)
        self._owner = owner

    def _changed(self):
        self._owner._bump()


def _tracked(name):
    def method(self, *args, **kwargs):
        r = getattr(list, name)(self, *args, **kwargs)
        self._changed()
        return self if name == "__iadd__" or name == "__imul__" else r
    method.__name__ = name
    return method


for _m in ("__setitem__", "__delitem__", "__iadd__", "__imul__", "append", "extend", "insert", "pop", "remove",
           "clear", "sort", "reverse"):
    setattr(_Times, _m, _tracked(_m))


class _Vec(np.ndarray):
    """A ViewportCamera basis vector: a writable fp32 array, like PyGLM's mutable vec3,
    that counts its camera's version up when it is written in place -- item assignment
    (``vc.position[0] = 1``, also through a view) or a ufunc writing into it
    (``vc.position += d``, ``np.add(a, b, out=vc.position)``). Arithmetic on it returns
    plain arrays. Writes that bypass both (``np.copyto``, ``fill``, a ``.view(np.ndarray)``)
    are not seen: call Scene.invalidate() after them."""

    def __array_finalize__(self, obj):
        self._owner = getattr(obj, "_owner", None)

    def _touch(self):
        o = self._owner() if self._owner is not None else None
        if o is not None:
            o._bump()

    def __setitem__(self, key, value):
        super().__setitem__(key, value)
        self._touch()

    def __array_ufunc__(self, ufunc, method, *inputs, out=None, **kwargs):
        plain = [x.view(np.ndarray) if isinstance(x, _Vec) else x for x in inputs]
        if out is None:
            return getattr(ufunc, method)(*plain, **kwargs)
        kwargs["out"] = tuple(o.view(np.ndarray) if isinstance(o, _Vec) else o for o in out)
        getattr(ufunc, method)(*plain, **kwargs)
        for o in out:
            if isinstance(o, _Vec):
                o._touch()
        return out[0] if len(out) == 1 else out


class ViewportCamera:
    """helperclasses.py:69-108: viewport, camera basis, lens and motion samples.

    Every attribute assignment counts ``_version`` up, so a Scene re-uploads its camera
    tables only after a change (Scene._set_camera). The basis vectors are kept as fp32
    ``_Vec`` copies and motion_times (any sequence assigned) as a list; both report
    in-place edits. A vector of another type (e.g. a PyGLM vec3 set by hand) makes the
    scene compare every camera value per render instead."""

    _VECS = ("position", "u", "v", "w")

    def __init__(self):
        object.__setattr__(self, "_version", 0)
        object.__setattr__(self, "_untracked", False)
        self.focal_length = 1.0
        self.aperture = 0.0
        self.dof_samples = 1
        self.motion_times = [0]

    def set_viewport(self, width, height):
        self.width = width
        self.height = height
        self.aspect = width / height
        return self

    def set_camera(self, position, lookat, up, fov):
        position, lookat, up = F.vec3(position), F.vec3(lookat), F.vec3(up)
        cam_dir = position - lookat
        self.position = position
        self.d = 1.0
        self.top = self.d * math.tan(math.radians(fov / 2))
        self.right = self.aspect * self.top
        self.bottom = -self.top
        self.left = -self.right
        self.w = F.normalize(cam_dir)
        self.u = F.normalize(F.cross(up, self.w))
        self.v = F.cross(self.w, self.u)
        return self

    def set_lens(self, focal_length, aperture, dof_samples):
        self.focal_length = focal_length
        self.aperture = aperture
        self.dof_samples = dof_samples
        return self

    def __setattr__(self, name, value):
        if name in self._VECS:
            if isinstance(value, np.ndarray):
                value = np.array(value).view(_Vec)
                value._owner = weakref.ref(self)
            else:
                object.__setattr__(self, "_untracked", True)
        elif name == "motion_times" and not (isinstance(value, _Times) and value._owner is self):
            try:
                value = _Times(list(value), self)
            except TypeError:  # not a sequence: compared by value per render
                object.__setattr__(self, "_untracked", True)
        object.__setattr__(self, name, value)
        self._bump()

    def _bump(self):
        # (a deep copy restores motion_times before _version)
        object.__setattr__(self, "_version", self.__dict__.get("_version", 0) + 1)

    def set_motion(self, time, motion_samples, motion_final):
        dt = time / motion_samples
        self.motion_times = [dt * i for i in range(motion_samples)]
        self.motion_times += [time] * motion_final
        return self


_SUNFLOWER_TERMS = {}


def _sunflower_terms(num_points):
    """Per point k: sqrt(k - 0.5), cos(theta_k), sin(theta_k) with theta_k = k * angle_stride,
    each computed as the reference computes it (numpy fp64 scalar calls); they do not
    depend on the origin or radius, so they are kept per num_points."""
    t = _SUNFLOWER_TERMS.get(num_points)
    if t is None:
        phi = (1 + np.sqrt(5)) / 2
        angle_stride = 2 * np.pi / phi
        sq = np.empty(num_points, np.float64)
        co = np.empty(num_points, np.float64)
        si = np.empty(num_points, np.float64)
        for k in range(1, num_points + 1):
            theta = k * angle_stride
            sq[k - 1] = np.sqrt(k - 0.5)
            co[k - 1] = np.cos(theta)
            si[k - 1] = np.sin(theta)
        t = (sq, co, si, np.sqrt(num_points - 0.5))
        if len(_SUNFLOWER_TERMS) < 64:
            _SUNFLOWER_TERMS[num_points] = t
    return t


def sunflower(num_points, origin, radius):
    """Scene._sunflower_spread (scene.py:118-138), evaluated with numpy fp64 as the
    reference does -- r = radius * sqrt(k - 0.5) / sqrt(n - 0.5), (r cos(theta) + ox,
    r sin(theta) + oy, oz) -- each element with the reference's operations in its order;
    points are PyGLM vec3 (float32)."""
    out = np.zeros((num_points, 3), dtype=np.float32)
    if num_points <= 0:
        return out
    sq, co, si, sn = _sunflower_terms(num_points)
    ox, oy, oz = float(origin[0]), float(origin[1]), origin[2]
    r = radius * sq / sn
    out[:, 0] = (r * co + ox).astype(np.float32)
    out[:, 1] = (r * si + oy).astype(np.float32)
    out[:, 2] = np.float32(np.float64(oz))
    return out


def sunflower_many(num_points, origins, radius):
    """sunflower(num_points, o, radius) for every row o of origins (float32 [m, 3]) at once:
    [m, num_points, 3], the same values (the per-element operations are sunflower's)."""
    origins = np.asarray(origins)
    m = len(origins)
    out = np.zeros((m, num_points, 3), dtype=np.float32)
    if num_points <= 0 or m == 0:
        return out
    sq, co, si, sn = _sunflower_terms(num_points)
    r = radius * sq / sn
    ox = origins[:, 0].astype(np.float64)[:, None]
    oy = origins[:, 1].astype(np.float64)[:, None]
    out[:, :, 0] = (r * co + ox).astype(np.float32)
    out[:, :, 1] = (r * si + oy).astype(np.float32)
    out[:, :, 2] = origins[:, 2].astype(np.float64).astype(np.float32)[:, None]
    return out
