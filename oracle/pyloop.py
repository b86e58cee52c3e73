"""The reference's Python render loop, restated in pure Python (TEST / BASELINE
INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg and tests/ import it; the product never
does). It is the CPU baseline the north star names — "the reference Python loop timed on
the same box's host cores" — for a box where the reference cannot travel and PyGLM is not
installed: one Python call per pixel, sample, ray and object, recursive cast_ray, hit
lists and min() by time, as provided/scene.py:35-209 and provided/geometry/*.py do, with
PyGLM's fp32 vector arithmetic done on numpy float32 scalars and Python's fp64 scalars
as Python floats. tests/test_pyloop.py proves it bit-identical to the C oracle
(oracle/rtx_oracle.c, itself pinned to the published renders).

Scope: every scene the oracle renders: spheres, planes with checkers, boxes, triangle
meshes with their bounding volume, point / directional lights, mirror and refractive
materials, motion blur, DOF / AA, replayed jitter, and (round 4) CSG hierarchies
(provided/geometry/hierarchy.py, with GLM's float mat4 restated below) and plane / box
textures (simple_geometry.py:150-173, :312-355).
"""
import ctypes
import math
import os

import numpy as np

f32 = np.float32
EPSILON = 10 ** (-4)          # geometry/__init__.py:12
SHADOW_EPSILON = 10 ** (-4)   # geometry/__init__.py:39
SPHERE_SHADOW_EPSILON = 10 ** (-3)  # simple_geometry.py:13
ZERO = (f32(0), f32(0), f32(0))


# ---------------------------------------------------------------- PyGLM vec3 (fp32)
def V(x, y, z):
    return (f32(x), f32(y), f32(z))


def add(a, b):
    return (a[0] + b[0], a[1] + b[1], a[2] + b[2])


def sub(a, b):
    return (a[0] - b[0], a[1] - b[1], a[2] - b[2])


def mul(a, b):
    return (a[0] * b[0], a[1] * b[1], a[2] * b[2])


def scale(a, s):
    s = f32(s)  # vec3 * Python number: the number is cast to float first
    return (a[0] * s, a[1] * s, a[2] * s)


def neg(a):
    return (-a[0], -a[1], -a[2])


def dot(a, b):
    """glm.dot: (x*x + y*y) + z*z in fp32."""
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]


def cross(a, b):
    return (a[1] * b[2] - b[1] * a[2], a[2] * b[0] - b[2] * a[0], a[0] * b[1] - b[0] * a[1])


def normalize(v):
    """glm.normalize = v * (1 / sqrt(dot(v, v)))."""
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = f32(1.0) / np.sqrt(dot(v, v))
    return (v[0] * inv, v[1] * inv, v[2] * inv)


def length(v):
    return np.sqrt(dot(v, v))


def reflect(i, n):
    """glm.reflect = I - N * dot(N, I) * 2."""
    return sub(i, scale(scale(n, dot(n, i)), 2.0))


def refract(i, n, eta):
    """glm.refract in float."""
    eta = f32(eta)
    d = dot(n, i)
    k = f32(1.0) - eta * eta * (f32(1.0) - d * d)
    if not k >= 0:
        return ZERO
    return sub(scale(i, eta), scale(n, eta * d + np.sqrt(k)))


# ---------------------------------------------------------------- GLM mat4 (float)
# m[column][row] of numpy float32 scalars, every operation in GLM 0.9.9's generic order
# (PyGLM wraps it); cos / sin of the float angle are libm's cosf / sinf, as GLM calls them.
_LIBM = ctypes.CDLL("libm.so.6")
_LIBM.cosf.restype = _LIBM.sinf.restype = ctypes.c_float
_LIBM.cosf.argtypes = _LIBM.sinf.argtypes = [ctypes.c_float]


def m_identity():
    return [[f32(1.0) if c == k else f32(0.0) for k in range(4)] for c in range(4)]


def m_translate(m, v):
    """glm.translate: column 3 = m0 v.x + m1 v.y + m2 v.z + m3."""
    r = [list(col) for col in m]
    r[3] = [((m[0][k] * v[0] + m[1][k] * v[1]) + m[2][k] * v[2]) + m[3][k] for k in range(4)]
    return r


def m_rotate(m, angle, v):
    """glm.rotate(m, angle, axis)."""
    c, s = f32(_LIBM.cosf(angle)), f32(_LIBM.sinf(angle))
    a = normalize(v)
    t = scale(a, f32(1.0) - c)
    R = [[c + t[0] * a[0], t[0] * a[1] + s * a[2], t[0] * a[2] - s * a[1]],
         [t[1] * a[0] - s * a[2], c + t[1] * a[1], t[1] * a[2] + s * a[0]],
         [t[2] * a[0] + s * a[1], t[2] * a[1] - s * a[0], c + t[2] * a[2]]]
    r = [[(m[0][k] * R[col][0] + m[1][k] * R[col][1]) + m[2][k] * R[col][2] for k in range(4)] for col in range(3)]
    return r + [list(m[3])]


def m_scale(m, v):
    """glm.scale: columns 0-2 times v's components."""
    return [[m[col][k] * v[col] for k in range(4)] for col in range(3)] + [list(m[3])]


def m_inverse(m):
    """glm.inverse (compute_inverse<4, 4>: cofactors, then one reciprocal of the determinant)."""
    c00 = m[2][2] * m[3][3] - m[3][2] * m[2][3]
    c02 = m[1][2] * m[3][3] - m[3][2] * m[1][3]
    c03 = m[1][2] * m[2][3] - m[2][2] * m[1][3]
    c04 = m[2][1] * m[3][3] - m[3][1] * m[2][3]
    c06 = m[1][1] * m[3][3] - m[3][1] * m[1][3]
    c07 = m[1][1] * m[2][3] - m[2][1] * m[1][3]
    c08 = m[2][1] * m[3][2] - m[3][1] * m[2][2]
    c10 = m[1][1] * m[3][2] - m[3][1] * m[1][2]
    c11 = m[1][1] * m[2][2] - m[2][1] * m[1][2]
    c12 = m[2][0] * m[3][3] - m[3][0] * m[2][3]
    c14 = m[1][0] * m[3][3] - m[3][0] * m[1][3]
    c15 = m[1][0] * m[2][3] - m[2][0] * m[1][3]
    c16 = m[2][0] * m[3][2] - m[3][0] * m[2][2]
    c18 = m[1][0] * m[3][2] - m[3][0] * m[1][2]
    c19 = m[1][0] * m[2][2] - m[2][0] * m[1][2]
    c20 = m[2][0] * m[3][1] - m[3][0] * m[2][1]
    c22 = m[1][0] * m[3][1] - m[3][0] * m[1][1]
    c23 = m[1][0] * m[2][1] - m[2][0] * m[1][1]
    f0, f1, f2 = (c00, c00, c02, c03), (c04, c04, c06, c07), (c08, c08, c10, c11)
    f3_, f4, f5 = (c12, c12, c14, c15), (c16, c16, c18, c19), (c20, c20, c22, c23)
    v0 = (m[1][0], m[0][0], m[0][0], m[0][0])
    v1 = (m[1][1], m[0][1], m[0][1], m[0][1])
    v2 = (m[1][2], m[0][2], m[0][2], m[0][2])
    v3 = (m[1][3], m[0][3], m[0][3], m[0][3])
    sa, sb = (f32(1), f32(-1), f32(1), f32(-1)), (f32(-1), f32(1), f32(-1), f32(1))
    inv = [[((v1[k] * f0[k] - v2[k] * f1[k]) + v3[k] * f2[k]) * sa[k] for k in range(4)],
           [((v0[k] * f0[k] - v2[k] * f3_[k]) + v3[k] * f4[k]) * sb[k] for k in range(4)],
           [((v0[k] * f1[k] - v1[k] * f3_[k]) + v3[k] * f5[k]) * sa[k] for k in range(4)],
           [((v0[k] * f2[k] - v1[k] * f4[k]) + v2[k] * f5[k]) * sb[k] for k in range(4)]]
    d0 = [m[0][k] * inv[k][0] for k in range(4)]
    one_over = f32(1.0) / ((d0[0] + d0[1]) + (d0[2] + d0[3]))
    return [[inv[c][k] * one_over for k in range(4)] for c in range(4)]


def m_transpose(m):
    return [[m[k][c] for k in range(4)] for c in range(4)]


def m_vec4(m, v):
    """mat4 * vec4: (m0 x + m1 y) + (m2 z + m3 w)."""
    return [(m[0][k] * v[0] + m[1][k] * v[1]) + (m[2][k] * v[2] + m[3][k] * v[3]) for k in range(4)]


def m_xform(m, p, w):
    """glm.vec3(m * glm.vec4(p, w))."""
    o = m_vec4(m, (p[0], p[1], p[2], f32(w)))
    return (o[0], o[1], o[2])


# ---------------------------------------------------------------- geometry (provided/geometry)
class Hit:
    """geometry/__init__.py:15-35 Intersection(time, normal, position, mat)."""
    __slots__ = ("time", "normal", "position", "mat", "geom")

    def __init__(self, time, normal, position, mat, geom):
        self.time, self.normal, self.position, self.mat, self.geom = time, normal, position, mat, geom


def get_point(o, d, t):
    return add(o, scale(d, t))  # helperclasses.py:21-22


class Sphere:
    """simple_geometry.py:12-83."""

    def __init__(self, center, radius, mats, speed):
        self.center, self.radius, self.mats, self.speed = center, float(radius), mats, speed

    def _roots(self, o, d, time):
        c = self.center if self.speed is None else add(self.center, scale(self.speed, time))
        a = float(dot(d, d))
        oc = sub(o, c)
        b = 2 * float(dot(d, oc))
        cc = float(dot(oc, oc)) - self.radius ** 2
        disc = b ** 2 - 4 * a * cc
        if disc < 0:
            return c, None
        return c, ((-b - math.sqrt(disc)) / (2 * a), (-b + math.sqrt(disc)) / (2 * a))

    def intersect(self, o, d, time):
        c, roots = self._roots(o, d, time)
        out = []
        if roots is not None:
            for t in roots:
                if t > 0:
                    p = get_point(o, d, t)
                    out.append(Hit(t, normalize(sub(p, c)), p, self.mats[0], self))
        return out

    def shadow_intersect(self, o, d, t_max, time):
        _, roots = self._roots(o, d, time)
        if roots is None:
            return False
        return any(SPHERE_SHADOW_EPSILON < t < t_max for t in roots)

    def is_inside(self, p, time):  # simple_geometry.py:74-80
        c = self.center if self.speed is None else add(self.center, scale(self.speed, time))
        return float(length(sub(p, c))) < self.radius

    def get_material(self, p, time):  # Geometry.get_material
        return self.mats[0]


class Plane:
    """simple_geometry.py:86-176."""

    def __init__(self, point, normal, mats, speed, texture=None, texture_scale=1.0):
        self.point, self.normal, self.mats, self.speed = point, normal, mats, speed
        self.texture, self.texture_scale = texture, texture_scale
        n = normal
        if n in (V(0, 1, 0), V(0, -1, 0), V(0, 0, 1)):
            self.width_axis = V(1, 0, 0)
        elif n == V(0, 0, -1):
            self.width_axis = V(-1, 0, 0)
        elif n == V(1, 0, 0):
            self.width_axis = V(0, 0, -1)
        elif n == V(-1, 0, 0):
            self.width_axis = V(0, 0, 1)
        else:
            self.width_axis = normalize(cross(n, V(0, 0, 1)))
        self.height_axis = normalize(cross(self.width_axis, n))

    def _pos(self, time):
        return self.point if self.speed is None else add(self.point, scale(self.speed, time))

    def material(self, p, time):
        pos = self._pos(time)
        if len(self.mats) == 1:
            return self.mats[0]
        p = sub(p, scale(self.normal, dot(sub(p, pos), self.normal)))
        x = float(dot(sub(p, pos), self.width_axis))
        z = float(dot(sub(p, pos), self.height_axis))
        return self.mats[(math.floor(float(pos[0]) - x) + math.floor(float(pos[2]) - z)) % 2]

    def get_material(self, p, time):
        return self.material(p, time)

    def is_inside(self, p, time):  # Geometry.is_inside
        return False

    def get_diffuse(self, p, time):
        """simple_geometry.py:150-173: the texel at the point projected on the plane (the
        projection uses the unmoved point, the texel offsets the moved one)."""
        if self.texture is None:
            return self.material(p, time).diffuse
        pos = self._pos(time)
        q = sub(p, scale(self.normal, dot(sub(p, self.point), self.normal)))
        tex = self.texture
        h, w = tex.shape[0], tex.shape[1]
        i = int((float(dot(sub(q, pos), self.width_axis)) * 1000.0 / self.texture_scale) % w)
        j = int((float(dot(sub(q, pos), self.height_axis)) * 1000.0 / self.texture_scale) % h)
        px = tex[j, i]
        return V(int(px[0]) / 255, int(px[1]) / 255, int(px[2]) / 255)

    def intersect(self, o, d, time):
        pos = self._pos(time)
        denom = float(dot(d, self.normal))
        if abs(denom) > EPSILON:
            t = float(dot(sub(pos, o), self.normal)) / denom
            if t >= 0:
                p = get_point(o, d, t)
                return [Hit(t, self.normal, p, self.material(p, time), self)]
        return []

    def shadow_intersect(self, o, d, t_max, time):
        pos = self._pos(time)
        denom = float(dot(d, self.normal))
        if abs(denom) > EPSILON:
            t = float(dot(sub(pos, o), self.normal)) / denom
            return SHADOW_EPSILON < t < t_max
        return False


def slabs(mn, mx, o, d):
    """The three AAIntervals of simple_geometry.py:196-221 (None: a zero-direction slab
    misses), then max(key=start) / min(key=end), first extreme kept."""
    iv = []
    for k in range(3):
        if d[k] == 0:
            if not (float(mn[k]) < float(o[k]) < float(mx[k])):
                return None
            iv.append((-math.inf, math.inf, k))
        else:
            t1 = (float(mn[k]) - float(o[k])) / float(d[k])
            t2 = (float(mx[k]) - float(o[k])) / float(d[k])
            iv.append((min(t1, t2), max(t1, t2), k))
    return max(iv, key=lambda x: x[0]), min(iv, key=lambda x: x[1])


_AXES = (V(1, 0, 0), V(0, 1, 0), V(0, 0, 1))


class AABB:
    """simple_geometry.py:179-355."""

    def __init__(self, minpos, maxpos, mats, speed, texture=None):
        self.minpos, self.maxpos, self.mats, self.speed = minpos, maxpos, mats, speed
        self.texture = texture

    def is_inside(self, p, time):  # simple_geometry.py:296-307
        mn, mx = self._box(time)
        return all(float(mn[k]) < float(p[k]) < float(mx[k]) for k in range(3))

    def get_material(self, p, time):
        return self.mats[0]

    def get_diffuse(self, p, time):
        """simple_geometry.py:312-355: the face the point lies on (within 1e-4) picks the
        texel; getpixel truncates the clamped float coordinates."""
        if self.texture is None:
            return self.mats[0].diffuse
        mn, mx = self._box(time)
        x = (float(p[0]) - float(mn[0])) / (float(mx[0]) - float(mn[0]))
        y = (float(p[1]) - float(mn[1])) / (float(mx[1]) - float(mn[1]))
        z = (float(p[2]) - float(mn[2])) / (float(mx[2]) - float(mn[2]))
        tex = self.texture
        h, w = tex.shape[0], tex.shape[1]
        if abs(p[0] - mn[0]) < EPSILON:
            i, j = z * w, (1 - y) * h
        elif abs(p[0] - mx[0]) < EPSILON:
            i, j = (1 - z) * w, (1 - y) * h
        elif abs(p[1] - mn[1]) < EPSILON:
            i, j = x * w, (1 - z) * h
        elif abs(p[1] - mx[1]) < EPSILON:
            i, j = x * w, z * h
        elif abs(p[2] - mn[2]) < EPSILON:
            i, j = (1 - x) * w, (1 - y) * h
        elif abs(p[2] - mx[2]) < EPSILON:
            i, j = x * w, (1 - y) * h
        else:
            i, j = 0, 0
        i = min(max(0, i), w - 1)
        j = min(max(0, j), h - 1)
        px = tex[int(j), int(i)]
        return V(int(px[0]) / 255, int(px[1]) / 255, int(px[2]) / 255)

    def _box(self, time):
        if self.speed is None:
            return self.minpos, self.maxpos
        s = scale(self.speed, time)
        return add(self.minpos, s), add(self.maxpos, s)

    def intersect(self, o, d, time):
        r = slabs(*self._box(time), o, d)
        if r is None:
            return []
        first, last = r
        if first[0] > last[1] or first[0] < 0:
            return []
        k = first[2]
        normal = neg(_AXES[k]) if d[k] > 0 else _AXES[k] if d[k] < 0 else ZERO
        return [Hit(t, normal, get_point(o, d, t), self.mats[0], self) for t in (first[0], last[1])]

    def shadow_intersect(self, o, d, t_max, time):
        r = slabs(*self._box(time), o, d)
        if r is None:
            return False
        first, last = r
        if first[0] > last[1]:
            return False
        return SHADOW_EPSILON < first[0] < t_max


class Mesh:
    """mesh.py:16-156: (v + translate) * scale, area-weighted smooth normals, AABB or
    sphere bounding volume, every face tested."""

    def __init__(self, verts64, faces, translate, scl, flat, mats):
        self.mats, self.flat = mats, flat
        self.verts = [scale(add(V(*v), translate), scl) for v in verts64]
        self.faces = [tuple(int(i) for i in f) for f in faces]
        if not flat:
            acc = [ZERO] * len(self.verts)
            for f in self.faces:
                v0, v1, v2 = (self.verts[i] for i in f)
                c = cross(sub(v1, v0), sub(v2, v0))
                w = scale(normalize(c), float(length(c)) / 2)
                for i in f:
                    acc[i] = add(acc[i], w)
            self.norms = [normalize(n) for n in acc]
        xs = [float(v[0]) for v in self.verts]
        ys = [float(v[1]) for v in self.verts]
        zs = [float(v[2]) for v in self.verts]
        center = V((max(xs) + min(xs)) / 2, (max(ys) + min(ys)) / 2, (max(zs) + min(zs)) / 2)
        max_dist = max(float(length(sub(v, center))) for v in self.verts)
        aabb_volume = (max(xs) - min(xs)) * (max(ys) - min(ys)) * (max(zs) - min(zs))
        self.bv_aabb = aabb_volume < 4 / 3 * math.pi * max_dist ** 3
        self.bv = (V(min(xs), min(ys), min(zs)), V(max(xs), max(ys), max(zs))) if self.bv_aabb else (center, max_dist)

    def _bv(self, o, d):
        """bounding_volumes.py:18-37 / :49-83."""
        if self.bv_aabb:
            r = slabs(self.bv[0], self.bv[1], o, d)
            return r is not None and not (r[0][0] > r[1][1] or r[0][0] < 0)
        c, radius = self.bv
        a = float(dot(d, d))
        oc = sub(o, c)
        b = 2 * float(dot(d, oc))
        cc = float(dot(oc, oc)) - radius ** 2
        disc = b ** 2 - 4 * a * cc
        if disc < 0:
            return False
        return (-b - math.sqrt(disc)) / (2 * a) > 0 or (-b + math.sqrt(disc)) / (2 * a) > 0

    def intersect(self, o, d, time):
        if not self._bv(o, d):
            return []
        out = []
        for f in self.faces:
            v0, v1, v2 = (self.verts[i] for i in f)
            normal = normalize(cross(sub(v1, v0), sub(v2, v0)))
            denom = float(dot(d, normal))
            if abs(denom) < EPSILON:
                continue
            t = float(dot(sub(v0, o), normal)) / denom
            if t < 0:
                continue
            p = get_point(o, d, t)
            if (dot(cross(sub(v1, v0), sub(p, v0)), normal) >= 0 and dot(cross(sub(v2, v1), sub(p, v1)), normal) >= 0
                    and dot(cross(sub(v0, v2), sub(p, v2)), normal) >= 0):
                if not self.flat:
                    b = barycentric(p, v0, v1, v2)
                    normal = normalize(add(add(scale(self.norms[f[0]], b[0]), scale(self.norms[f[1]], b[1])),
                                           scale(self.norms[f[2]], b[2])))
                out.append(Hit(t, normal, p, self.mats[0], self))
        return out

    def shadow_intersect(self, o, d, t_max, time):
        if not self._bv(o, d):
            return False
        for f in self.faces:  # no t_max test (mesh.py:121-153)
            v0, v1, v2 = (self.verts[i] for i in f)
            normal = cross(sub(v1, v0), sub(v2, v0))
            denom = float(dot(d, normal))
            if abs(denom) < EPSILON:
                continue
            t = float(dot(sub(v0, o), normal)) / denom
            if t < SHADOW_EPSILON:
                continue
            p = get_point(o, d, t)
            if (dot(cross(sub(v1, v0), sub(p, v0)), normal) >= 0 and dot(cross(sub(v2, v1), sub(p, v1)), normal) >= 0
                    and dot(cross(sub(v0, v2), sub(p, v2)), normal) >= 0):
                return True
        return False


def _no_inside(self, p, time):  # Geometry.is_inside (meshes, hierarchy.py reads it)
    return False


def _first_material(self, p, time):  # Geometry.get_material
    return self.mats[0]


Mesh.is_inside = _no_inside
Mesh.get_material = _first_material


class Hierarchy:
    """hierarchy.py:11-138: children in the node's frame (Minv applied to rays and points
    on the way down, M and transpose(Minv) to hit positions and normals on the way up)."""

    def __init__(self, kind, trs, mats):
        self.kind, self.mats, self.children = kind, mats, []
        t, r, sc = V(*trs[0:3]), V(*trs[3:6]), V(*trs[6:9])
        k = math.pi / 180.0  # glm.radians of a Python float: fp64, then the float angle
        m = m_translate(m_identity(), t)
        m = m_rotate(m, f32(float(r[0]) * k), V(1, 0, 0))
        m = m_rotate(m, f32(float(r[1]) * k), V(0, 1, 0))
        m = m_rotate(m, f32(float(r[2]) * k), V(0, 0, 1))
        self.M = m_scale(m, sc)
        self.Minv = m_inverse(self.M)
        self.MinvT = m_transpose(self.Minv)

    def intersect(self, o, d, time):
        mo, md = m_xform(self.Minv, o, 1.0), m_xform(self.Minv, d, 0.0)
        out = []
        if self.kind == "union":
            for c in self.children:
                out += c.intersect(mo, md, time)
        elif self.kind == "intersection":
            for c in self.children:
                for h in c.intersect(mo, md, time):
                    if all(o2 is c or o2.is_inside(h.position, time) for o2 in self.children):
                        out.append(h)
        elif self.kind == "difference":
            a, b = self.children[0], self.children[1]
            ha, hb = a.intersect(mo, md, time), b.intersect(mo, md, time)
            for h in ha:
                if not b.is_inside(h.position, time):
                    out.append(h)
            for h in hb:
                if a.is_inside(h.position, time):
                    h.mat = a.get_material(h.position, time)
                    h.normal = neg(h.normal)
                    out.append(h)
        for h in out:
            if h.mat is None:
                h.mat = self.mats[0]  # IndexError without materials, as the reference
            h.position = m_xform(self.M, h.position, 1.0)
            v = m_vec4(self.MinvT, (h.normal[0], h.normal[1], h.normal[2], f32(0.0)))
            inv = f32(1.0) / np.sqrt((v[0] * v[0] + v[1] * v[1]) + (v[2] * v[2] + v[3] * v[3]))
            h.normal = (v[0] * inv, v[1] * inv, v[2] * inv)  # the vec4's w stays in the length
        return out

    def shadow_intersect(self, o, d, t_max, time):
        mo, md = m_xform(self.Minv, o, 1.0), m_xform(self.Minv, d, 0.0)
        if self.kind == "union":
            return any(c.shadow_intersect(mo, md, t_max, time) for c in self.children)
        if self.kind == "intersection":
            return all(c.shadow_intersect(mo, md, t_max, time) for c in self.children)
        if self.kind == "difference":
            a, b = self.children[0], self.children[1]
            if any(h.time > SHADOW_EPSILON and not b.is_inside(h.position, time) for h in a.intersect(mo, md, time)):
                return True
            return any(h.time > SHADOW_EPSILON and a.is_inside(h.position, time) for h in b.intersect(mo, md, time))
        return False

    def is_inside(self, p, time):
        q = m_xform(self.Minv, p, 1.0)
        if self.kind == "union":
            return any(c.is_inside(q, time) for c in self.children)
        if self.kind == "intersection":
            return all(c.is_inside(q, time) for c in self.children)
        if self.kind == "difference":
            return self.children[0].is_inside(q, time) and not self.children[1].is_inside(q, time)
        return False

    def get_material(self, p, time):
        q = m_xform(self.Minv, p, 1.0)
        for c in self.children:
            if c.is_inside(q, time):
                return c.get_material(q, time)
        return None


def barycentric(p, a, b, c):
    """igl.barycentric_coordinates_tri on float32 rows (mesh.py:104-111), as the oracle
    restates it."""
    v0, v1, v2 = sub(b, a), sub(c, a), sub(p, a)
    d00, d01, d11 = dot(v0, v0), dot(v0, v1), dot(v1, v1)
    d20, d21 = dot(v2, v0), dot(v2, v1)
    den = d00 * d11 - d01 * d01
    v = (d11 * d20 - d01 * d21) / den
    w = (d00 * d21 - d01 * d20) / den
    return ((f32(1.0) - v) - w, v, w)


# ---------------------------------------------------------------- scene (provided/scene.py)
class Material:
    __slots__ = ("diffuse", "specular", "hardness", "kind", "tint", "refr_index")


class PyLoopScene:
    """Built from the oracle's independent JSON restatement (oracle.OracleScene)."""

    def __init__(self, osc):
        s = osc.s
        v = lambda p, i: V(p[3 * i], p[3 * i + 1], p[3 * i + 2])  # noqa: E731
        self.width, self.height = s.width, s.height
        # ViewportCamera (helperclasses.py:69-108)
        position, lookat, up = V(*s.cam[0:3]), V(*s.cam[3:6]), V(*s.cam[6:9])
        aspect = s.width / s.height
        self.position, self.d = position, 1.0
        self.top = self.d * math.tan(math.radians(s.cam[9] / 2))
        self.right = aspect * self.top
        self.bottom, self.left = -self.top, -self.right
        self.w = normalize(sub(position, lookat))
        self.u = normalize(cross(up, self.w))
        self.v = cross(self.w, self.u)
        self.focal_length, self.aperture, self.dof_samples = s.focal_length, s.aperture, s.dof_samples
        dt = s.motion_time / s.motion_samples
        self.motion_times = [dt * i for i in range(s.motion_samples)] + [s.motion_time] * s.motion_final
        self.jitter, self.samples = bool(s.jitter), s.samples
        self.ambient = V(*s.ambient)
        self.lights = [(s.light_type[i], v(s.light_colour, i), v(s.light_vector, i), s.light_power[i])
                       for i in range(s.n_lights)]
        self.mats = []
        for i in range(s.n_mats):
            m = Material()
            m.diffuse, m.specular, m.hardness = v(s.mat_diffuse, i), v(s.mat_specular, i), s.mat_hardness[i]
            m.kind, m.tint, m.refr_index = s.mat_type[i], s.mat_tint[i], s.mat_refr[i]
            self.mats.append(m)
        from . import oracle as _O
        textures = {}
        built = []
        for i, r in enumerate(osc.records):
            mats = [self.mats[k] for k in r["mats"]]
            speed = v(s.obj_speed, i) if s.obj_has_speed[i] else None
            kind = r["kind"]
            tex = None
            if s.obj_tex[i] >= 0:  # the oracle's scene-order texture list (Image.open + getpixel)
                path = r["json"]["texture"]
                if osc.base_dir is not None and not os.path.exists(path):
                    path = os.path.join(osc.base_dir, path)
                if path not in textures:
                    textures[path] = _O._load_texture(path)
                tex = textures[path]
            if kind == "node":
                g = Hierarchy(r["htype"] if r["htype"] in ("union", "intersection", "difference") else None,
                              [s.node_trs[9 * i + k] for k in range(9)], mats)
            elif kind == "sphere":
                g = Sphere(v(s.obj_a, i), s.obj_scalar[i], mats, speed)
            elif kind == "plane":
                g = Plane(v(s.obj_a, i), v(s.obj_b, i), mats, speed, tex, s.obj_tex_scale[i])
            elif kind == "box":
                if s.obj_box_mode[i] == 0:
                    half = tuple(x / f32(2) for x in v(s.obj_b, i))  # dimension / 2
                    c = v(s.obj_a, i)
                    g = AABB(sub(c, half), add(c, half), mats, speed, tex)
                else:
                    g = AABB(v(s.obj_c, i), v(s.obj_b, i), mats, speed, tex)
            else:
                vo, nv, fo, nf = s.mesh_vert_off[i], s.mesh_nverts[i], s.mesh_face_off[i], s.mesh_nfaces[i]
                verts = [(s.verts[3 * k], s.verts[3 * k + 1], s.verts[3 * k + 2]) for k in range(vo, vo + nv)]
                faces = [(s.faces[3 * k], s.faces[3 * k + 1], s.faces[3 * k + 2]) for k in range(fo, fo + nf)]
                g = Mesh(verts, faces, v(s.obj_a, i), s.obj_scalar[i], bool(s.obj_flat[i]), mats)
            built.append(g)
            if r["parent"] >= 0:
                built[r["parent"]].children.append(g)
        self.objects = [g for g, r in zip(built, osc.records) if r["parent"] < 0]
        self.current_time = 0.0
        self.rays = 0

    # scene.py:118-138
    @staticmethod
    def sunflower(n, origin, radius):
        phi = (1 + math.sqrt(5)) / 2
        stride = 2 * math.pi / phi
        out = []
        for k in range(1, n + 1):
            r = radius * math.sqrt(k - 0.5) / math.sqrt(n - 0.5)
            theta = k * stride
            out.append(V(r * math.cos(theta) + float(origin[0]), r * math.sin(theta) + float(origin[1]), origin[2]))
        return out

    # scene.py:81-116
    def cast_ray(self, o, d, max_recursion=10, in_shape=False):
        if max_recursion == 0:
            return ZERO
        time = self.current_time
        hits = []
        for obj in self.objects:
            hits += obj.intersect(o, d, time)
        if not hits:
            return ZERO
        hit = min(hits, key=lambda h: h.time)
        m = hit.mat
        if m.kind == 1:  # mirror
            r = reflect(d, hit.normal)
            reflection = self.cast_ray(add(hit.position, scale(r, 0.01)), r, max_recursion - 1, False)
            c = self.lighting(d, hit)
            c = add(scale(c, m.tint), scale(reflection, 1 - m.tint))
        elif m.kind == 2:  # refractive (scene.py:189-209)
            if in_shape:
                eta = m.refr_index
                hit.normal = neg(hit.normal)  # in place: the lighting below sees it too
            else:
                eta = 1 / m.refr_index
            r = refract(d, hit.normal, eta)
            refraction = ZERO if r == ZERO else self.cast_ray(add(hit.position, scale(r, 0.0001)), r,
                                                               max_recursion - 1, not in_shape)
            c = self.lighting(d, hit)
            c = add(scale(c, m.tint), scale(refraction, 1 - m.tint))
        else:
            c = self.lighting(d, hit)
        return tuple(f32(max(0, min(1, float(x)))) for x in c)

    # scene.py:140-187
    def lighting(self, d, hit):
        colour = ZERO
        m = hit.mat
        # scene.py:143-146: Plane / AABB hits (hierarchy leaves too) shade with get_diffuse
        diffuse = hit.geom.get_diffuse(hit.position, self.current_time) if isinstance(hit.geom, (Plane, AABB)) \
            else m.diffuse
        p, n = hit.position, hit.normal
        for kind, lcol, lvec, power in self.lights:
            if kind == 0:
                sd, t_max = sub(lvec, p), 1
            else:
                sd, t_max = neg(lvec), math.inf
            self.rays += 1
            if any(obj.shadow_intersect(p, sd, t_max, self.current_time) for obj in self.objects):
                continue
            light_dir = normalize(sub(lvec, p)) if kind == 0 else normalize(neg(lvec))
            lambert = scale(diffuse, max(0, float(dot(n, light_dir))))
            half = normalize(sub(light_dir, d))
            spec = scale(m.specular, max(0, float(dot(n, half))) ** m.hardness)
            colour = add(colour, mul(scale(lcol, power), add(lambert, spec)))
        return add(colour, mul(self.ambient, diffuse))

    # scene.py:35-79
    def render(self, subimage=0, tasks=1, rows=None, noise=None, cols=None):
        """(strip_w, H, 3) float64 like Scene.render; ``rows`` (reference row indices,
        y from the bottom) restricts the rendered rows (others stay 0), ``cols`` to the
        strip's first ``cols`` columns (a bounded CPU-baseline sample)."""
        W, H = self.width, self.height
        strip = np.array_split(np.arange(W), tasks)[subimage]
        dx = (self.right - self.left) / W
        dy = (self.top - self.bottom) / H
        ys = []
        y = self.bottom + 0.5 * dy
        for _ in range(H):
            ys.append(y)
            y += dy
        rows = range(H) if rows is None else rows
        img = np.zeros((len(strip), H, 3))
        divisor = self.samples * self.dof_samples * len(self.motion_times)
        nz = 0
        x = self.left + (0.5 + strip[0]) * dx
        for i in range(len(strip) if cols is None else min(cols, len(strip))):
            for j in rows:
                colour = ZERO
                base_dir = normalize(sub(add(scale(self.u, x), scale(self.v, ys[j])), scale(self.w, self.d)))
                focal = add(self.position, scale(base_dir, self.focal_length))
                for dof_origin in self.sunflower(self.dof_samples, self.position, self.aperture):
                    dof_dir = normalize(sub(focal, dof_origin))
                    for origin in self.sunflower(self.samples, dof_origin, 2 * (dx + dy)):
                        if self.jitter:
                            rnd = V(noise[nz], noise[nz + 1], noise[nz + 2])
                            nz += 3
                            origin = add(origin, scale(normalize(rnd), 0.1 * (dx + dy)))
                        for t in self.motion_times:
                            self.current_time = t
                            colour = add(colour, self.cast_ray(origin, dof_dir))
                img[i, j] = [float(c / f32(divisor)) for c in colour]
            x += dx
        return img
