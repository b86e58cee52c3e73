"""Test-only stand-in for PyGLM (not installed in this image), so the reference's own
Python modules can be imported in this container to build reference-shaped objects
(tests/golden/make_refobjects.py). float32 components, GLM operation order:
dot = (x*x + y*y) + z*z, normalize = v * (1 / sqrt(dot(v, v))). Only what
/root/reference/provided calls at scene-construction time is needed to be exact; the
render-time functions are included so the modules import and run.
"""
import math

import numpy as np

f32 = np.float32


class _Vec:
    N = 3
    __slots__ = ("a",)
    __array_ufunc__ = None  # numpy scalars defer to the vector ops (NumPy-1.x float32 semantics)

    def __init__(self, *args):
        if not args:
            self.a = np.zeros(self.N, f32)
            return
        vals = []
        for x in args:
            if isinstance(x, _Vec):
                vals.extend(x.a.tolist())
            elif isinstance(x, (list, tuple, np.ndarray)):
                vals.extend(np.asarray(x, np.float64).ravel().tolist())
            else:
                vals.append(float(x))
        if len(vals) == 1:
            vals = vals * self.N
        self.a = np.array(vals[:self.N], dtype=np.float64).astype(f32)

    @classmethod
    def _wrap(cls, a):
        o = cls.__new__(cls)
        o.a = np.asarray(a).astype(f32, copy=False)
        return o

    @staticmethod
    def _other(o):
        return o.a if isinstance(o, _Vec) else f32(o)

    def __add__(self, o):
        return self._wrap(self.a + self._other(o))
    __radd__ = __add__

    def __sub__(self, o):
        return self._wrap(self.a - self._other(o))

    def __rsub__(self, o):
        return self._wrap(self._other(o) - self.a)

    def __mul__(self, o):
        return self._wrap(self.a * self._other(o))
    __rmul__ = __mul__

    def __truediv__(self, o):
        return self._wrap(self.a / self._other(o))

    def __neg__(self):
        return self._wrap(-self.a)

    def __eq__(self, o):
        return isinstance(o, _Vec) and bool(np.all(self.a == o.a))

    def __hash__(self):
        return hash(self.a.tobytes())

    def __getitem__(self, i):
        return float(self.a[i])

    def __iter__(self):
        return iter(self.a.tolist())

    def __len__(self):
        return self.N

    def __array__(self, dtype=None, copy=None):
        return self.a.astype(dtype or f32)

    def __repr__(self):
        return "vec%d(%s)" % (self.N, ", ".join("%g" % v for v in self.a))

    x = property(lambda s: float(s.a[0]))
    y = property(lambda s: float(s.a[1]))
    z = property(lambda s: float(s.a[2]))


class vec3(_Vec):
    N = 3


class vec4(_Vec):
    N = 4
    w = property(lambda s: float(s.a[3]))
    xyz = property(lambda s: vec3._wrap(s.a[:3].copy()))


class mat4:
    def __init__(self, diag=1.0):
        self.m = np.eye(4, dtype=f32) * f32(diag)

    @staticmethod
    def _wrap(m):
        o = mat4.__new__(mat4)
        o.m = np.asarray(m).astype(f32)
        return o

    def __mul__(self, o):
        if isinstance(o, mat4):
            return mat4._wrap(self.m @ o.m)
        return vec4._wrap(self.m @ o.a)


def dot(a, b):
    p = a.a * b.a
    return float((p[0] + p[1]) + p[2]) if len(p) == 3 else float(((p[0] + p[1]) + p[2]) + p[3])


def cross(a, b):
    x, y = a.a, b.a
    return vec3._wrap(np.array([x[1] * y[2] - y[1] * x[2], x[2] * y[0] - y[2] * x[0], x[0] * y[1] - y[0] * x[1]]))


def length(v):
    return float(np.sqrt(f32(dot(v, v))))


def normalize(v):
    with np.errstate(all="ignore"):
        return type(v)._wrap(v.a * (f32(1.0) / np.sqrt(f32(dot(v, v)))))


def reflect(i, n):
    return i - n * f32(dot(n, i) * 2.0)


def refract(i, n, eta):
    d, e = f32(dot(n, i)), f32(eta)
    k = f32(1) - e * e * (f32(1) - d * d)
    if k < 0:
        return vec3()
    return vec3._wrap(e * i.a - (e * d + np.sqrt(k)) * n.a)


def radians(x):
    return math.radians(x)


def tan(x):
    return math.tan(x)


def translate(m, v):
    r = m.m.copy()
    r[:, 3] = m.m[:, 0] * v.a[0] + m.m[:, 1] * v.a[1] + m.m[:, 2] * v.a[2] + m.m[:, 3]
    return mat4._wrap(r)


def scale(m, v):
    r = m.m.copy()
    r[:, 0] *= v.a[0]
    r[:, 1] *= v.a[1]
    r[:, 2] *= v.a[2]
    return mat4._wrap(r)


def rotate(m, angle, axis):
    c, s = math.cos(angle), math.sin(angle)
    a = axis.a / np.linalg.norm(axis.a)
    t = (1 - c) * a
    r = np.eye(4, dtype=f32)
    r[0, 0], r[1, 0], r[2, 0] = c + t[0] * a[0], t[0] * a[1] + s * a[2], t[0] * a[2] - s * a[1]
    r[0, 1], r[1, 1], r[2, 1] = t[1] * a[0] - s * a[2], c + t[1] * a[1], t[1] * a[2] + s * a[0]
    r[0, 2], r[1, 2], r[2, 2] = t[2] * a[0] + s * a[1], t[2] * a[1] - s * a[0], c + t[2] * a[2]
    return mat4._wrap(m.m @ r)


def inverse(m):
    return mat4._wrap(np.linalg.inv(m.m.astype(np.float64)))


def transpose(m):
    return mat4._wrap(m.m.T.copy())
