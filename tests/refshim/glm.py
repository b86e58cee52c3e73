"""Test-only stand-in for PyGLM (not installed in this image), so the reference's own
Python modules can be imported in this container to build reference-shaped objects
(tests/golden/make_refobjects.py). float32 components, GLM operation order:
dot = (x*x + y*y) + z*z, normalize = v * (1 / sqrt(dot(v, v))). Every function the
reference calls is restated from GLM 0.9.9's generic code (which PyGLM wraps) with its
operation order, so the reference can also RENDER here to produce golden vectors
(tests/golden/make_refvectors.py): vec/mat arithmetic componentwise in fp32, mat4 * vec4
as (m0 x + m1 y) + (m2 z + m3 w), vec4 dot as (x*x + y*y) + (z*z + w*w), rotate with
libm cosf/sinf of the float angle, inverse by cofactors.
"""
import ctypes
import ctypes.util
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
    """GLM mat4 (float). ``m`` holds the matrix row-major as numpy float32: GLM's column
    c, component k is m[k, c]."""

    def __init__(self, diag=1.0):
        self.m = np.eye(4, dtype=f32) * f32(diag)

    @staticmethod
    def _wrap(m):
        o = mat4.__new__(mat4)
        o.m = np.asarray(m).astype(f32)
        return o

    def __mul__(self, o):
        m = self.m
        if isinstance(o, mat4):  # Result[i] = ((m1[0] * m2[i][0] + m1[1] * m2[i][1]) + m1[2] * m2[i][2]) + m1[3] * m2[i][3]
            r = np.empty((4, 4), f32)
            for i in range(4):
                b = o.m[:, i]
                r[:, i] = ((m[:, 0] * b[0] + m[:, 1] * b[1]) + m[:, 2] * b[2]) + m[:, 3] * b[3]
            return mat4._wrap(r)
        v = o.a  # GLM mat4 * vec4: (m[0] * v.x + m[1] * v.y) + (m[2] * v.z + m[3] * v.w)
        return vec4._wrap((m[:, 0] * v[0] + m[:, 1] * v[1]) + (m[:, 2] * v[2] + m[:, 3] * v[3]))


def dot(a, b):
    """GLM compute_dot: vec3 (x + y) + z, vec4 (x + y) + (z + w), in fp32."""
    p = a.a * b.a
    return float((p[0] + p[1]) + p[2]) if len(p) == 3 else float((p[0] + p[1]) + (p[2] + p[3]))


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
    """GLM translate: Result[3] = ((m[0] * v[0] + m[1] * v[1]) + m[2] * v[2]) + m[3]."""
    r = m.m.copy()
    r[:, 3] = ((m.m[:, 0] * v.a[0] + m.m[:, 1] * v.a[1]) + m.m[:, 2] * v.a[2]) + m.m[:, 3]
    return mat4._wrap(r)


def scale(m, v):
    """GLM scale: Result[i] = m[i] * v[i] for i < 3, Result[3] = m[3]."""
    r = m.m.copy()
    r[:, 0] *= v.a[0]
    r[:, 1] *= v.a[1]
    r[:, 2] *= v.a[2]
    return mat4._wrap(r)


_libm = ctypes.CDLL(ctypes.util.find_library("m"))
_libm.cosf.restype = _libm.sinf.restype = ctypes.c_float
_libm.cosf.argtypes = _libm.sinf.argtypes = [ctypes.c_float]


def rotate(m, angle, axis):
    """GLM 0.9.9 rotate(m, angle, v) with T = float: c = cos(a), s = sin(a) on the float
    angle (libm cosf / sinf), axis = normalize(v), temp = (1 - c) * axis, and
    Result[i] = (m[0] * R[i][0] + m[1] * R[i][1]) + m[2] * R[i][2]."""
    a = f32(angle)
    c, s = f32(_libm.cosf(a)), f32(_libm.sinf(a))
    ax = normalize(axis).a
    t = (f32(1) - c) * ax
    R = [[c + t[0] * ax[0], t[0] * ax[1] + s * ax[2], t[0] * ax[2] - s * ax[1]],
         [t[1] * ax[0] - s * ax[2], c + t[1] * ax[1], t[1] * ax[2] + s * ax[0]],
         [t[2] * ax[0] + s * ax[1], t[2] * ax[1] - s * ax[0], c + t[2] * ax[2]]]
    r = m.m.copy()
    for i in range(3):
        r[:, i] = (m.m[:, 0] * R[i][0] + m.m[:, 1] * R[i][1]) + m.m[:, 2] * R[i][2]
    return mat4._wrap(r)


def inverse(m):
    """GLM 0.9.9 compute_inverse<4, 4> (cofactors, then * (1 / determinant)), in fp32."""
    g = [[f32(m.m[k, c]) for k in range(4)] for c in range(4)]  # g[column][component]
    c00 = g[2][2] * g[3][3] - g[3][2] * g[2][3]
    c02 = g[1][2] * g[3][3] - g[3][2] * g[1][3]
    c03 = g[1][2] * g[2][3] - g[2][2] * g[1][3]
    c04 = g[2][1] * g[3][3] - g[3][1] * g[2][3]
    c06 = g[1][1] * g[3][3] - g[3][1] * g[1][3]
    c07 = g[1][1] * g[2][3] - g[2][1] * g[1][3]
    c08 = g[2][1] * g[3][2] - g[3][1] * g[2][2]
    c10 = g[1][1] * g[3][2] - g[3][1] * g[1][2]
    c11 = g[1][1] * g[2][2] - g[2][1] * g[1][2]
    c12 = g[2][0] * g[3][3] - g[3][0] * g[2][3]
    c14 = g[1][0] * g[3][3] - g[3][0] * g[1][3]
    c15 = g[1][0] * g[2][3] - g[2][0] * g[1][3]
    c16 = g[2][0] * g[3][2] - g[3][0] * g[2][2]
    c18 = g[1][0] * g[3][2] - g[3][0] * g[1][2]
    c19 = g[1][0] * g[2][2] - g[2][0] * g[1][2]
    c20 = g[2][0] * g[3][1] - g[3][0] * g[2][1]
    c22 = g[1][0] * g[3][1] - g[3][0] * g[1][1]
    c23 = g[1][0] * g[2][1] - g[2][0] * g[1][1]
    f0, f1, f2 = [c00, c00, c02, c03], [c04, c04, c06, c07], [c08, c08, c10, c11]
    f3, f4, f5 = [c12, c12, c14, c15], [c16, c16, c18, c19], [c20, c20, c22, c23]
    v0 = [g[1][0], g[0][0], g[0][0], g[0][0]]
    v1 = [g[1][1], g[0][1], g[0][1], g[0][1]]
    v2 = [g[1][2], g[0][2], g[0][2], g[0][2]]
    v3 = [g[1][3], g[0][3], g[0][3], g[0][3]]
    sa, sb = [f32(1), f32(-1), f32(1), f32(-1)], [f32(-1), f32(1), f32(-1), f32(1)]
    inv = [[None] * 4 for _ in range(4)]
    for k in range(4):
        inv[0][k] = ((v1[k] * f0[k] - v2[k] * f1[k]) + v3[k] * f2[k]) * sa[k]
        inv[1][k] = ((v0[k] * f0[k] - v2[k] * f3[k]) + v3[k] * f4[k]) * sb[k]
        inv[2][k] = ((v0[k] * f1[k] - v1[k] * f3[k]) + v3[k] * f5[k]) * sa[k]
        inv[3][k] = ((v0[k] * f2[k] - v1[k] * f4[k]) + v2[k] * f5[k]) * sb[k]
    d = [g[0][k] * inv[k][0] for k in range(4)]
    one_over = f32(1) / ((d[0] + d[1]) + (d[2] + d[3]))
    r = np.empty((4, 4), f32)
    for c in range(4):
        for k in range(4):
            r[k, c] = inv[c][k] * one_over
    return mat4._wrap(r)


def transpose(m):
    return mat4._wrap(m.m.T.copy())
