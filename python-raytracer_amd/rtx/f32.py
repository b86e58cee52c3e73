"""fp32 vec3 helpers with PyGLM's operation order, for host-side precomputation.

The reference does its vector math with PyGLM (float32 components); Python scalars are
float64 and are cast to float32 when they multiply a vec3. These helpers reproduce that
on numpy float32 values (numpy float32 ufuncs are single IEEE operations, never fused).
Vectorised forms take arrays of shape (..., 3).
"""
import numpy as np

f32 = np.float32


def vec3(x, y=None, z=None):
    if y is None:
        return np.asarray(x, dtype=np.float64).astype(f32).reshape(3)
    return np.array([x, y, z], dtype=np.float64).astype(f32)


def dot(a, b):
    """glm::dot: (x*x + y*y) + z*z in fp32 (vectorised over leading axes)."""
    p = np.asarray(a, f32) * np.asarray(b, f32)
    return (p[..., 0] + p[..., 1]) + p[..., 2]


def cross(a, b):
    a = np.asarray(a, f32)
    b = np.asarray(b, f32)
    return np.stack([a[..., 1] * b[..., 2] - b[..., 1] * a[..., 2],
                     a[..., 2] * b[..., 0] - b[..., 2] * a[..., 0],
                     a[..., 0] * b[..., 1] - b[..., 0] * a[..., 1]], axis=-1)


def length(v):
    return np.sqrt(dot(v, v))


def normalize(v):
    """glm::normalize = v * (1 / sqrt(dot(v, v)))."""
    v = np.asarray(v, f32)
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = f32(1.0) / np.sqrt(dot(v, v))
    return v * np.asarray(inv, f32)[..., None]


def scale(v, s):
    """vec3 * Python scalar: the scalar is cast to float32 first."""
    return np.asarray(v, f32) * f32(s)
