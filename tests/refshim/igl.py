"""Test-only stand-in for libigl's read_obj (not installed in this image): the six-tuple
mesh.py:20 unpacks (V, TC, N, F, FTC, FN), 0-based triangle faces."""
import numpy as np


def read_obj(path):
    v, n, f = [], [], []
    with open(path) as fh:
        for line in fh:
            p = line.split()
            if not p:
                continue
            if p[0] == "v":
                v.append([float(x) for x in p[1:4]])
            elif p[0] == "vn":
                n.append([float(x) for x in p[1:4]])
            elif p[0] == "f":
                f.append([int(x.split("/")[0]) - 1 for x in p[1:4]])
    return (np.array(v, dtype=np.float64).reshape(-1, 3), np.zeros((0, 2)), np.array(n, dtype=np.float64).reshape(-1, 3),
            np.array(f, dtype=np.int64).reshape(-1, 3), None, None)


def barycentric_coordinates_tri(p, a, b, c):
    v0, v1, v2 = b - a, c - a, p - a
    d00, d01, d11 = (v0 * v0).sum(), (v0 * v1).sum(), (v1 * v1).sum()
    d20, d21 = (v2 * v0).sum(), (v2 * v1).sum()
    den = d00 * d11 - d01 * d01
    v = (d11 * d20 - d01 * d21) / den
    w = (d00 * d21 - d01 * d20) / den
    return np.array([1 - v - w, v, w])
