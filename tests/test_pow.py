"""`x ** hardness` (provided/scene.py:181: `max(0, dot(normal, half_vect)) ** hardness`,
CPython float_pow -> libm pow, then the fp32 vec3 scale) as the kernels evaluate it
(csrc/rtx_trace.h spec_pow: fp64 binary exponentiation, with a double-double recompute
for lanes whose result lies within the error bound of an fp32 rounding boundary).

Dense check: every integer hardness 0..128 (the bundled scenes use 0, 2, 16, 32, 50, 64
and 100) on 10^6 fp32 bases in [0, 1], half of them in [0.95, 1] where high exponents
keep the result in range, plus edge values. The reference is numpy's float64 power with
an array exponent (libm pow, as CPython's `**`; checked against `**` on a sub-sample).
The host emulation (CPU) and the MI355X (-m gpu) must both give 0 mismatches; the fp64
binary exponentiation alone misses 2 of these 1.29e8 values, which the test asserts too,
so the recompute branch is exercised."""
import ctypes as C
import os

import numpy as np
import pytest

import hostemu

HARDNESS = list(range(0, 129))
# the fp64 binary exponentiation alone rounds these to the wrong fp32 (exponent, base bits)
KNOWN_BOUNDARY = [(34, 0x3DC70AF8), (77, 0x3F76B0BC)]


def bases():
    rng = np.random.default_rng(1)
    n = 1_000_000
    x = np.concatenate([rng.random(n // 2, dtype=np.float32),
                        (1 - rng.random(n // 2, dtype=np.float32) * 0.05).astype(np.float32)])
    edge = np.array([0.0, 1.0, np.nextafter(np.float32(1), np.float32(2)), np.nextafter(np.float32(1), np.float32(0)),
                     np.float32(1e-45), np.float32(1.17549435e-38), 0.5, 0.25], np.float32)
    known = np.array([b for _, b in KNOWN_BOUNDARY], np.uint32).view(np.float32)
    return np.concatenate([x, edge, known])


def reference(x, n):
    """fl32(libm pow(fl64(x), n))."""
    x64 = x.astype(np.float64)
    return np.power(x64, np.full_like(x64, float(n))).astype(np.float32)


def binexp_only(x, n):
    """The fast path without its boundary check (numpy restatement of the loop)."""
    r = np.ones(x.shape, np.float64)
    b = x.astype(np.float64)
    while n:
        if n & 1:
            r = r * b
        b = b * b
        n >>= 1
    return r.astype(np.float32)


def host_spec_pow(x, n):
    out = np.empty_like(x)
    f = hostemu.lib().rtx_hostemu_spec_pow
    f.argtypes = [C.c_void_p, C.c_int64, C.c_int32, C.c_void_p, C.c_int]
    f.restype = None
    f(x.ctypes.data, x.size, n, out.ctypes.data, 8)
    return out


def mismatches(fn, x):
    bad = []
    for n in HARDNESS:
        got = fn(x, n)
        ref = reference(x, n)
        m = np.nonzero(got.view(np.uint32) != ref.view(np.uint32))[0]
        bad += [(n, float(x[i]), float(got[i]), float(ref[i])) for i in m[:5]]
    return bad


def test_reference_is_cpython_pow():
    x = bases()[::997]
    for n in (0, 2, 16, 34, 50, 77, 100, 128):
        ref = reference(x, n)
        py = np.array([float(v) ** n for v in x.astype(np.float64)]).astype(np.float32)
        assert np.array_equal(ref.view(np.uint32), py.view(np.uint32)), n


def test_binary_exponentiation_alone_misses_known_boundaries():
    for n, b in KNOWN_BOUNDARY:
        x = np.array([b], np.uint32).view(np.float32)
        assert binexp_only(x, n)[0] != reference(x, n)[0], (n, hex(b))


def test_spec_pow_host_dense():
    bad = mismatches(host_spec_pow, bases())
    assert not bad, bad


@pytest.mark.gpu
def test_spec_pow_gpu_dense():
    import torch
    assert torch.cuda.is_available()
    path = os.path.join(os.path.dirname(__file__), "native", "librtx_mathcheck.so")
    assert os.path.exists(path), "build it first: make -C tests/native (__graft_entry__.build does)"
    lib = C.CDLL(path)
    lib.rtx_powcheck.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_void_p]

    def dev(x, n):
        out = np.empty_like(x)
        assert lib.rtx_powcheck(x.ctypes.data, x.size, n, out.ctypes.data) == 0
        return out
    bad = mismatches(dev, bases())
    assert not bad, bad
