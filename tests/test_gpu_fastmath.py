"""The fast correctly rounded fp32 sqrt / reciprocal of csrc/rtx_fastmath.h (used by the
render kernels' normalize for dot products in [2^-100, 2^100]) against IEEE sqrtf and
1.0f / x for EVERY fp32 significand of every binade in that range, on the MI355X."""
import ctypes as C
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

LIB = os.path.join(os.path.dirname(__file__), "native", "librtx_mathcheck.so")


def test_fast_sqrt_and_reciprocal_are_ieee_exhaustive():
    assert torch.cuda.is_available()
    assert os.path.exists(LIB), "build it first: make -C tests/native (__graft_entry__.build does)"
    lib = C.CDLL(LIB)
    lib.rtx_mathcheck.argtypes = [C.c_int, C.c_void_p]
    bad = np.zeros(2, np.uint64)
    total = np.zeros(3, np.uint64)
    for e in range(-100, 99, 2):  # x in [2^e, 2^(e+2)): 2^24 values per launch
        out = np.zeros(3, np.uint64)
        assert lib.rtx_mathcheck(e, out.ctypes.data) == 0
        total += out
        bad[0] += out[0] > 0
        bad[1] += out[1] > 0
    assert total[2] > 0, "harness self-check: raw v_rcp_f32 should differ from 1/x somewhere"
    assert total[0] == 0, "sqrt_rn differs from sqrtf on %d inputs (%d binade pairs)" % (total[0], bad[0])
    assert total[1] == 0, "rcp_rn differs from 1/x on %d inputs (%d binade pairs)" % (total[1], bad[1])
