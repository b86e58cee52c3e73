"""The production jitter stream (Philox4x32-10, include/rtx.h RTX_JITTER_PHILOX), pinned on
the CPU: the numpy restatement (oracle/philox.py) against Random123's known-answer
vectors, the device source (rtx_trace.h philox4x32, rtx_kernels.h jitter_block /
jitter_rnd, built for the host) against both, and whole jittered frames of the device
source against the oracle fed with the restated stream. The reference's jitter itself is
provided/scene.py:63-65 (unseeded np.random draws); tests/test_gpu_parity.py runs the
same frame comparisons on the MI355X."""
import numpy as np
import pytest

import hostemu
from common import assert_parity, oracle_render, product_scene
from oracle import philox as PH

SEED = 0x5EED  # rtx.scene.DEFAULT_SEED


@pytest.mark.parametrize("ctr,key,want", PH.KAT)
def test_restatement_known_answers(ctr, key, want):
    assert tuple(int(x) for x in PH.philox4x32_10(np.array([ctr], np.uint32), key)[0]) == want


@pytest.mark.parametrize("ctr,key,want", PH.KAT)
def test_device_philox_known_answers(ctr, key, want):
    assert tuple(int(x) for x in hostemu.philox(ctr, key)) == want


def test_device_philox_equals_restatement_random_counters():
    rng = np.random.RandomState(1)
    ctr = rng.randint(0, 2 ** 32, size=(200, 4), dtype=np.uint64).astype(np.uint32)
    for key in ((0, 0), (SEED, 0), (0xDEADBEEF, 0x12345678)):
        want = PH.philox4x32_10(ctr, key)
        got = np.stack([hostemu.philox(c, key) for c in ctr])
        assert np.array_equal(got, want)


@pytest.mark.parametrize("seed,col0,ncols,height,n_dof,n_aa", [
    (SEED, 0, 5, 7, 32, 2),          # DepthOfField's 64 samples
    (SEED, 3000, 1, 40, 32, 2),      # a column of BASELINE config 5 (subimage 3000 of 3840)
    (SEED, 17, 3, 4, 1, 3),          # odd sample count: the last sample is an even half alone
    (SEED, 0, 4, 4, 15, 2),          # NovelScene2's DOF 15 x AA 2
    (0x123456789ABCDEF, 11, 2, 3, 5, 1),  # both key words used
])
def test_device_jitter_stream_equals_restatement(seed, col0, ncols, height, n_dof, n_aa):
    got = hostemu.jitter(seed, col0, ncols, height, n_dof, n_aa)
    want = PH.jitter_noise(seed, col0, ncols, height, n_dof, n_aa)
    assert np.array_equal(got.astype(np.float64), want)
    # the uniforms are multiples of 2^-21 in [0, 1), so the fp32 table is exact
    assert np.array_equal(want * 2.0 ** 21, np.floor(want * 2.0 ** 21)) and want.min() >= 0 and want.max() < 1


def test_halves_use_disjoint_bits():
    """Half 0 and half 1 of a block read disjoint bits: flipping any one bit of the block
    changes exactly one of the six 21-bit integers, in exactly one bit."""
    rng = np.random.RandomState(2)
    blk = rng.randint(0, 2 ** 32, size=(1, 4), dtype=np.uint64).astype(np.uint32)
    base = np.concatenate([PH.sample_uniforms(blk, [0]), PH.sample_uniforms(blk, [1])], axis=-1)[0]
    used = 0
    for w in range(4):
        for b in range(32):
            f = blk.copy()
            f[0, w] ^= np.uint32(1 << b)
            new = np.concatenate([PH.sample_uniforms(f, [0]), PH.sample_uniforms(f, [1])], axis=-1)[0]
            changed = np.nonzero(new != base)[0]
            if w == 3 and b >= 30:  # bits 30-31 of word 3 are not used
                assert changed.size == 0
                continue
            assert changed.size == 1
            assert bin(int(new[changed[0]] ^ base[changed[0]])).count("1") == 1
            used += 1
    assert used == 6 * 21


def _philox_frame(name, res, edits, subimage=0, tasks=1):
    sc = product_scene(name, res, **edits)
    assert sc.jitter and sc.jitter_noise is None and sc.seed == SEED  # production mode
    W, H = res
    col0 = sum(len(c) for c in np.array_split(np.arange(W), tasks)[:subimage])
    ncols = len(np.array_split(np.arange(W), tasks)[subimage])
    noise = PH.jitter_noise(SEED, col0, ncols, H, sc.vc.dof_samples, sc.samples)
    img, _ = hostemu.render(sc, subimage, tasks)
    ref = oracle_render(name, res, subimage=subimage, tasks=tasks, noise=noise, **edits)
    return img, ref


@pytest.mark.parametrize("name,res,edits,subimage,tasks", [
    ("DepthOfField", (24, 18), {"AA": {"jitter": True, "samples": 2}}, 0, 1),
    ("DepthOfField", (64, 48), {"AA": {"jitter": True, "samples": 2}}, 5, 8),   # col0 = 40
    ("TwoSpheresPlane", (33, 21), {"AA": {"jitter": True, "samples": 3}}, 0, 1),  # odd sample count
])
def test_hostemu_philox_frames_equal_oracle(name, res, edits, subimage, tasks):
    img, ref = _philox_frame(name, res, edits, subimage, tasks)
    assert assert_parity(img, ref, name)["frac_diff"] == 0.0
