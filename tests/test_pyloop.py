"""The pure-Python restatement of the reference's render loop (oracle/pyloop.py, the
CPU baseline the north star names) is bit-identical to the C oracle (itself pinned to the
reference's published renders) on small frames of every benchmark scene."""
import numpy as np
import pytest

from oracle import oracle as O
from oracle import pyloop as P

CASES = [
    ("TwoSpheresPlane", (24, 16), {}),
    ("TwoSpheresPlane", (11, 7), {"AA": {"jitter": False, "samples": 3}}),
    ("MirrorRefraction", (32, 18), {}),
    ("TorusMesh", (16, 16), {}),
    ("MotionBlur", (12, 10), {}),
    ("DepthOfField", (8, 6), {"AA": {"jitter": False, "samples": 2}}),
]


def scenes(name, res, edits):
    d, base = O.load_bundle(name, resolution=list(res), **edits)
    osc = O.OracleScene(d, base)
    return osc, P.PyLoopScene(osc)


@pytest.mark.parametrize("name,res,edits", CASES)
def test_pyloop_equals_oracle(name, res, edits):
    osc, ps = scenes(name, res, edits)
    assert np.array_equal(ps.render(), osc.render())


def test_pyloop_smooth_mesh_and_strips():
    d, base = O.load_bundle("TorusMesh", resolution=[12, 12])
    for g in d["objects"]:
        if g["type"] == "mesh":
            g["flat_shaded"] = False
    osc = O.OracleScene(d, base)
    ps = P.PyLoopScene(osc)
    for k in range(3):
        assert np.array_equal(ps.render(k, 3), osc.render(k, 3))


def test_pyloop_jitter_replay_and_row_subset():
    osc, ps = scenes("DepthOfField", (6, 5), {"AA": {"jitter": True, "samples": 2}})
    noise = np.random.RandomState(2).rand(6 * 5 * 2 * 32 * 3)
    assert np.array_equal(ps.render(noise=noise), osc.render(noise=noise))
    osc, ps = scenes("MirrorRefraction", (20, 12), {})
    part = ps.render(rows=[0, 5, 11])
    full = osc.render()
    assert np.array_equal(part[:, [0, 5, 11]], full[:, [0, 5, 11]])


@pytest.mark.parametrize("name,res", [("NovelScene1", (24, 12)), ("NovelScene2", (4, 2))])
def test_pyloop_hierarchies_and_textures_equal_oracle(name, res):
    """CSG hierarchies (GLM mat4 restated in Python floats) and plane / box textures."""
    d, base = O.load_bundle(name, resolution=list(res), AA={"jitter": False, "samples": 1})
    osc = O.OracleScene(d, base)
    assert np.array_equal(P.PyLoopScene(osc).render(), osc.render())


@pytest.mark.parametrize("seed", range(6))
def test_pyloop_random_hierarchy_scenes_equal_oracle(seed):
    import os
    from scenegen import random_hier_scene
    d = random_hier_scene(seed, res=(20, 15), mesh=(seed % 4 == 0))
    osc = O.OracleScene(d, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets"))
    assert np.array_equal(P.PyLoopScene(osc).render(), osc.render())


def _config1_strip(k):
    d, base = O.load_bundle("TwoSpheresPlane", resolution=[256, 256], AA={"jitter": False, "samples": 1})
    return P.PyLoopScene(O.OracleScene(d, base)).render(k, 4)


def test_config1_tsp256_python_loop_equals_reference():
    """BASELINE config 1 (TwoSpheresPlane 256x256, 1 spp, the reference's CPU path) at its
    stated size: the Python loop, run as 4 column-strip processes like render.nu, glued,
    equals the reference's own render (tests/golden/refvectors/render_tsp256_config1.npz)
    and the C oracle, bit for bit."""
    from multiprocessing import get_context

    import refvectors as R
    with get_context("fork").Pool(4) as pool:
        img = np.concatenate(pool.map(_config1_strip, range(4)), axis=0)
    fx = R.load("render", "tsp256_config1")
    assert np.array_equal(img, fx["image"])
    d, base = O.load_bundle("TwoSpheresPlane", resolution=[256, 256], AA={"jitter": False, "samples": 1})
    assert np.array_equal(O.OracleScene(d, base).render(), fx["image"])
