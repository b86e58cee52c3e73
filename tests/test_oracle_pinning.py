"""The oracle is pinned against the reference's published renders (renders/*.png,
committed as tests/golden/published/). SURVEY.md §4 lists which renders are pinnable."""
import os

import numpy as np
import pytest
from PIL import Image

from common import oracle_render
from oracle import oracle as O

PUB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "published")


def _png(name):
    return np.asarray(Image.open(os.path.join(PUB, name + ".png")).convert("RGB"))


@pytest.mark.parametrize("scene,render,edits", [
    ("TwoSpheresPlane", "TwoSpheresPlane", {}),            # 640x480, 3 spp AA
    ("MirrorRefraction", "MirrorRefraction", {}),          # reflect/refract chains
    ("MotionBlur", "MotionBlur", {}),                      # 17 motion samples
    ("TorusMesh", "TorusMesh_flat", {}),                   # flat mesh, AABB bounding volume
    ("TorusMesh", "TorusMesh", {"flat_shaded": False}),    # smooth normals
])
def test_oracle_reproduces_published_render(scene, render, edits):
    img = oracle_render(scene, **edits)
    png = O.to_png_array(img)
    ref = _png(render)
    assert png.shape == ref.shape
    assert np.array_equal(png, ref), "%.4f%% pixels differ" % (100 * (png != ref).any(axis=2).mean())


def test_oracle_depth_of_field_statistical():
    """DepthOfField.png used an unseeded RNG for jitter: compare statistically."""
    rng = np.random.RandomState(1)
    img = oracle_render("DepthOfField", noise=rng.rand(256 * 256 * 32 * 3))
    d = O.to_png_array(img).astype(int) - _png("DepthOfField").astype(int)
    assert np.abs(d).mean() < 0.25      # mean |delta| in LSB (measured 0.127)
    assert abs(d.mean()) < 0.05         # unbiased
    assert (np.abs(d).max(axis=2) == 0).mean() > 0.9


def test_oracle_tallies_match_survey_appendix_c():
    """Rays per primary sample (measured on the reference)."""
    _, t = oracle_render("TwoSpheresPlane", res=(192, 108), AA={"jitter": False, "samples": 1}, tallies=True)
    n = 192 * 108
    assert t[0] == n and abs(t[11] / n - 1.796) < 1e-3 and abs(t[12] / n - 0.898) < 1e-3
    _, t = oracle_render("MirrorRefraction", res=(192, 108), tallies=True)
    assert abs(t[1] / n - 0.326) < 1e-3 and abs(t[2] / n - 0.182) < 1e-3 and abs(t[11] / n - 1.241) < 1e-3
    _, t = oracle_render("TorusMesh", res=(192, 108), tallies=True)
    assert t[11] == 3 * n and t[12] == n


def _novel_strip(args):
    name, tasks, k, seed = args
    d, base = O.load_bundle(name)
    sc = O.OracleScene(d, base)
    base_, extra = divmod(sc.width, tasks)
    ncol = base_ + (1 if k < extra else 0)
    c0 = k * base_ + min(k, extra)
    noise = np.random.RandomState(seed).rand(ncol * sc.height * sc.spp_rays * 3)
    return c0, O.to_png_array(sc.render(k, tasks, noise=noise))


@pytest.mark.parametrize("name,tasks,strips,max_mean", [
    ("NovelScene1", 64, (30, 33), 0.1),   # 2048x1024, AA 32 jittered: hierarchies + textures
    ("NovelScene2", 128, (64,), 0.2),     # 1024x512, AA 2 x DOF 15 x 16 motion times
])
def test_oracle_novel_scenes_statistical(name, tasks, strips, max_mean):
    """NovelScene1/2.png (CSG hierarchies, `ref` copies, fallback materials, plane
    textures; NovelScene2 also motion blur through hierarchies and DOF) used unseeded
    jitter: column strips through the bikes compare statistically (full-frame check:
    tools/pin_novel.py, 98.7% / 97% of pixels identical)."""
    from multiprocessing import Pool
    ref = _png(name)
    with Pool(len(strips)) as pool:
        outs = pool.map(_novel_strip, [(name, tasks, k, 100 + k) for k in strips])
    for c0, png in outs:
        d = png.astype(int) - ref[:, c0:c0 + png.shape[1]].astype(int)
        assert np.abs(d).mean() < max_mean, (name, c0, np.abs(d).mean())
        assert abs(d.mean()) < 0.05
        assert (np.abs(d).max(axis=2) == 0).mean() > 0.93
