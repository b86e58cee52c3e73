"""The HIP path (librtx.so on the MI355X) against reference-held data directly, with no
oracle in between:

- golden vectors the REFERENCE's own code produced (tests/golden/refvectors, made by
  tests/golden/make_refvectors.py): renders of boxes, CSG hierarchies, textures, random
  scenes and BASELINE config 5's AA2 x DOF32 jitter (the reference's seeded np.random
  stream replayed, scene.py:63-65), bit for bit, with the reference's ray tallies; and
  the reference's closest hit / any-hit shadow answers for seeded rays (scene.py:86-94,
  :161-164);
- the reference's published renders (renders/*.png) that are deterministic, at their
  native sizes: the uint8 PNG bytes must be identical (main.py:30-34)."""
import os

import numpy as np
import pytest
import torch

import refvectors as R
from common import product_scene, product_scene_dict

pytestmark = pytest.mark.gpu

PUB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "published")


@pytest.fixture(scope="module", autouse=True)
def _device():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    torch.cuda.set_device(0)


@pytest.mark.parametrize("name", R.names("render"))
def test_hip_equals_reference_render(name):
    fx = R.load("render", name)
    sc = product_scene_dict(R.scene(fx))
    sc.jitter_noise = R.noise(fx)
    img = sc.render(int(fx["subimage"]), int(fx["tasks"]))
    assert img.shape == fx["image"].shape
    diff = img != fx["image"]
    assert not diff.any(), "%s: %d of %d values differ (max %g), kernel %s" % (
        name, diff.sum(), diff.size, np.abs(img - fx["image"]).max(), sc.last_kernel)
    cnt = torch.zeros(16, dtype=torch.int64, device="cuda")
    sc.render_device(int(fx["subimage"]), int(fx["tasks"]), counters=cnt)
    c, t = cnt.cpu().numpy(), [int(x) for x in fx["tallies"]]
    assert list(c[:10]) == t[:10] and c[10] == t[11] and c[11] == t[12], (name, list(c), t)


@pytest.mark.parametrize("name", R.names("kat"))
def test_hip_equals_reference_closest_hit_and_shadow(name):
    fx = R.load("kat", name)
    sc = product_scene_dict(R.scene(fx))
    o, d, tmax = fx["o"], fx["d"], fx["tmax"]
    for ti, time in enumerate(fx["times"]):
        got = sc.intersect(o, d, float(time))
        ob = fx["t%d_closest_obj" % ti]
        hit = ob >= 0
        assert np.array_equal(got["obj"], ob), (name, time)
        assert np.array_equal(got["t"][hit], fx["t%d_closest_t" % ti][hit])
        assert np.array_equal(got["mat"], fx["t%d_closest_mat" % ti])
        assert np.array_equal(got["normal"][hit], fx["t%d_closest_normal" % ti][hit])
        assert np.array_equal(got["position"][hit], fx["t%d_closest_position" % ti][hit])
        assert np.array_equal(sc.occluded(o, d, tmax, float(time)), fx["t%d_occluded" % ti]), (name, time)


@pytest.mark.parametrize("scene,png,edits", [
    ("TwoSpheresPlane", "TwoSpheresPlane", {}),            # 640x480, AA 3
    ("MirrorRefraction", "MirrorRefraction", {}),          # 900x512, reflect/refract chains
    ("MotionBlur", "MotionBlur", {}),                      # 300x256, 17 motion times
    ("TorusMesh", "TorusMesh_flat", {}),                   # 256x256, flat mesh
    ("TorusMesh", "TorusMesh", {"flat_shaded": False}),    # 256x256, smooth normals
])
def test_hip_reproduces_published_render(scene, png, edits):
    from PIL import Image
    sc = product_scene(scene, **edits)
    got = sc.render_rgb8()
    want = np.asarray(Image.open(os.path.join(PUB, png + ".png")).convert("RGB"))
    assert got.shape == want.shape
    bad = (got != want).any(axis=2)
    assert not bad.any(), "%s: %d pixels differ (kernel %s)" % (png, bad.sum(), sc.last_kernel)
