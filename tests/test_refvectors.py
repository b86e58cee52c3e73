"""The oracle against golden vectors produced by the REFERENCE's own code
(tests/golden/refvectors, made by tests/golden/make_refvectors.py): bit-exact renders of
boxes (DepthOfField's AA2 x DOF32 jitter replayed from the reference's seeded np.random
stream), CSG hierarchies, textures and random scenes, with the reference's ray tallies,
and per-object known answers of intersect / shadow_intersect / is_inside
(provided/geometry/*.py) and the scene's closest hit (provided/scene.py:86-94)."""
import numpy as np
import pytest

import refvectors as R
from common import oracle_render_dict

from oracle import oracle as O


@pytest.mark.parametrize("name", R.names("render"))
def test_oracle_equals_reference_render(name):
    fx = R.load("render", name)
    img, tl = oracle_render_dict(R.scene(fx), int(fx["subimage"]), int(fx["tasks"]), noise=R.noise(fx), tallies=True)
    assert img.shape == fx["image"].shape
    diff = img != fx["image"]
    assert not diff.any(), "%s: %d of %d values differ (max %g)" % (
        name, diff.sum(), diff.size, np.abs(img - fx["image"]).max())
    assert list(tl) == [int(x) for x in fx["tallies"]], (name, list(tl), list(fx["tallies"]))


def _oracle(fx):
    import os
    base = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets")
    return O.OracleScene(R.scene(fx), base)


@pytest.mark.parametrize("name", R.names("kat"))
def test_oracle_equals_reference_kat(name):
    fx = R.load("kat", name)
    osc = _oracle(fx)
    roots = osc.roots
    assert len(roots) == int(fx["nobj"])
    o, d, tmax = fx["o"], fx["d"], fx["tmax"]
    for ti, time in enumerate(fx["times"]):
        pts = fx["t%d_points" % ti]
        for k, rec in enumerate(roots):
            for i in range(len(o)):
                want = R.hits(fx, ti, k, i)
                got = osc.object_intersect(rec, time, o[i], d[i])
                assert len(got[0]) == len(want[0]), (name, time, k, i, got[0], want[0])
                for g, w in zip(got[:4], want):
                    assert np.array_equal(g, w), (name, time, k, i, g, w)
            assert np.array_equal(osc.object_shadow(rec, time, o, d, tmax), fx["t%d_obj%d_shadow" % (ti, k)]), (name, k)
            assert np.array_equal(osc.object_inside(rec, time, pts), fx["t%d_obj%d_inside" % (ti, k)]), (name, k)
        t, ob, _, m, nn, pp = osc.closest(time, o, d)
        assert np.array_equal(ob, fx["t%d_closest_obj" % ti])
        assert np.array_equal(t, fx["t%d_closest_t" % ti]) and np.array_equal(m, fx["t%d_closest_mat" % ti])
        assert np.array_equal(nn, fx["t%d_closest_normal" % ti])
        assert np.array_equal(pp, fx["t%d_closest_position" % ti])
        assert np.array_equal(osc.shadow(time, o, d, tmax).astype(bool), fx["t%d_occluded" % ti])


def test_fixture_coverage():
    """The vectors cover what only jittered published renders covered before: boxes,
    hierarchies (every node type), textures, BASELINE config 5's AA2 x DOF32 jitter."""
    kinds = set()
    for name in R.names("render"):
        d = R.scene(R.load("render", name))

        def walk(objs):
            for g in objs:
                kinds.add(g["type"])
                if "texture" in g:
                    kinds.add("texture_" + g["type"])
                if g["type"] == "node":
                    kinds.add("node_" + g.get("hierarchy_type", "union"))
                    walk(g.get("children", []))
        walk(d["objects"])
    for k in ("box", "texture_box", "texture_plane", "node_union", "node_intersection", "node_difference", "mesh"):
        assert k in kinds, k
    fx = R.load("render", "dof_aa2_jitter")
    assert R.scene(fx)["AA"] == {"jitter": True, "samples": 2} and R.scene(fx)["DOF"]["samples"] == 32
