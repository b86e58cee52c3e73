"""The reference-side binding: a Scene built by the reference's own
scene_parser (provided/scene_parser.py:50-163) — its classes and attribute names:
Mesh.verts/faces/norms/bounding_volume (mesh.py:17-51), Plane.point/normal/texture
(simple_geometry.py:87-103), AABB.minpos/maxpos (:180-186), Hierarchy.t/r/s/children
(hierarchy.py:12-40), PyGLM vectors — bound through rtx.Scene.from_reference, must give
the C ABI exactly the descriptor and camera tables rtx.load_scene gives for the same JSON.

The reference-shaped objects come from tests/golden/refobjects.json (written by
tests/golden/make_refobjects.py, which imports the reference itself); where the reference
snapshot is mounted the fixture is also regenerated and compared."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import refobjects as R
import rtx
from rtx import _native as N
from rtx.records import desc_bytes, kind

HERE = os.path.dirname(os.path.abspath(__file__))


def product(name, res):
    return rtx.load_bundled_scene(name, resolution=res)


@pytest.mark.parametrize("name", R.names())
def test_reference_objects_give_the_same_descriptor(name):
    ref, res = R.load(name)
    assert type(ref).__name__ == "Scene" and type(ref.vc).__name__ == "ViewportCamera"
    bound = rtx.Scene.from_reference(ref)
    ours = product(name, res)
    a, b = desc_bytes(bound.scene_desc()), desc_bytes(ours.scene_desc())
    assert len(a) == len(b)
    for k, (x, y) in enumerate(zip(a, b)):
        assert x == y, (name, k)


@pytest.mark.parametrize("name", R.names())
def test_reference_camera_gives_the_same_tables(name):
    ref, res = R.load(name)
    bound, ours = rtx.Scene.from_reference(ref), product(name, res)
    for sub, tasks in ((0, 1), (1, 3)):
        ta, tb = bound.camera_tables(sub, tasks), ours.camera_tables(sub, tasks)
        assert ta.keys() == tb.keys()
        for k in ta:
            assert np.array_equal(np.asarray(ta[k]), np.asarray(tb[k])), (name, k)
        da, _ = bound.camera_desc(sub, tasks)
        db, _ = ours.camera_desc(sub, tasks)
        for f in ("width", "height", "col0", "ncols", "d", "focal_length", "n_dof", "n_aa", "n_times", "jitter",
                  "jitter_scale"):
            assert getattr(da, f) == getattr(db, f), (name, f)
        for f in ("position", "u", "v", "w"):
            assert list(getattr(da, f)) == list(getattr(db, f)), (name, f)


def test_reference_shapes_are_what_the_binding_reads():
    """The fixture really carries the reference's shapes (not this package's)."""
    ref, _ = R.load("TorusMesh")
    mesh = ref.objects[1]
    assert type(mesh).__name__ == "Mesh" and isinstance(mesh.verts, list)
    assert type(mesh.bounding_volume).__name__ == "BoundingAABB"
    assert not hasattr(mesh, "bv_type") and not hasattr(mesh, "triangles")
    plane = ref.objects[0]
    assert hasattr(plane, "width_axis") and plane.texture is None and not hasattr(plane, "texture_scale")
    node = R.load("NovelScene1")[0].objects[1]
    assert type(node).__name__ == "Hierarchy" and hasattr(node, "Minv") and node.children


def test_kind_falls_back_to_the_class_attributes():
    """Objects built by hand may carry any gtype: the attributes that define each class decide."""
    class G:
        def __init__(self, **kw):
            self.__dict__.update(kw, gtype="custom")
    assert kind(G(center=(0, 0, 0), radius=1.0)) == N.RTX_SPHERE
    assert kind(G(point=(0, 0, 0), normal=(0, 1, 0))) == N.RTX_PLANE
    assert kind(G(minpos=(0, 0, 0), maxpos=(1, 1, 1))) == N.RTX_BOX
    assert kind(G(verts=[], faces=[], bounding_volume=None)) == N.RTX_MESH
    assert kind(G(hierarchy_type="union", children=[])) == N.RTX_NODE
    with pytest.raises(NotImplementedError):
        kind(G(foo=1))


@pytest.mark.skipif(not os.path.isdir("/root/reference/provided"), reason="reference snapshot not mounted")
def test_fixture_matches_the_live_reference(tmp_path):
    """Regenerate the fixture from the reference's own parser and compare."""
    out = str(tmp_path / "refobjects.json")
    subprocess.check_call([sys.executable, os.path.join(HERE, "golden", "make_refobjects.py"), out])
    with open(out) as f, open(R.FIXTURE) as g:
        assert json.load(f) == json.load(g)


def test_descriptor_comparison_sees_a_changed_attribute():
    """Negative control for the byte comparison above."""
    ref, res = R.load("TorusMesh")
    ref.objects[1].verts[5] = ref.objects[1].verts[5] + 1e-3
    a, b = desc_bytes(rtx.Scene.from_reference(ref).scene_desc()), desc_bytes(product("TorusMesh", res).scene_desc())
    assert a[0] == b[0] and a[3] != b[3]  # same object records, different triangles
