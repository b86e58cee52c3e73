"""Host logic that needs no GPU: parser defaults, partitions, tables, mesh
preprocessing, and the C ABI of librtx.so (loads and exports every declared symbol)."""
import ctypes as C
import json
import os
import re

import numpy as np
import pytest

import rtx
from rtx import _native as N
from rtx import f32 as F
from rtx.scene import split_rows, strip_columns

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_header_symbol():
    hdr = open(os.path.join(REPO, "include", "rtx.h")).read()
    decl = set(re.findall(r"^(?:int|int32_t|const char\*)\s+(rtx_\w+)\s*\(", hdr, re.M))
    assert decl == set(N.EXPORTS)
    lib = N.load()
    for sym in decl:
        assert hasattr(lib, sym), sym
    assert lib.rtx_abi_version() == N.ABI_VERSION


def test_options_table_documented_and_round_trips():
    """Every library option is named in INTEGRATION.md or DESIGN.md §6s, reads back what
    was set (rtx_set_option / rtx_get_option, no GPU), and an unknown name or a malformed
    number is refused."""
    names = rtx.option_names()
    docs = open(os.path.join(REPO, "DESIGN.md")).read() + open(os.path.join(REPO, "INTEGRATION.md")).read()
    for n in names:
        assert "`%s`" % n in docs, n
    for n, v in (("tile_block", "256"), ("xcd_map", "1"), ("jit_ilp", "0"), ("split_bytes", "1073741824")):
        old = rtx.get_option(n)
        try:
            rtx.set_option(n, v)
            assert float(rtx.get_option(n)) == float(v), n
        finally:
            rtx.set_option(n, old)
    with pytest.raises(N.RtxError):
        rtx.set_option("no_such_option", "1")
    with pytest.raises(N.RtxError):
        rtx.set_option("bins", "not-a-number")


def test_abi_struct_layouts_match_the_header():
    import hostemu
    lib = hostemu.lib()
    lib.rtx_hostemu_sizeof.restype = C.c_int64
    for i, st in enumerate([N.rtx_object, N.rtx_triangle, N.rtx_material, N.rtx_light, N.rtx_scene_desc,
                            N.rtx_camera_desc, N.rtx_texture]):
        assert lib.rtx_hostemu_sizeof(i) == C.sizeof(st), st.__name__


def test_invalid_scene_is_rejected_without_gpu():
    """Validation happens before any HIP call (rtx_scene_create returns RTX_ERR_INVALID)."""
    lib = N.load()
    h = C.c_void_p()
    d = N.rtx_scene_desc()
    d.n_objects = 1  # objects == NULL
    assert lib.rtx_scene_create(C.byref(d), C.byref(h)) == N.RTX_ERR_INVALID
    assert b"null array" in lib.rtx_last_error()


@pytest.mark.parametrize("W,tasks", [(10, 3), (1920, 7), (5, 5), (256, 1), (7, 2)])
def test_strip_and_row_partitions_follow_array_split(W, tasks):
    parts = np.array_split(np.arange(W), tasks)
    for k in range(tasks):
        c0, n = strip_columns(W, k, tasks)
        assert n == len(parts[k]) and c0 == parts[k][0]
        r0, nr = split_rows(W, tasks, k)
        assert (r0, nr) == (parts[k][0], len(parts[k]))


def test_empty_strip_raises_like_reference():
    with pytest.raises(IndexError):
        strip_columns(3, 4, 5)


def test_parser_defaults():
    d = {"camera": {"position": [0, 0, 5], "lookAt": [0, 0, 0], "up": [0, 1, 0], "fov": 45},
         "materials": [{"name": "m", "ID": 3}],
         "objects": [{"name": "s", "type": "sphere", "radius": 1, "materials": [3]},
                     {"name": "x", "type": "unknowncube"}],
         "lights": [{"name": "l", "type": "directional", "colour": [1, 1, 1], "direction": [0, -1, 0], "power": 5}]}
    sc = rtx.load_scene(d, verbose=False)
    assert (sc.vc.width, sc.vc.height) == (1080, 720)
    assert (sc.jitter, sc.samples) == (False, 1)
    assert (sc.vc.focal_length, sc.vc.aperture, sc.vc.dof_samples) == (1, 0, 1)
    assert sc.vc.motion_times == [0.0]
    assert np.array_equal(sc.ambient, np.zeros(3, np.float32))
    m = sc.materials[0]
    assert (m.mat_type, m.hardness, m.tint, m.refr_index) == ("diffuse", 32, 0.0, 1.0)
    assert sc.lights[0].power == 1.0          # directional power forced to 1.0
    assert len(sc.objects) == 1               # unknown type skipped


def test_parser_light_keyerror_drops_all_lights():
    d = {"camera": {"position": [0, 0, 5], "lookAt": [0, 0, 0], "up": [0, 1, 0], "fov": 45},
         "materials": [], "objects": [],
         "lights": [{"name": "a", "type": "point", "colour": [1, 1, 1], "position": [0, 1, 0], "power": 1},
                    {"name": "b", "type": "point", "colour": [1, 1, 1], "position": [0, 1, 0]}]}
    assert rtx.load_scene(d, verbose=False).lights == []


def _novel(name="NovelScene1"):
    with open(os.path.join(REPO, "assets", "scenes.json")) as f:
        d = json.load(f)[name]
    d["__base_dir__"] = os.path.join(REPO, "assets")
    return d


def test_hierarchy_parsing_follows_reference():
    """scene_parser.py:177-205, :261-285 and hierarchy.py:21-28 on NovelScene1."""
    from rtx import geometry as geom
    sc = rtx.load_scene(_novel(), verbose=False)
    names = [o.name for o in sc.objects]
    assert names == ["ground", "wall1", "wall2", "wall4", "wall3", "bike", "bike2", "trail1", "trail2"]
    bike, bike2 = sc.objects[5], sc.objects[6]
    assert isinstance(bike, geom.Hierarchy) and bike.hierarchy_type == "union"
    # ref copy: its own name, materials and transform, the copied subtree (and its speeds)
    assert bike2.name == "bike2" and [m.ID for m in bike2.materials] == [9]
    assert np.array_equal(bike2.t, np.float32([-2.0, -2.5, 2.0]))
    assert len(bike2.children) == len(bike.children)
    assert bike2.children[0] is not bike.children[0]
    # fallback: leaves get the root's materials appended, nested node materials untouched
    inner = bike.children[0].children[0].children[0].children[0]   # front_wheel/cutout/main/inner
    assert inner.name == "inner" and [m.ID for m in inner.materials] == [1, 0]
    inner2 = bike2.children[0].children[0].children[0].children[0]
    assert [m.ID for m in inner2.materials] == [1, 9]
    outer = bike.children[0].children[0].children[0].children[1]
    assert [m.ID for m in outer.materials] == [0]
    assert bike.children[0].materials == []
    # speeds: root speed + own speed for every leaf, at any depth
    assert np.array_equal(inner.speed, np.float32([0, 0, 0.5]))
    # walls: no root materials, so nothing is appended; planes keep their texture
    wall = sc.objects[1]
    assert [m.ID for m in wall.children[0].materials] == [8] and wall.children[0].texture is not None
    assert wall.children[0].texture_scale == 35.0 and wall.children[1].speed is None
    assert sc.objects[0].texture.size == (1024, 1024) and sc.objects[0].texture_scale == 4.0


def test_unknown_ref_is_skipped():
    d = _novel()
    d["objects"] = [o for o in d["objects"] if o["name"] != "bike"]
    sc = rtx.load_scene(d, verbose=False)
    assert "bike2" not in [o.name for o in sc.objects]


def test_descriptor_is_preorder_with_parents():
    sc = rtx.load_scene(_novel(), verbose=False)
    desc = sc.scene_desc()
    n = desc.n_objects
    par = [desc.objects[i].parent for i in range(n)]
    top = [i for i in range(n) if par[i] == -1]
    assert len(top) == len(sc.objects)
    for i in range(n):
        assert par[i] < i
        if par[i] >= 0:
            assert desc.objects[par[i]].type == N.RTX_NODE
    assert desc.n_textures == 5  # ground + four walls, each opened once per plane
    t = desc.textures[0]
    assert (t.width, t.height) == (1024, 1024)


def test_texture_rgb8_matches_getpixel():
    from PIL import Image
    from rtx import geometry as geom
    from rtx.records import texture_rgb8
    for name in ("wall1.png", "brick.jpg", "axes.png"):
        im = geom.open_texture(os.path.join(REPO, "assets", "textures", name))
        a = texture_rgb8(im)
        for (i, j) in ((0, 0), (5, 17), (im.width - 1, im.height - 1), (100, 3)):
            assert tuple(a[j, i]) == tuple(im.getpixel((i, j))[:3])


def test_invalid_hierarchy_is_rejected_without_gpu():
    lib = N.load()
    objs = (N.rtx_object * 2)()
    objs[0].type, objs[0].parent, objs[0].hierarchy_type = N.RTX_NODE, -1, N.RTX_DIFFERENCE
    objs[1].type, objs[1].parent, objs[1].n_mats, objs[1].texture = N.RTX_SPHERE, 0, 1, -1
    objs[0].texture = -1
    mats = (N.rtx_material * 1)()
    d = N.rtx_scene_desc()
    d.n_objects, d.objects, d.n_materials, d.materials = 2, objs, 1, mats
    h = C.c_void_p()
    assert lib.rtx_scene_create(C.byref(d), C.byref(h)) == N.RTX_ERR_INVALID
    assert b"two children" in lib.rtx_last_error()
    objs[1].parent = 1  # not an earlier node
    assert lib.rtx_scene_create(C.byref(d), C.byref(h)) == N.RTX_ERR_INVALID
    assert b"parent" in lib.rtx_last_error()


def test_camera_tables_follow_reference_sequences():
    sc = rtx.load_bundled_scene("TwoSpheresPlane", resolution=(64, 48))
    t = sc.camera_tables(1, 3)
    vc = sc.vc
    dx = (vc.right - vc.left) / vc.width
    cols = np.array_split(np.arange(64), 3)[1]
    x = vc.left + (0.5 + cols[0]) * dx
    for i in range(len(cols)):
        assert t["xs"][i] == np.float32(x)
        x += dx
    # 1 spp AA still shifts the origin by 2(dx+dy) at theta_1
    assert not np.array_equal(t["aa"][0, 0], vc.position)


def test_torus_mesh_preprocessing():
    sc = rtx.load_bundled_scene("TorusMesh", resolution=(8, 8))
    m = sc.objects[1]
    assert m.verts.shape == (64, 3) and m.faces.shape == (128, 3)
    # box volume < bounding sphere volume (mesh.py:48-49)
    assert type(m.bounding_volume).__name__ == "BoundingAABB"


def test_f32_helpers_follow_glm_order():
    a = np.array([1e8, 1.0, -1e8], np.float32)
    b = np.array([1.0, 1.0, 1.0], np.float32)
    assert F.dot(a, b) == np.float32(np.float32(1e8 + np.float32(1.0)) - np.float32(1e8))
    v = F.normalize(np.array([3, 4, 0], np.float32))
    assert v.dtype == np.float32 and abs(float(F.length(v)) - 1) < 1e-6


def test_camera_key_follows_every_camera_change():
    """Scene._camera_key (which decides when rtx_camera_set re-uploads the tables) is
    cached by the camera's version: equal while nothing changes, new after an attribute
    assignment, an in-place edit of a basis vector or of motion_times (a list or any other
    sequence assigned to it), or a scene sample setting."""
    import numpy as np
    import rtx
    from rtx import f32 as F
    sc = rtx.load_bundled_scene("TwoSpheresPlane", resolution=(64, 48))
    vc = sc.vc
    seen = [sc._camera_key(0, 1)]
    assert sc._camera_key(0, 1) == seen[0]

    def changed():
        k = sc._camera_key(0, 1)
        assert all(k != s for s in seen)
        seen.append(k)

    vc.set_camera(F.vec3(0.0, 2.0, 7.0), F.vec3(0.0, 0.0, 0.0), F.vec3(0.0, 1.0, 0.0), 40.0)
    changed()
    vc.motion_times.append(0.5)
    changed()
    vc.motion_times[1] = 0.25
    changed()
    vc.motion_times += [1.0]
    changed()
    vc.aperture = 0.1
    changed()
    sc.samples = 2
    changed()
    sc.seed = 7
    changed()
    assert sc._camera_key(1, 2) != sc._camera_key(0, 1)
    assert vc.motion_times == [0, 0.25, 1.0]
    # basis vectors are writable in place, like PyGLM's vec3, and every write is seen
    vc.position[0] = 1.0
    changed()
    vc.u[1:] = 0.5
    changed()
    vc.v += F.vec3(0.0, 0.0, 1e-3)
    changed()
    np.multiply(vc.w, 2.0, out=vc.w)
    changed()
    assert float(vc.position[0]) == 1.0 and vc.position.dtype == np.float32
    d = vc.position - vc.w  # arithmetic gives plain arrays, not tracked views of the camera
    assert type(d) is np.ndarray
    d[0] = 5.0
    assert sc._camera_key(0, 1) == seen[-1]
    # motion_times assigned as an ndarray: kept as a tracked list
    vc.motion_times = np.array([0.0, 0.5])
    changed()
    vc.motion_times[1] = 0.75
    changed()
    assert list(vc.motion_times) == [0.0, 0.75]
    # a camera vector of another type: every render compares the values themselves
    vc.position = [0.0, 2.0, 7.5]
    k1 = sc._camera_key(0, 1)
    vc.position[2] = 8.0
    assert sc._camera_key(0, 1) != k1
