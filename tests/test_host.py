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
    decl = set(re.findall(r"^(?:int|const char\*)\s+(rtx_\w+)\s*\(", hdr, re.M))
    assert decl == set(N.EXPORTS)
    lib = N.load()
    for sym in decl:
        assert hasattr(lib, sym), sym
    assert lib.rtx_abi_version() == N.ABI_VERSION


def test_abi_struct_layouts_match_the_header():
    import hostemu
    lib = hostemu.lib()
    lib.rtx_hostemu_sizeof.restype = C.c_int64
    for i, st in enumerate([N.rtx_object, N.rtx_triangle, N.rtx_material, N.rtx_light, N.rtx_scene_desc,
                            N.rtx_camera_desc]):
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


def test_hierarchy_nodes_fail_loudly():
    with open(os.path.join(REPO, "assets", "scenes.json")) as f:
        d = json.load(f)["NovelScene1"]
    d["__base_dir__"] = os.path.join(REPO, "assets")
    with pytest.raises(NotImplementedError):
        rtx.load_scene(d, verbose=False)


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
    assert m.bv_type == "aabb"  # box volume < bounding sphere volume


def test_f32_helpers_follow_glm_order():
    a = np.array([1e8, 1.0, -1e8], np.float32)
    b = np.array([1.0, 1.0, 1.0], np.float32)
    assert F.dot(a, b) == np.float32(np.float32(1e8 + np.float32(1.0)) - np.float32(1e8))
    v = F.normalize(np.array([3, 4, 0], np.float32))
    assert v.dtype == np.float32 and abs(float(F.length(v)) - 1) < 1e-6
