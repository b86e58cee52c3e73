"""Host side of the split passes specialized on a scene's CSG trees (rtx_api.hip
jit_csg_tables / csg_cost / jit_split_spec, through the host emulation): which scenes
qualify, the node table and matrices the kernel source carries, and the options it is
compiled with. No GPU: the GPU tests (test_gpu_split.py) render with the kernels."""
import ctypes as C
import re

import numpy as np
import pytest

import hostemu
from common import OPTS, product_scene, product_scene_dict


def split_spec(sc, pas=0, cnt=0, jit=0):
    f = hostemu.lib().rtx_hostemu_jit_split
    f.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_char_p, C.c_int64, C.POINTER(C.c_int64)]
    f.restype = C.c_int64
    sd = sc.scene_desc()
    cost = C.c_int64()
    n = f(C.addressof(sd), pas, cnt, jit, None, 0, C.byref(cost))
    if n < 0:
        return None, cost.value
    buf = C.create_string_buffer(int(n) + 1)
    f(C.addressof(sd), pas, cnt, jit, buf, n + 1, C.byref(cost))
    head, src = buf.value.decode().split("\n\n", 1)
    name, *opts = head.split("\n")
    return (name, opts, src), cost.value


def tables(src):
    """kNode rows and the kM / kMinv matrices of a specialized pass's source."""
    nodes = [tuple(int(x) for x in m.split(","))
             for m in re.findall(r"\{(-?\d+(?:,-?\d+){8})\}", src.split("kNode[] = {", 1)[1].split("};", 1)[0])]

    def mats(name):
        body = src.split("%s[][16] = {" % name, 1)[1].split("};", 1)[0]
        rows = re.findall(r"\{([^{}]*)\}", body)
        return [np.array([float.fromhex(v.rstrip("f")) for v in r.split(",") if v], dtype=np.float32) for r in rows]
    return nodes, mats("kM"), mats("kMinv")


def test_novel_scene_tables_and_options():
    """NovelScene1: its trees qualify (csg_cost 578), the trace and shadow sources carry one
    kNode row and two exact matrices per node, inner nodes' M * Minv is the identity, and
    the passes compile with rays in registers, the shadow pass at 4 waves/SIMD."""
    sc = product_scene("NovelScene1", (64, 32))
    (name, opts, src), cost = split_spec(sc, 0, 0, 1)
    assert name == "rtx_jit_split_trace_0101" and cost == 578
    assert "#define RTX_CSG_STATIC 1" in src and "rtx::split_trace<false, true, false, true>" in src
    assert "-DRTX_CSG_RAYREG=1" in opts and "-ffp-contract=off" in opts
    nodes, M, Minv = tables(src)
    n = int(re.search(r"kCount = (\d+);", src).group(1))
    assert len(nodes) == len(M) == len(Minv) == n > 50
    inner = [i for i, nd in enumerate(nodes) if nd[0] != 4]  # (kind 4: leaf)
    for i in inner:
        a = M[i].astype(np.float64).reshape(4, 4)
        b = Minv[i].astype(np.float64).reshape(4, 4)
        assert np.allclose(a @ b, np.eye(4), atol=1e-5), i
    for i, (kind, parent, cidx, depth, end, pkind, obj, mat0, oid) in enumerate(nodes):
        assert i < end <= n and (parent < 0) == (depth == 0)
        if parent >= 0:
            assert nodes[parent][3] == depth - 1 and nodes[parent][0] == pkind
    (sname, sopts, ssrc), _ = split_spec(sc, 1)
    assert sname == "rtx_jit_split_shadow_00" and "rtx::split_shadow<false, false>" in ssrc
    assert sopts.index("-DRTX_LB_SPLIT_B=4") > sopts.index("-URTX_LB_SPLIT_B")


def test_ray_storage_option_and_baked_boxes(monkeypatch):
    """csg_rays 0: the LDS ray stack (no shadow bound); jit_csg 2 / 3: the boxes / and the
    object records as byte arrays in the source."""
    sc = product_scene("NovelScene2", (32, 16))
    monkeypatch.setattr(OPTS, "csg_rays", "0")
    (_, opts, _), _ = split_spec(sc, 1)
    assert "-DRTX_CSG_RAYREG=0" in opts and "-DRTX_LB_SPLIT_B=4" not in opts
    monkeypatch.setattr(OPTS, "csg_rays", "3")
    for level, objs in (("2", False), ("3", True)):
        monkeypatch.setattr(OPTS, "jit_csg", level)
        (_, _, src), _ = split_spec(sc, 0)
        assert "kBoxes[]" in src and ("kObjs[]" in src) == objs and "#define RTX_CSG_BAKED %s" % level in src


def deep_intersections(depth, fan):
    """A scene of one tree: intersections `fan` wide down to `depth`, spheres below."""
    k = [0]

    def node(d):
        k[0] += 1
        if d == depth:
            return {"name": "s%d" % k[0], "type": "sphere", "radius": 1.0, "position": [0.01 * k[0], 0, 0]}
        return {"name": "n%d" % k[0], "type": "node", "hierarchy_type": "intersection",
                "children": [node(d + 1) for _ in range(fan)]}
    root = dict(node(0), materials=[0])
    return {"resolution": [32, 24], "ambient": [0.1, 0.1, 0.1],
            "camera": {"position": [0, 1, 6], "lookAt": [0, 0, 0], "up": [0, 1, 0], "fov": 45},
            "materials": [{"name": "m", "ID": 0, "diffuse": [0.5, 0.5, 0.5], "specular": [0, 0, 0], "hardness": 1}],
            "lights": [{"type": "point", "position": [0, 4, 4], "colour": [1, 1, 1], "power": 1}],
            "objects": [root]}


def test_scenes_that_keep_the_precompiled_passes():
    """Trees whose unrolled walk-ups would repeat too much (csg_cost > 6000: each leaf's
    walk-up tests its siblings' subtrees at every intersection above it) and flat scenes
    keep the precompiled passes; a small tree of the same shape is specialized. (A
    difference with one child is refused at scene creation, as the reference raises.)"""
    spec, cost = split_spec(product_scene_dict(deep_intersections(5, 3)))
    assert spec is None and cost > 6000
    spec, cost = split_spec(product_scene_dict(deep_intersections(2, 3)))
    assert spec is not None and 0 < cost <= 6000
    spec, cost = split_spec(product_scene("TwoSpheresPlane", (32, 16)))
    assert spec is None and cost == -1


@pytest.mark.parametrize("seed", [1, 4, 12])
def test_random_trees_cost_and_tables(seed):
    from scenegen import random_hier_scene
    d = random_hier_scene(seed, res=(32, 24), mesh=(seed % 4 == 0))
    spec, cost = split_spec(product_scene_dict(d))
    assert 0 < cost <= 6000 and spec is not None
    nodes, M, Minv = tables(spec[2])
    assert len(nodes) == len(M) and all(np.all(np.isfinite(m)) for m in M + Minv)
