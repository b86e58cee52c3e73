"""Python harness of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module. The product package (``python-raytracer_amd/rtx``) never does.

It restates the JSON side of the reference's ``scene_parser.load_scene``
(provided/scene_parser.py:50-163, defaults at :62-142, ``associate_material`` at
:288-294, ``add_basic_shape`` at :212-258) independently of the product's parser, reads
OBJ files like ``igl.read_obj`` (provided/geometry/mesh.py:20) and hands everything to
``rtx_oracle.c`` (the restated render path) through ctypes.
"""
import ctypes as C
import json
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")

_i = C.POINTER(C.c_int)
_d = C.POINTER(C.c_double)
_f = C.POINTER(C.c_float)


class _SceneIn(C.Structure):
    _fields_ = [
        ("width", C.c_int), ("height", C.c_int),
        ("cam", C.c_double * 10),
        ("ambient", C.c_double * 3),
        ("jitter", C.c_int), ("samples", C.c_int),
        ("focal_length", C.c_double), ("aperture", C.c_double),
        ("dof_samples", C.c_int),
        ("motion_time", C.c_double),
        ("motion_samples", C.c_int), ("motion_final", C.c_int),
        ("n_lights", C.c_int),
        ("light_type", _i), ("light_colour", _d), ("light_vector", _d), ("light_power", _d),
        ("n_mats", C.c_int),
        ("mat_diffuse", _d), ("mat_specular", _d), ("mat_hardness", _d), ("mat_type", _i),
        ("mat_tint", _d), ("mat_refr", _d),
        ("n_objs", C.c_int),
        ("obj_type", _i), ("obj_nmat", _i), ("obj_mat", _i), ("obj_has_speed", _i),
        ("obj_speed", _d), ("obj_a", _d), ("obj_b", _d), ("obj_c", _d), ("obj_box_mode", _i),
        ("obj_scalar", _d), ("obj_flat", _i),
        ("mesh_vert_off", _i), ("mesh_nverts", _i), ("mesh_face_off", _i), ("mesh_nfaces", _i),
        ("verts", _d), ("faces", _i),
        ("obj_parent", _i), ("obj_child_off", _i), ("obj_nchild", _i), ("child_idx", _i),
        ("node_htype", _i), ("node_trs", _d),
        ("obj_tex", _i), ("obj_tex_scale", _d),
        ("n_tex", C.c_int), ("tex_w", _i), ("tex_h", _i), ("tex_off", C.POINTER(C.c_longlong)),
        ("tex_data", C.POINTER(C.c_ubyte)),
    ]


def build(force=False):
    """Compile rtx_oracle.c with gcc (oracle/Makefile recipe)."""
    if force or not os.path.exists(LIB_PATH) or \
            os.path.getmtime(LIB_PATH) < os.path.getmtime(os.path.join(HERE, "rtx_oracle.c")):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = C.CDLL(build())
        _lib.oracle_render.argtypes = [C.POINTER(_SceneIn), C.c_int, C.c_int, _d, _d, C.POINTER(C.c_longlong)]
        _lib.oracle_object_intersect.argtypes = [C.POINTER(_SceneIn), C.c_int, C.c_double, _f, _f, C.c_int,
                                                 _d, _f, _f, _i, _i]
        _lib.oracle_closest_batch.argtypes = [C.POINTER(_SceneIn), C.c_double, C.c_int, _f, _f,
                                              _d, _i, _i, _i, _f, _f]
        _lib.oracle_shadow_batch.argtypes = [C.POINTER(_SceneIn), C.c_double, C.c_int, _f, _f, _d, _i]
        _lib.oracle_object_shadow_batch.argtypes = [C.POINTER(_SceneIn), C.c_int, C.c_double, C.c_int, _f, _f,
                                                    _d, _i]
        _lib.oracle_object_inside_batch.argtypes = [C.POINTER(_SceneIn), C.c_int, C.c_double, C.c_int, _f, _i]
    return _lib


# ------------------------------------------------------------------ JSON restatement
_MAT_TYPES = {"diffuse": 0, "mirror": 1, "refractive": 2}


def _read_obj(path):
    """igl.read_obj restated for the triangle OBJ files the reference uses."""
    V, F = [], []
    with open(path) as f:
        for line in f:
            p = line.split()
            if not p:
                continue
            if p[0] == "v":
                V.append([float(x) for x in p[1:4]])
            elif p[0] == "f":
                F.append([int(x.split("/")[0]) - 1 for x in p[1:4]])
    return np.array(V, dtype=np.float64).reshape(-1, 3), np.array(F, dtype=np.int32).reshape(-1, 3)


def _vec(v):
    return [float(v[0]), float(v[1]), float(v[2])]

_TYPES = {"sphere": 0, "plane": 1, "box": 2, "mesh": 3, "node": 4}
_HTYPES = {"union": 0, "intersection": 1, "difference": 2}


def _f32vec(v):
    return [float(x) for x in np.asarray(v, np.float64).astype(np.float32)]


def _load_texture(path):
    """Image.open(texture) + getpixel((i, j))[0:3] (simple_geometry.py:168-169): RGB8 [h, w, 3]."""
    from PIL import Image
    im = Image.open(path)
    if im.mode not in ("RGB", "RGBA", "RGBX", "CMYK", "RGBa", "YCbCr", "LAB", "HSV"):
        raise TypeError("texture %s: getpixel of mode %s is not indexable as RGB" % (path, im.mode))
    return np.ascontiguousarray(np.asarray(im)[:, :, :3], dtype=np.uint8)


def _parse_objects(data, ids, base_dir):
    """scene_parser.py:144-161 + parse_geometry/add_basic_shape/traverse_children
    (:166-285) + Hierarchy.set_fallback_material (hierarchy.py:21-28), restated on plain
    dicts. Returns geometry records in preorder (top-level objects have parent -1)."""
    import copy

    def mats_of(g):
        return [k for i in g.get("materials", []) for k, mid in enumerate(ids) if mid == i]

    def basic(g, speed):
        t = g["type"]
        g["name"]  # noqa: B018
        if t not in ("sphere", "plane", "box", "mesh"):
            return None
        if t == "sphere":
            g["radius"]  # noqa: B018
        return {"kind": t, "json": g, "pos": _f32vec(g.get("position", [0, 0, 0])), "mats": mats_of(g),
                "speed": speed, "children": []}

    def node(g, speed, children_speed):
        return {"kind": "node", "json": {}, "mats": mats_of(g), "speed": speed,
                "htype": g.get("hierarchy_type", "union"),
                "trs": _f32vec(g.get("position", [0, 0, 0])) + _f32vec(g.get("rotation", [0, 0, 0]))
                + _f32vec(g.get("scale", [1, 1, 1])),
                "children": traverse(g["children"], children_speed)}

    def traverse(children, speed):
        out = []
        for g in children:
            g["name"]  # noqa: B018
            gt = g["type"]
            g.get("position", [0, 0, 0])
            cs = None if speed is None else _f32vec(np.float32(speed) + np.float32(g.get("speed", [0, 0, 0])))
            leaf = basic(g, cs)
            if leaf is not None:
                out.append(leaf)
            elif gt == "node":
                out.append(node(g, cs, speed))   # grandchildren get the ROOT's speed again (:283)
        return out

    objects, root_names, roots = [], [], []
    for g in data["objects"]:
        sp = g.get("speed")
        sp = None if sp is None else _f32vec(sp)
        leaf = basic(g, sp)
        if leaf is not None:
            objects.append(leaf)
        elif g["type"] == "node":
            ref = g.get("ref", "")
            if ref == "":
                root_names.append(g["name"])
                n = node(g, sp, sp)
                roots.append(n)
                objects.append(n)
            elif ref in root_names:
                n = copy.deepcopy(roots[root_names.index(ref)])
                n["mats"] = mats_of(g)
                n["trs"] = (_f32vec(g.get("position", [0, 0, 0])) + _f32vec(g.get("rotation", [0, 0, 0]))
                            + _f32vec(g.get("scale", [1, 1, 1])))
                objects.append(n)
    # set_fallback_material(obj.materials) for every top-level hierarchy, after parsing
    def fallback(n, mats):
        if not mats:
            return
        for c in n["children"]:
            if c["kind"] == "node":
                fallback(c, mats)
            else:
                c["mats"] = c["mats"] + mats
    for o in objects:
        if o["kind"] == "node":
            fallback(o, list(o["mats"]))
    records = []

    def flatten(o, parent):
        idx = len(records)
        rec = dict(o)
        rec["parent"] = parent
        records.append(rec)
        rec["child_ids"] = [flatten(c, idx) for c in o["children"]]
        return idx
    for o in objects:
        flatten(o, -1)
    for r in records:
        if r["kind"] != "node" and not r["mats"]:
            raise IndexError("object has no material (the reference raises IndexError when it is hit)")
    return records


class OracleScene:
    """A scene JSON dictionary converted to the oracle's C input struct."""

    def __init__(self, data, base_dir=None):
        self._keep = []
        s = _SceneIn()
        cam = data["camera"]
        s.cam[:] = _vec(cam["position"]) + _vec(cam["lookAt"]) + _vec(cam["up"]) + [float(cam["fov"])]
        res = data.get("resolution", [1080, 720])
        s.width, s.height = int(res[0]), int(res[1])
        s.ambient[:] = _vec(data.get("ambient", [0, 0, 0]))
        try:
            jitter, samples = data["AA"]["jitter"], data["AA"]["samples"]
        except KeyError:
            jitter, samples = False, 1
        s.jitter, s.samples = int(bool(jitter)), int(samples)
        try:
            fl, ap, ds = data["DOF"]["focal_length"], data["DOF"]["aperture"], data["DOF"]["samples"]
        except KeyError:
            fl, ap, ds = 1, 0, 1
        s.focal_length, s.aperture, s.dof_samples = float(fl), float(ap), int(ds)
        try:
            mt, ms, mf = data["motion"]["time"], data["motion"]["samples"], data["motion"]["final"]
        except KeyError:
            mt, ms, mf = 0, 1, 0
        s.motion_time, s.motion_samples, s.motion_final = float(mt), int(ms), int(mf)

        lt, lc, lv, lp = [], [], [], []
        try:
            for L in data["lights"]:
                t = L["type"]
                col = _vec(L["colour"])
                if t == "point":
                    vec, pw, code = _vec(L["position"]), float(L["power"]), 0
                elif t == "directional":
                    vec, pw, code = _vec(L["direction"]), 1.0, 1
                else:
                    continue
                L["name"]  # noqa: B018  (KeyError semantics of scene_parser.py:109)
                lt.append(code); lc += col; lv += vec; lp.append(pw)
        except KeyError:
            lt, lc, lv, lp = [], [], [], []
        s.n_lights = len(lt)
        s.light_type, s.light_colour = self._ai(lt), self._ad(lc)
        s.light_vector, s.light_power = self._ad(lv), self._ad(lp)

        ids, md, msp, mh, mty, mti, mr = [], [], [], [], [], [], []
        for m in data["materials"]:
            ids.append(m["ID"])
            m["name"]  # noqa: B018
            mty.append(_MAT_TYPES.get(m.get("type", "diffuse"), 0))
            md += _vec(m.get("diffuse", [0, 0, 0]))
            msp += _vec(m.get("specular", [0, 0, 0]))
            mh.append(float(m.get("hardness", 32)))
            mti.append(float(m.get("tint", 0.0)))
            mr.append(float(m.get("refr_index", 1.0)))
        s.n_mats = len(ids)
        s.mat_diffuse, s.mat_specular, s.mat_hardness = self._ad(md), self._ad(msp), self._ad(mh)
        s.mat_type, s.mat_tint, s.mat_refr = self._ai(mty), self._ad(mti), self._ad(mr)

        records = _parse_objects(data, ids, base_dir)
        ot, on, om, ohs, osp, oa, ob, oc, obm, osc, ofl = ([] for _ in range(11))
        mvo, mnv, mfo, mnf = [], [], [], []
        opar, coff, nch, cidx, hty, trs, otex, otsc = [], [], [], [], [], [], [], []
        allv, allf = [np.zeros((0, 3))], [np.zeros((0, 3), np.int32)]
        textures, tex_index = [], {}
        nv_total = nf_total = 0
        for r in records:
            mats = r["mats"]
            code = _TYPES[r["kind"]]
            a, b, c, bm, sc, fl_, vo, nv, fo, nf = r.get("pos", [0.0] * 3), [0.0] * 3, [0.0] * 3, 0, 0.0, 0, 0, 0, 0, 0
            tex, tsc = -1, 1.0
            g = r.get("json", {})
            if r["kind"] == "sphere":
                sc = float(g["radius"])
            elif r["kind"] == "plane":
                b = _vec(g["normal"])
            elif r["kind"] == "box":
                if "size" in g:
                    b = _vec(g["size"])
                else:
                    bm, c, b = 1, _vec(g["min"]), _vec(g["max"])
            elif r["kind"] == "mesh":
                path = g["filepath"]
                if base_dir is not None and not os.path.exists(path):
                    path = os.path.join(base_dir, path)
                V, F = _read_obj(path)
                sc, fl_ = float(g["scale"]), int(bool(g.get("flat_shaded", False)))
                vo, nv, fo, nf = nv_total, len(V), nf_total, len(F)
                allv.append(V); allf.append(F)
                nv_total += nv; nf_total += nf
            if r["kind"] in ("plane", "box") and "texture" in g:
                path = g["texture"]
                if base_dir is not None and not os.path.exists(path):
                    path = os.path.join(base_dir, path)
                if path not in tex_index:
                    tex_index[path] = len(textures)
                    textures.append(_load_texture(path))
                tex = tex_index[path]
                if r["kind"] == "plane":
                    tsc = float(g.get("texture_scale", 1.0))
            sp = r.get("speed")
            ot.append(code); on.append(len(mats)); om += (mats + [0, 0, 0, 0])[:4]
            ohs.append(0 if sp is None else 1); osp += [0.0] * 3 if sp is None else [float(x) for x in sp]
            oa += a; ob += b; oc += c; obm.append(bm); osc.append(sc); ofl.append(fl_)
            mvo.append(vo); mnv.append(nv); mfo.append(fo); mnf.append(nf)
            opar.append(r["parent"]); coff.append(len(cidx)); nch.append(len(r["child_ids"])); cidx += r["child_ids"]
            hty.append(_HTYPES.get(r.get("htype"), 3)); trs += r.get("trs", [0.0] * 9)
            otex.append(tex); otsc.append(tsc)
        s.n_objs = len(ot)
        s.obj_type, s.obj_nmat, s.obj_mat, s.obj_has_speed = self._ai(ot), self._ai(on), self._ai(om), self._ai(ohs)
        s.obj_speed, s.obj_a, s.obj_b, s.obj_c = self._ad(osp), self._ad(oa), self._ad(ob), self._ad(oc)
        s.obj_box_mode, s.obj_scalar, s.obj_flat = self._ai(obm), self._ad(osc), self._ai(ofl)
        s.mesh_vert_off, s.mesh_nverts = self._ai(mvo), self._ai(mnv)
        s.mesh_face_off, s.mesh_nfaces = self._ai(mfo), self._ai(mnf)
        s.verts = self._ad(np.concatenate(allv).ravel())
        s.faces = self._ai(np.concatenate(allf).ravel())
        s.obj_parent, s.obj_child_off, s.obj_nchild, s.child_idx = self._ai(opar), self._ai(coff), self._ai(nch), self._ai(cidx)
        s.node_htype, s.node_trs = self._ai(hty), self._ad(trs)
        s.obj_tex, s.obj_tex_scale = self._ai(otex), self._ad(otsc)
        s.n_tex = len(textures)
        s.tex_w = self._ai([t.shape[1] for t in textures])
        s.tex_h = self._ai([t.shape[0] for t in textures])
        offs = np.cumsum([0] + [t.size for t in textures])[:-1]
        a = np.ascontiguousarray(np.asarray(offs, np.int64))
        self._keep.append(a)
        s.tex_off = a.ctypes.data_as(C.POINTER(C.c_longlong))
        td = np.ascontiguousarray(np.concatenate([t.ravel() for t in textures]) if textures else np.zeros(1, np.uint8))
        self._keep.append(td)
        s.tex_data = td.ctypes.data_as(C.POINTER(C.c_ubyte))
        self.records = records
        self.base_dir = base_dir
        self.s = s
        self.width, self.height = s.width, s.height
        self.n_samples = s.samples * s.dof_samples * (s.motion_samples + s.motion_final)
        self.jitter = bool(s.jitter)
        self.spp_rays = s.samples * s.dof_samples

    def _ad(self, x):
        a = np.ascontiguousarray(np.asarray(x, dtype=np.float64).ravel())
        if a.size == 0:
            a = np.zeros(1)
        self._keep.append(a)
        return a.ctypes.data_as(_d)

    def _ai(self, x):
        a = np.ascontiguousarray(np.asarray(x, dtype=np.int32).ravel())
        if a.size == 0:
            a = np.zeros(1, np.int32)
        self._keep.append(a)
        return a.ctypes.data_as(_i)

    # -------------------------------------------------------------- render paths
    def render(self, subimage=0, tasks=1, noise=None, tallies=False):
        """Scene.render(subimage, tasks) -> (strip_w, H, 3) float64 (scene.py:35-79)."""
        W, H = self.width, self.height
        base, extra = divmod(W, tasks)
        ncol = base + (1 if subimage < extra else 0)
        out = np.zeros((ncol, H, 3), dtype=np.float64)
        nz = None
        if self.jitter:
            if noise is None:
                raise ValueError("jittered scene: pass the replayed np.random stream as noise")
            nz = np.ascontiguousarray(noise, dtype=np.float64).ravel()
            need = ncol * H * self.spp_rays * 3
            if nz.size < need:
                raise ValueError("noise stream too short: %d < %d" % (nz.size, need))
        tl = (C.c_longlong * 13)()
        rc = lib().oracle_render(C.byref(self.s), subimage, tasks, out.ctypes.data_as(_d),
                                 None if nz is None else nz.ctypes.data_as(_d), tl)
        if rc == -3:
            raise IndexError("oracle_render: the reference raises here (texture index / missing material)")
        if rc != 0:
            raise RuntimeError("oracle_render failed: %d" % rc)
        if tallies:
            return out, list(tl)
        return out

    def object_intersect(self, obj, time, o, d, max_hits=256):
        t = np.zeros(max_hits); n = np.zeros((max_hits, 3), np.float32); p = np.zeros((max_hits, 3), np.float32)
        m = np.zeros(max_hits, np.int32); sb = np.zeros(max_hits, np.int32)
        o = np.ascontiguousarray(o, np.float32); d = np.ascontiguousarray(d, np.float32)
        k = lib().oracle_object_intersect(C.byref(self.s), obj, float(time), o.ctypes.data_as(_f),
                                          d.ctypes.data_as(_f), max_hits, t.ctypes.data_as(_d),
                                          n.ctypes.data_as(_f), p.ctypes.data_as(_f),
                                          m.ctypes.data_as(_i), sb.ctypes.data_as(_i))
        k = min(k, max_hits)
        return t[:k], n[:k], p[:k], m[:k], sb[:k]

    def closest(self, time, o, d):
        o = np.ascontiguousarray(o, np.float32).reshape(-1, 3); d = np.ascontiguousarray(d, np.float32).reshape(-1, 3)
        n = len(o)
        t = np.zeros(n); ob = np.zeros(n, np.int32); sb = np.zeros(n, np.int32); m = np.zeros(n, np.int32)
        nn = np.zeros((n, 3), np.float32); pp = np.zeros((n, 3), np.float32)
        lib().oracle_closest_batch(C.byref(self.s), float(time), n, o.ctypes.data_as(_f), d.ctypes.data_as(_f),
                                   t.ctypes.data_as(_d), ob.ctypes.data_as(_i), sb.ctypes.data_as(_i),
                                   m.ctypes.data_as(_i), nn.ctypes.data_as(_f), pp.ctypes.data_as(_f))
        return t, ob, sb, m, nn, pp

    def shadow(self, time, o, d, t_max):
        o = np.ascontiguousarray(o, np.float32).reshape(-1, 3); d = np.ascontiguousarray(d, np.float32).reshape(-1, 3)
        tm = np.ascontiguousarray(np.broadcast_to(np.asarray(t_max, np.float64), (len(o),)))
        occ = np.zeros(len(o), np.int32)
        lib().oracle_shadow_batch(C.byref(self.s), float(time), len(o), o.ctypes.data_as(_f),
                                  d.ctypes.data_as(_f), tm.ctypes.data_as(_d), occ.ctypes.data_as(_i))
        return occ


    @property
    def roots(self):
        """Record indices of the top-level objects (Scene.objects order)."""
        return [i for i, r in enumerate(self.records) if r["parent"] == -1]

    def object_shadow(self, obj, time, o, d, t_max):
        """obj.shadow_intersect(ray_i, t_max_i) for n rays (record index obj)."""
        o = np.ascontiguousarray(o, np.float32).reshape(-1, 3); d = np.ascontiguousarray(d, np.float32).reshape(-1, 3)
        tm = np.ascontiguousarray(np.broadcast_to(np.asarray(t_max, np.float64), (len(o),)))
        occ = np.zeros(len(o), np.int32)
        rc = lib().oracle_object_shadow_batch(C.byref(self.s), obj, float(time), len(o), o.ctypes.data_as(_f),
                                              d.ctypes.data_as(_f), tm.ctypes.data_as(_d), occ.ctypes.data_as(_i))
        if rc != 0:
            raise IndexError("object %d" % obj)
        return occ.astype(bool)

    def object_inside(self, obj, time, p):
        """obj.is_inside(p_i) for n points (record index obj)."""
        p = np.ascontiguousarray(p, np.float32).reshape(-1, 3)
        out = np.zeros(len(p), np.int32)
        rc = lib().oracle_object_inside_batch(C.byref(self.s), obj, float(time), len(p), p.ctypes.data_as(_f),
                                              out.ctypes.data_as(_i))
        if rc != 0:
            raise IndexError("object %d" % obj)
        return out.astype(bool)


def to_png_array(image):
    """main.py:325-327: rot90(k=1, axes=(0, 1)) then truncating uint8 conversion."""
    return (np.rot90(image, k=1, axes=(0, 1)) * 255).astype(np.uint8)


def load_bundle(name, **edits):
    """A scene dictionary from assets/scenes.json with optional edits (resolution, AA ...)."""
    repo = os.path.dirname(HERE)
    with open(os.path.join(repo, "assets", "scenes.json")) as f:
        sc = json.load(f)[name]
    for k, v in edits.items():
        sc[k] = v
    return sc, os.path.join(repo, "assets")
