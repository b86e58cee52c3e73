"""Scene objects -> the rtx_scene_desc records of include/rtx.h.

The flattening reads only the attributes the reference's own classes carry, so it takes
either this package's objects (rtx.geometry, rtx.helperclasses) or the reference's
(provided/geometry/*.py, provided/helperclasses.py) unchanged — PyGLM vectors included
(anything ``numpy.asarray`` turns into three floats). The geometry kind is the parser's
``gtype`` ("sphere", "plane", "box", "mesh", "node": scene_parser.py:177,215-250), or,
for objects built by hand with another gtype, the attributes that define each class:

  node   Hierarchy   hierarchy_type, children, t, r, s          hierarchy.py:12-40
  mesh   Mesh        verts, faces, norms, flat_shaded,
                     bounding_volume (BoundingAABB minpos/maxpos |
                     BoundingSphere center/radius)              mesh.py:17-70, bounding_volumes.py:12-47
  sphere Sphere      center, radius                             simple_geometry.py:15-18
  box    AABB        minpos, maxpos, texture                    simple_geometry.py:180-186
  plane  Plane       point, normal, texture, texture_scale      simple_geometry.py:87-103, scene_parser.py:222-227

Materials (ID, name, mat_type, diffuse, specular, hardness, tint, refr_index) and lights
(type, colour, vector, power) are read the same way (helperclasses.py:28-59).
"""
import ctypes as C
import hashlib

import numpy as np

from . import _native as N

_MAT_CODE = {"diffuse": N.RTX_MAT_DIFFUSE, "mirror": N.RTX_MAT_MIRROR, "refractive": N.RTX_MAT_REFRACTIVE}
_HIER_CODE = {"union": N.RTX_UNION, "intersection": N.RTX_INTERSECTION, "difference": N.RTX_DIFFERENCE}
_GTYPE = {"sphere": N.RTX_SPHERE, "plane": N.RTX_PLANE, "box": N.RTX_BOX, "mesh": N.RTX_MESH, "node": N.RTX_NODE}


def vec(v):
    """A vec3 (PyGLM, numpy or a sequence) as float32[3]."""
    return np.asarray(v, dtype=np.float64).astype(np.float32).reshape(3)


def vec_rows(seq):
    """A list of vec3 (the reference's Mesh.verts / norms) or an [n, 3] array as float32[n, 3]."""
    if isinstance(seq, np.ndarray):
        return np.ascontiguousarray(seq, dtype=np.float32).reshape(-1, 3)
    return np.array([vec(v) for v in seq], dtype=np.float32).reshape(-1, 3)


def kind(g):
    """The rtx_object_type of a geometry object (see the module docstring)."""
    k = _GTYPE.get(getattr(g, "gtype", None))
    if k is not None:
        return k
    if hasattr(g, "hierarchy_type") and hasattr(g, "children"):
        return N.RTX_NODE
    if hasattr(g, "faces") and hasattr(g, "verts"):
        return N.RTX_MESH
    if hasattr(g, "center") and hasattr(g, "radius"):
        return N.RTX_SPHERE
    if hasattr(g, "minpos") and hasattr(g, "maxpos"):
        return N.RTX_BOX
    if hasattr(g, "point") and hasattr(g, "normal"):
        return N.RTX_PLANE
    raise NotImplementedError("unsupported geometry %r" % (g,))


def mesh_triangles(g):
    """(v0, v1, v2, n0, n1, n2) per face in OBJ face order, float32 [nfaces, 6, 3]. The
    vertex normals are _compute_normals' (mesh.py:53-70); flat meshes read none."""
    v = vec_rows(g.verts)
    f = np.asarray(g.faces, dtype=np.int64).reshape(-1, 3)
    if len(f) and (f.min() < 0 or f.max() >= len(v)):
        raise ValueError("%r: face index out of range" % (g,))
    norms = getattr(g, "norms", None)
    n = vec_rows(norms) if norms is not None and len(norms) else np.zeros((0, 3), np.float32)
    if bool(g.flat_shaded) or len(n) != len(v):
        n = np.zeros_like(v)
    return np.stack([v[f[:, 0]], v[f[:, 1]], v[f[:, 2]], n[f[:, 0]], n[f[:, 1]], n[f[:, 2]]], axis=1)


def _bounding_volume(o, bv):
    """Mesh.bounding_volume (mesh.py:48-51): BoundingAABB(minpos, maxpos) or
    BoundingSphere(center, radius)."""
    if hasattr(bv, "minpos"):
        o.bv_type, o.bv_a, o.bv_b = N.RTX_BV_AABB, N.f3(vec(bv.minpos)), N.f3(vec(bv.maxpos))
    else:
        o.bv_type, o.bv_a, o.bv_radius = N.RTX_BV_SPHERE, N.f3(vec(bv.center)), float(bv.radius)


def texture_rgb8(im):
    """getpixel((i, j))[:3] for every texel of a PIL image: uint8 [height, width, 3]."""
    return np.ascontiguousarray(np.asarray(im)[:, :, :3], dtype=np.uint8)


def scene_desc(objects, materials, lights, ambient):
    """Flatten a scene into an rtx_scene_desc (scene order kept; hierarchies in preorder).
    The returned descriptor keeps the host arrays it points at alive (``desc._keep``)."""
    mats = list(materials)
    index = {id(m): i for i, m in enumerate(mats)}

    def value(m):
        return (m.ID, m.name, m.mat_type, tuple(vec(m.diffuse)), tuple(vec(m.specular)), float(m.hardness),
                float(m.tint), float(m.refr_index))
    by_value = {}
    for i, m in enumerate(mats):
        by_value.setdefault(value(m), i)

    def mat_index(m):
        # a `ref` node's deep copy (scene_parser.py:199) carries copies of the scene
        # materials: same values, same slot
        if id(m) not in index:
            v = value(m)
            if v not in by_value:
                by_value[v] = len(mats)
                mats.append(m)
            index[id(m)] = by_value[v]
        return index[id(m)]

    # Records in preorder: top-level objects in scene order, each hierarchy followed by
    # its subtree (rtx.h: parent indices, children in child order).
    records = []

    def walk(g, parent):
        k = kind(g)
        records.append((g, k, parent))
        if k == N.RTX_NODE:
            me = len(records) - 1
            for c in g.children:
                walk(c, me)
    for g in objects:
        walk(g, -1)
    objs = (N.rtx_object * max(1, len(records)))()
    tris = []
    ntri = 0
    textures, tex_index = [], {}

    def texture_index(im):
        if id(im) not in tex_index:
            tex_index[id(im)] = len(textures)
            textures.append(texture_rgb8(im))
        return tex_index[id(im)]
    for i, (g, k, parent) in enumerate(records):
        o = objs[i]
        o.type = k
        o.parent = parent
        o.texture = -1
        o.texture_scale = 1.0
        o.n_mats = len(g.materials)
        for j, m in enumerate(g.materials[:2]):
            o.mat[j] = mat_index(m)
        speed = getattr(g, "speed", None)
        o.has_speed = 0 if speed is None else 1
        o.speed = N.f3(vec(speed) if speed is not None else (0, 0, 0))
        if k == N.RTX_NODE:
            o.hierarchy_type = _HIER_CODE.get(g.hierarchy_type, N.RTX_HIER_OTHER)
            o.trs[:] = [float(x) for x in np.concatenate([vec(g.t), vec(g.r), vec(g.s)])]
        elif k == N.RTX_SPHERE:
            o.a, o.radius = N.f3(vec(g.center)), float(g.radius)
        elif k == N.RTX_PLANE:
            o.a, o.b = N.f3(vec(g.point)), N.f3(vec(g.normal))
            if getattr(g, "texture", None) is not None:
                # Plane.get_diffuse: texture_scale, or 1.0 when unset (simple_geometry.py:157-160)
                o.texture, o.texture_scale = texture_index(g.texture), float(getattr(g, "texture_scale", 1.0))
        elif k == N.RTX_BOX:
            o.a, o.b = N.f3(vec(g.minpos)), N.f3(vec(g.maxpos))
            if getattr(g, "texture", None) is not None:
                o.texture = texture_index(g.texture)
        else:  # mesh
            t = mesh_triangles(g)
            o.tri_begin, o.tri_count = ntri, len(t)
            ntri += len(t)
            tris.append(t)
            o.flat = 1 if g.flat_shaded else 0
            _bounding_volume(o, g.bounding_volume)
        if k != N.RTX_NODE and not g.materials:
            raise IndexError("%r has no material: the reference raises IndexError (list index out of "
                             "range) when it is hit" % (g,))
    cm = (N.rtx_material * max(1, len(mats)))()
    for i, m in enumerate(mats):
        cm[i].diffuse, cm[i].specular = N.f3(vec(m.diffuse)), N.f3(vec(m.specular))
        cm[i].hardness = float(m.hardness)
        cm[i].type = _MAT_CODE.get(m.mat_type, N.RTX_MAT_DIFFUSE)  # other strings shade as diffuse
        cm[i].tint, cm[i].refr_index = float(m.tint), float(m.refr_index)
    lights = list(lights)
    cl = (N.rtx_light * max(1, len(lights)))()
    for i, L in enumerate(lights):
        cl[i].type = N.RTX_LIGHT_POINT if L.type == "point" else N.RTX_LIGHT_DIRECTIONAL
        cl[i].colour, cl[i].vector, cl[i].power = N.f3(vec(L.colour)), N.f3(vec(L.vector)), float(L.power)
    tri = np.ascontiguousarray(np.concatenate(tris).astype(np.float32)) if tris else np.zeros((1, 6, 3), np.float32)
    desc = N.rtx_scene_desc()
    desc.n_objects, desc.objects = len(records), objs
    desc.n_materials, desc.materials = len(mats), cm
    desc.n_lights, desc.lights = len(lights), cl
    desc.n_triangles = ntri
    desc.triangles = tri.ctypes.data_as(C.POINTER(N.rtx_triangle))
    desc.ambient = N.f3(vec(ambient))
    ct = (N.rtx_texture * max(1, len(textures)))()
    for i, t in enumerate(textures):
        ct[i].height, ct[i].width = t.shape[0], t.shape[1]
        ct[i].rgb = t.ctypes.data_as(C.POINTER(C.c_uint8))
    desc.n_textures, desc.textures = len(textures), ct
    desc._keep = (objs, cm, cl, tri, ct, textures)
    return desc


def desc_bytes(desc):
    """A canonical byte image of a descriptor (record structs + the arrays they point at),
    for comparing two descriptors (tests)."""
    def raw(ptr, n, st):
        return C.string_at(C.cast(ptr, C.c_void_p).value, C.sizeof(st) * n) if n else b""
    out = [raw(desc.objects, desc.n_objects, N.rtx_object)]
    out.append(raw(desc.materials, desc.n_materials, N.rtx_material))
    out.append(raw(desc.lights, desc.n_lights, N.rtx_light))
    out.append(raw(desc.triangles, desc.n_triangles, N.rtx_triangle))
    out.append(bytes(desc.ambient))
    for i in range(desc.n_textures):
        t = desc.textures[i]
        out.append(b"%d,%d" % (t.width, t.height) + C.string_at(t.rgb, 3 * t.width * t.height))
    return out


def desc_digest(desc):
    """A digest of desc_bytes: equal for descriptors the library would upload alike."""
    h = hashlib.blake2b(digest_size=16)
    for b in desc_bytes(desc):
        h.update(len(b).to_bytes(8, "little"))
        h.update(b)
    return h.digest()
