"""ctypes binding of librtx.so (include/rtx.h).

The binding fails loudly: there is no CPU fallback anywhere in the product path. If the
HIP library is missing or cannot be loaded, importing the render entry points raises.
torch is imported first so that the HIP runtime librtx.so links against is the one
PyTorch-ROCm already loaded (both carry the soname libamdhip64.so.7).
"""
import ctypes as C
import os
import threading

import torch  # noqa: F401  (loads the process' HIP runtime before librtx.so)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_lib", "librtx.so")
# Experiment builds (tools/ablate.sh) point this at another build of the same HIP source.
_BUILT_PATH = LIB_PATH
LIB_PATH = os.environ.get("RTX_LIB_OVERRIDE", LIB_PATH)
ABI_VERSION = 5

RTX_OK, RTX_ERR_INVALID, RTX_ERR_HIP, RTX_ERR_UNSUPPORTED, RTX_ERR_STATE = 0, -1, -2, -3, -4
RTX_SPHERE, RTX_PLANE, RTX_BOX, RTX_MESH, RTX_NODE = 0, 1, 2, 3, 4
RTX_UNION, RTX_INTERSECTION, RTX_DIFFERENCE, RTX_HIER_OTHER = 0, 1, 2, 3
RTX_MAT_DIFFUSE, RTX_MAT_MIRROR, RTX_MAT_REFRACTIVE = 0, 1, 2
RTX_LIGHT_POINT, RTX_LIGHT_DIRECTIONAL = 0, 1
RTX_BV_AABB, RTX_BV_SPHERE = 0, 1
RTX_JITTER_OFF, RTX_JITTER_PHILOX, RTX_JITTER_REPLAY = 0, 1, 2
RTX_COUNTERS = 16
RTX_CNT_SHADOW, RTX_CNT_SHADE, RTX_CNT_TRI = 10, 11, 12

_f3 = C.c_float * 3


class rtx_object(C.Structure):
    _fields_ = [("type", C.c_int32), ("n_mats", C.c_int32), ("mat", C.c_int32 * 2),
                ("has_speed", C.c_int32), ("speed", _f3), ("a", _f3), ("b", _f3),
                ("radius", C.c_double), ("tri_begin", C.c_int32), ("tri_count", C.c_int32),
                ("bv_type", C.c_int32), ("flat", C.c_int32), ("bv_a", _f3), ("bv_b", _f3),
                ("bv_radius", C.c_double), ("parent", C.c_int32), ("hierarchy_type", C.c_int32),
                ("trs", C.c_float * 9), ("texture", C.c_int32), ("texture_scale", C.c_double)]


class rtx_texture(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("rgb", C.POINTER(C.c_uint8))]


class rtx_triangle(C.Structure):
    _fields_ = [("v0", _f3), ("v1", _f3), ("v2", _f3), ("n0", _f3), ("n1", _f3), ("n2", _f3)]


class rtx_material(C.Structure):
    _fields_ = [("diffuse", _f3), ("specular", _f3), ("hardness", C.c_double), ("type", C.c_int32),
                ("tint", C.c_double), ("refr_index", C.c_double)]


class rtx_light(C.Structure):
    _fields_ = [("type", C.c_int32), ("colour", _f3), ("vector", _f3), ("power", C.c_double)]


class rtx_scene_desc(C.Structure):
    _fields_ = [("n_objects", C.c_int32), ("objects", C.POINTER(rtx_object)),
                ("n_materials", C.c_int32), ("materials", C.POINTER(rtx_material)),
                ("n_lights", C.c_int32), ("lights", C.POINTER(rtx_light)),
                ("n_triangles", C.c_int32), ("triangles", C.POINTER(rtx_triangle)),
                ("ambient", _f3), ("n_textures", C.c_int32), ("textures", C.POINTER(rtx_texture))]


_pf = C.POINTER(C.c_float)
_pd = C.POINTER(C.c_double)


class rtx_camera_desc(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("col0", C.c_int32), ("ncols", C.c_int32),
                ("xs", _pf), ("ys", _pf), ("position", _f3), ("u", _f3), ("v", _f3), ("w", _f3),
                ("d", C.c_double), ("focal_length", C.c_double), ("n_dof", C.c_int32), ("n_aa", C.c_int32),
                ("dof_origins", _pf), ("aa_origins", _pf), ("n_times", C.c_int32), ("times", _pd),
                ("jitter", C.c_int32), ("jitter_scale", C.c_double), ("seed", C.c_uint64), ("noise", _pf)]


class RtxError(RuntimeError):
    def __init__(self, fn, code, msg):
        super().__init__("%s failed (%d): %s" % (fn, code, msg))
        self.code = code


_lock = threading.Lock()
_lib = None

EXPORTS = ["rtx_abi_version", "rtx_last_error", "rtx_scene_create", "rtx_scene_destroy", "rtx_camera_set",
           "rtx_render", "rtx_render_groups", "rtx_group_rows", "rtx_intersect", "rtx_occluded", "rtx_fb_to_rgb8",
           "rtx_render_rgb8", "rtx_render_groups_rgb8", "rtx_last_kernel", "rtx_render_frames",
           "rtx_render_groups_frames", "rtx_jit_modules", "rtx_set_option", "rtx_get_option", "rtx_option_name",
           "rtx_graph_launch", "rtx_jit_wait"]


def load():
    """Load librtx.so once; raises if it is missing (run __graft_entry__.build())."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("librtx.so not built at %s — run `python -c 'import __graft_entry__ as g; g.build()'`"
                               % LIB_PATH)
        lib = C.CDLL(LIB_PATH)
        vp = C.c_void_p
        lib.rtx_abi_version.restype = C.c_int
        lib.rtx_last_error.restype = C.c_char_p
        lib.rtx_scene_create.argtypes = [C.POINTER(rtx_scene_desc), C.POINTER(vp)]
        lib.rtx_scene_destroy.argtypes = [vp]
        lib.rtx_camera_set.argtypes = [vp, C.POINTER(rtx_camera_desc)]
        lib.rtx_render.argtypes = [vp, C.c_int32, C.c_int32, vp, vp, vp]
        lib.rtx_render_groups.argtypes = [vp, C.c_int32, C.c_int32, vp, vp, vp]
        lib.rtx_render_rgb8.argtypes = [vp, C.c_int32, C.c_int32, vp, vp, vp]
        lib.rtx_render_groups_rgb8.argtypes = [vp, C.c_int32, C.c_int32, vp, vp, vp]
        lib.rtx_render_frames.argtypes = [vp, C.c_int32, C.c_int32, vp, C.c_int32, C.c_int32, C.c_int64, vp, vp]
        lib.rtx_render_groups_frames.argtypes = [vp, C.c_int32, C.c_int32, vp, C.c_int32, C.c_int32, C.c_int64, vp,
                                                 vp]
        lib.rtx_group_rows.argtypes = [C.c_int32, C.c_int32, C.c_int32]
        lib.rtx_group_rows.restype = C.c_int32
        lib.rtx_intersect.argtypes = [vp, C.c_int64, vp, vp, C.c_double, vp, vp, vp, vp, vp, vp]
        lib.rtx_occluded.argtypes = [vp, C.c_int64, vp, vp, vp, C.c_double, vp, vp]
        lib.rtx_fb_to_rgb8.argtypes = [vp, vp, C.c_int64, vp]
        for fn in EXPORTS:  # every status-returning entry point (not the string / count ones)
            if not hasattr(lib, fn):
                continue  # (an earlier round's library, see below)
            if fn not in ("rtx_abi_version", "rtx_last_error", "rtx_last_kernel", "rtx_group_rows", "rtx_jit_modules",
                          "rtx_option_name", "rtx_jit_wait"):
                getattr(lib, fn).restype = C.c_int
        lib.rtx_last_kernel.argtypes = [vp]
        lib.rtx_last_kernel.restype = C.c_char_p
        lib.rtx_jit_modules.argtypes = []
        lib.rtx_jit_modules.restype = C.c_int32
        v = lib.rtx_abi_version()
        # (tools/ab_lib.sh times an earlier round's library through RTX_LIB_OVERRIDE: ABI 4
        # lacks only the options, which the render calls do not use)
        older = v == 4 and LIB_PATH != _BUILT_PATH
        if v != ABI_VERSION and not older:
            raise RuntimeError("librtx.so ABI %d != binding ABI %d" % (v, ABI_VERSION))
        if not older:
            lib.rtx_set_option.argtypes = [C.c_char_p, C.c_char_p]
            lib.rtx_get_option.argtypes = [C.c_char_p, C.c_char_p, C.c_int32]
            lib.rtx_option_name.argtypes = [C.c_int32]
            lib.rtx_option_name.restype = C.c_char_p
        if hasattr(lib, "rtx_graph_launch"):
            lib.rtx_graph_launch.argtypes = [vp, C.c_int32, vp]
            lib.rtx_jit_wait.argtypes = [vp, C.c_int32]
            lib.rtx_jit_wait.restype = C.c_int32
        _lib = lib
        return lib


def check(fn, rc):
    if rc != RTX_OK:
        raise RtxError(fn, rc, load().rtx_last_error().decode(errors="replace"))


def call(fn, *args):
    check(fn, getattr(load(), fn)(*args))


def set_option(name, value):
    """rtx_set_option: a library option by name (include/rtx.h; INTEGRATION.md "Options")."""
    call("rtx_set_option", str(name).encode(), str(value).encode())


def get_option(name):
    """rtx_get_option: the option's value (a float, or a str for jit_cache / jit_flags)."""
    buf = C.create_string_buffer(4096)
    call("rtx_get_option", str(name).encode(), buf, len(buf))
    v = buf.value.decode()
    if name in ("jit_cache", "jit_flags"):
        return v
    return float(v)


def option_names():
    lib = load()
    out, i = [], 0
    while True:
        n = lib.rtx_option_name(i)
        if n is None:
            return out
        out.append(n.decode())
        i += 1


def f3(v):
    a = _f3()
    a[0], a[1], a[2] = float(v[0]), float(v[1]), float(v[2])
    return a
