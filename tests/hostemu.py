"""Tests-only harness: the device source run on the host CPU (tests/native/rtx_hostemu.hip)."""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "rtx_hostemu.hip")
LIB = os.path.join(HERE, "native", "librtx_hostemu.so")
DEPS = [SRC, os.path.join(HERE, "..", "python-raytracer_amd", "csrc", "rtx_api.hip"),
        os.path.join(HERE, "..", "python-raytracer_amd", "csrc", "rtx_trace.h"),
        os.path.join(HERE, "..", "python-raytracer_amd", "csrc", "rtx_kernels.h"),
        os.path.join(HERE, "..", "python-raytracer_amd", "csrc", "rtx_fastmath.h"),
        os.path.join(HERE, "..", "python-raytracer_amd", "csrc", "rtx_launch.h"),
        os.path.join(HERE, "..", "python-raytracer_amd", "csrc", "rtx_split.h"),
        os.path.join(HERE, "..", "python-raytracer_amd", "csrc", "rtx_bins.h"),
        os.path.join(HERE, "..", "python-raytracer_amd", "csrc", "rtx_jit_sources.inc"),
        os.path.join(HERE, "..", "include", "rtx.h")]


def build():
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(p) for p in DEPS):
        subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O2", "-std=c++17", "-ffp-contract=off", "-fopenmp",
                               "-fPIC", "-shared", "-o", LIB, SRC, "-lhiprtc"])
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = C.CDLL(build())
        vp = C.c_void_p
        _lib.rtx_hostemu_render.argtypes = [vp, vp, C.c_int32, C.c_int32, vp, vp, C.c_int]
        _lib.rtx_hostemu_render_rows.argtypes = [vp, vp, vp, C.c_int32, vp, C.c_int]
        _lib.rtx_hostemu_intersect.argtypes = [vp, C.c_int64, vp, vp, C.c_double, vp, vp, vp, vp, vp]
        _lib.rtx_hostemu_occluded.argtypes = [vp, C.c_int64, vp, vp, vp, C.c_double, vp]
        _lib.rtx_hostemu_occluded_light.argtypes = [vp, C.c_int64, vp, C.c_int32, C.c_int32, vp, vp]
        _lib.rtx_hostemu_last_error.restype = C.c_char_p
    return _lib


def _chk(rc):
    if rc != 0:
        raise RuntimeError("hostemu failed %d: %s" % (rc, lib().rtx_hostemu_last_error().decode()))


def render(scene, subimage=0, tasks=1, threads=8):
    """Same result layout as Scene.render(): float64 (strip_w, H, 3). Returns (image, counters)."""
    sd = scene.scene_desc()
    cd, tables = scene.camera_desc(subimage, tasks)
    H = scene.vc.height
    fb = np.zeros((H, cd.ncols, 3), np.float32)
    cnt = np.zeros(16, np.uint64)
    _chk(lib().rtx_hostemu_render(C.addressof(sd), C.addressof(cd), 0, H, fb.ctypes.data, cnt.ctypes.data, threads))
    img = np.ascontiguousarray(np.transpose(fb[::-1], (1, 0, 2))).astype(np.float64)
    return img, cnt


def render_split(scene, subimage=0, tasks=1, threads=8, budget=1 << 31, ratio=9.0, with_redone=False):
    """The hierarchy/texture scenes' three split passes (csrc/rtx_split.h) on the host,
    chunked like render_split of librtx.so (`budget` record bytes per chunk, `ratio` deeper
    records per sample; the default reserves every level, so no block is redone and the
    tallies are the passes' own); same layout as render(). with_redone: also the number of
    blocks rendered again because their chains found the pool full."""
    sd = scene.scene_desc()
    cd, tables = scene.camera_desc(subimage, tasks)
    H = scene.vc.height
    fb = np.zeros((H, cd.ncols, 3), np.float32)
    cnt = np.zeros(16, np.uint64)
    redone = C.c_int64(0)
    f = lib().rtx_hostemu_render_split
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p, C.c_int, C.c_int64,
                  C.c_double, C.c_void_p]
    _chk(f(C.addressof(sd), C.addressof(cd), 0, H, fb.ctypes.data, cnt.ctypes.data, threads, budget, ratio,
           C.addressof(redone)))
    img = np.ascontiguousarray(np.transpose(fb[::-1], (1, 0, 2))).astype(np.float64)
    return (img, cnt, redone.value) if with_redone else (img, cnt)


def render_rows(scene, rows, threads=8):
    """Image rows ``rows`` (row 0 = top) only, packed: float32 [len(rows), W, 3], the
    block one rank renders (rtx_render / rtx_render_groups layout)."""
    sd = scene.scene_desc()
    cd, tables = scene.camera_desc()
    rows = np.ascontiguousarray(np.asarray(rows, np.int32))
    fb = np.zeros((len(rows), cd.ncols, 3), np.float32)
    _chk(lib().rtx_hostemu_render_rows(C.addressof(sd), C.addressof(cd), rows.ctypes.data, len(rows), fb.ctypes.data,
                                       threads))
    return fb


def intersect(scene, o, d, time=0.0):
    sd = scene.scene_desc()
    o = np.ascontiguousarray(np.asarray(o, np.float32).reshape(-1, 3).T)
    d = np.ascontiguousarray(np.asarray(d, np.float32).reshape(-1, 3).T)
    n = o.shape[1]
    t = np.zeros(n); ob = np.zeros(n, np.int32); m = np.zeros(n, np.int32)
    nn = np.zeros((3, n), np.float32); pp = np.zeros((3, n), np.float32)
    _chk(lib().rtx_hostemu_intersect(C.addressof(sd), n, o.ctypes.data, d.ctypes.data, time, t.ctypes.data,
                                     ob.ctypes.data, m.ctypes.data, nn.ctypes.data, pp.ctypes.data))
    return dict(t=t, obj=ob, mat=m, normal=nn.T.copy(), position=pp.T.copy())


def occluded(scene, o, d, t_max, time=0.0):
    sd = scene.scene_desc()
    o = np.ascontiguousarray(np.asarray(o, np.float32).reshape(-1, 3).T)
    d = np.ascontiguousarray(np.asarray(d, np.float32).reshape(-1, 3).T)
    n = o.shape[1]
    tm = np.ascontiguousarray(np.broadcast_to(np.asarray(t_max, np.float64), (n,)))
    occ = np.zeros(n, np.uint8)
    _chk(lib().rtx_hostemu_occluded(C.addressof(sd), n, o.ctypes.data, d.ctypes.data, tm.ctypes.data, time,
                                    occ.ctypes.data))
    return occ.astype(bool)


def occluded_light(scene, o, light, grids):
    """Shadow rays from points o to point light ``light`` as regular_lighting casts them
    (d = L - o, t_max 1), through the light's grid (grids=True; None if it has none) or
    the BVH walk. Returns (occluded bool [n], grid cell per point: -1 outside the cone,
    -2 walked)."""
    sd = scene.scene_desc()
    o = np.ascontiguousarray(np.asarray(o, np.float32).reshape(-1, 3).T)
    n = o.shape[1]
    occ = np.zeros(n, np.uint8)
    cells = np.zeros(n, np.int32)
    rc = lib().rtx_hostemu_occluded_light(C.addressof(sd), n, o.ctypes.data, light, 1 if grids else 0,
                                          occ.ctypes.data, cells.ctypes.data)
    if rc == -1:
        return None
    _chk(rc)
    return occ.astype(bool), cells


def bins(scene, subimage=0, tasks=1, roots=False):
    """The primary-ray bins rtx_camera_set builds (rtx_api.hip primary_bins): the object
    mask (uint32 [bins_y, bins_x]: spheres bits 0-15, boxes 16-31) and mesh-face count per
    8x8 bin (roots=True: and the hierarchy-root mask), or None when the camera has none."""
    sd = scene.scene_desc()
    cd, tables = scene.camera_desc(subimage, tasks)
    bx, by = (cd.ncols + 7) // 8, (cd.height + 7) // 8
    mask = np.zeros(bx * by, np.uint32)
    nf = np.zeros(bx * by, np.int32)
    rm = np.zeros(bx * by, np.uint32)
    f = lib().rtx_hostemu_bins
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64]
    f.restype = C.c_int64
    n = f(C.addressof(sd), C.addressof(cd), mask.ctypes.data, nf.ctypes.data, rm.ctypes.data, bx * by)
    if n == 0:
        return None
    assert n == bx * by, n
    out = (mask.reshape(by, bx), nf.reshape(by, bx))
    return out + (rm.reshape(by, bx),) if roots else out


def dir_shadow_mask(scene, p, light):
    """What directional light ``light``'s shadow rays from points p may meet by its shadow
    grid (built for time 0): uint32 [n, 2] = (sphere bits 0-15 | box bits 16-31, hierarchy
    root bits), all ones where everything is tested; None when the light has no grid."""
    sd = scene.scene_desc()
    p = np.ascontiguousarray(np.asarray(p, np.float32).reshape(-1, 3).T)
    n = p.shape[1]
    out = np.zeros((n, 2), np.uint32)
    f = lib().rtx_hostemu_dir_shadow_mask
    f.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int32, C.c_void_p]
    rc = f(C.addressof(sd), n, p.ctypes.data, light, out.ctypes.data)
    if rc == -1:
        return None
    _chk(rc)
    return out


def dsgrid_self(scene, light, subimage=0, tasks=1):
    """The boxes (bits 16-31) whose own shadow test toward directional light ``light`` a
    camera ray's hit on them skips (DSGrid.self_boxes), or None without a grid."""
    sd = scene.scene_desc()
    cd, tables = scene.camera_desc(subimage, tasks)
    f = lib().rtx_hostemu_dsgrid_self
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
    f.restype = C.c_int64
    r = f(C.addressof(sd), C.addressof(cd), light)
    return None if r < 0 else int(r)


def plane_self(scene):
    """The planes' self-test limits for this camera (rtx_api.hip plane_self_limits):
    float32 [n_lights, 4], -1 where a plane's own shadow test is always run."""
    sd = scene.scene_desc()
    cd, tables = scene.camera_desc()
    out = np.zeros((sd.n_lights, 4), np.float32)
    f = lib().rtx_hostemu_plane_self
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    _chk(f(C.addressof(sd), C.addressof(cd), out.ctypes.data))
    return out


def philox(ctr, key):
    """The device's Philox4x32-10 of one counter (4 uint32) and key (k0, k1)."""
    c = np.ascontiguousarray(np.asarray(ctr, np.uint32))
    f = lib().rtx_hostemu_philox
    f.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
    f.restype = None
    f(c.ctypes.data, int(key[0]), int(key[1]))
    return c


def jitter(seed, col0, ncols, height, n_dof, n_aa):
    """The device's production jitter uniforms (jitter_block / jitter_rnd) in the replay
    table's layout, float32 flat."""
    out = np.zeros(ncols * height * n_dof * n_aa * 3, np.float32)
    f = lib().rtx_hostemu_jitter
    f.argtypes = [C.c_uint64, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_void_p]
    f.restype = None
    f(seed, col0, ncols, height, n_dof, n_aa, out.ctypes.data)
    return out


def jit_baked(scene):
    """The scene-record prelude librtx.so hands its scene-specialized kernels
    (rtx_api.hip jit_baked_records), as a string."""
    sd = scene.scene_desc()
    f = lib().rtx_hostemu_jit_baked
    f.argtypes = [C.c_void_p, C.c_char_p, C.c_int64]
    f.restype = C.c_int64
    n = f(C.addressof(sd), None, 0)
    if n < 0:
        raise RuntimeError("hostemu jit_baked failed: %s" % lib().rtx_hostemu_last_error().decode())
    buf = C.create_string_buffer(int(n) + 1)
    f(C.addressof(sd), buf, n + 1)
    return buf.value.decode()


def set_option(name, value):
    """rtx_set_option of the host emulation's copy of the library options."""
    f = lib().rtx_set_option
    f.argtypes = [C.c_char_p, C.c_char_p]
    _chk(f(str(name).encode(), str(value).encode()))
