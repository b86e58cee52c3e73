"""Wavefront (SoA, one launch per ray level) vs megakernel (rtx_render) on the MI355X:
bit-equality of the frames and time per frame, both through _abl/librtx_wf.so (built by
tools/wavefront/build.sh; it carries the library's own rtx_render too).
usage: python tools/wavefront/bench_wf.py [--steps K]  -> one JSON line per scene"""
import argparse
import ctypes as C
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "python-raytracer_amd"))
import torch  # noqa: E402
import rtx  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    lib = C.CDLL(os.path.join(REPO, "_abl", "librtx_wf.so"))
    vp = C.c_void_p
    lib.rtx_scene_create.argtypes = [vp, vp]
    lib.rtx_camera_set.argtypes = [vp, vp]
    lib.rtx_render.argtypes = [vp, C.c_int32, C.c_int32, vp, vp, vp]
    lib.rtx_wf_render.argtypes = [vp, vp, vp]
    lib.rtx_last_error.restype = C.c_char_p
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream()
    sh = C.c_void_p(stream.cuda_stream)

    def chk(rc):
        if rc != 0:
            raise RuntimeError(lib.rtx_last_error().decode())

    for name in ("TwoSpheresPlane", "MirrorRefraction", "TorusMesh"):
        from rtx.io import bundled_scene_dict
        d = bundled_scene_dict(name, resolution=(1920, 1080))
        d["AA"] = {"jitter": False, "samples": 1}  # the bench's 1-spp configs
        d["__base_dir__"] = os.path.join(REPO, "assets")
        sc = rtx.load_scene(d, verbose=False)
        sd = sc.scene_desc()
        cd, tables = sc.camera_desc()
        s = C.c_void_p()
        chk(lib.rtx_scene_create(C.addressof(sd), C.byref(s)))
        chk(lib.rtx_camera_set(s, C.addressof(cd)))
        H, W = cd.height, cd.ncols
        fa = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
        fb = torch.empty_like(fa)
        fb.fill_(float("nan"))
        mega = lambda: chk(lib.rtx_render(s, 0, H, C.c_void_p(fa.data_ptr()), None, sh))  # noqa: E731
        wave = lambda: chk(lib.rtx_wf_render(s, C.c_void_p(fb.data_ptr()), sh))  # noqa: E731
        out = {"scene": name, "res": [W, H]}
        for tag, fn in (("megakernel", mega), ("wavefront", wave)):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(a.steps):
                fn()
            e1.record(stream)
            torch.cuda.synchronize()
            out[tag + "_ms"] = e0.elapsed_time(e1) / a.steps
        out["bit_identical"] = bool(torch.equal(fa, fb))
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
