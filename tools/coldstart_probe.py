"""Cold start of one process, step by step (bench.py's setup_ms, itemized): CUDA context,
loading libhiprtc, loading librtx.so, parse, rtx_scene_create, rtx_camera_set, first and
second frame, with an empty on-disk JIT cache. Run once per process (it is the first use).
usage: python tools/coldstart_probe.py [config]"""
import ctypes
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "python-raytracer_amd")]
os.environ.setdefault("RTX_JIT_CACHE", tempfile.mkdtemp(prefix="rtx_jit_cold_"))

T = {}
t = time.perf_counter()
import torch  # noqa: E402
T["import_torch"] = time.perf_counter() - t


def step(name, fn):
    t0 = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    T[name] = time.perf_counter() - t0
    return r


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "tsp1080"
    step("cuda_context", lambda: (torch.cuda.set_device(0), torch.zeros(1, device="cuda")))
    if os.environ.get("PROBE_HIPRTC", "1") == "1":
        step("dlopen_hiprtc", lambda: ctypes.CDLL("libhiprtc.so", mode=ctypes.RTLD_GLOBAL))
    import rtx
    from rtx import _native
    step("load_librtx", _native.load)
    import bench
    sc = step("parse", lambda: bench.make_scene(cfg))
    step("scene_create", sc.native)
    step("camera_set", lambda: sc._set_camera(0, 1))
    fb = torch.empty((sc.vc.height, sc.vc.width, 3), dtype=torch.float32, device="cuda")
    step("first_frame", lambda: sc.render_device(out=fb))
    k1 = sc.last_kernel
    step("second_frame", lambda: sc.render_device(out=fb))
    k2 = sc.last_kernel
    for _ in range(20):
        sc.render_device(out=fb)
    torch.cuda.synchronize()
    time.sleep(0.5)
    step("frame_after_0.5s", lambda: sc.render_device(out=fb))
    k3 = sc.last_kernel
    print(json.dumps({"config": cfg, "ms": {k: round(v * 1e3, 3) for k, v in T.items()},
                      "kernels": [k1, k2, k3], "jit_cache": os.environ["RTX_JIT_CACHE"]}), flush=True)


if __name__ == "__main__":
    main()
