"""Compile a scene-specialized kernel with hiprtc itself on the host (no GPU needed), as
librtx.so does on the box: the same header set by name (python-raytracer_amd/Makefile's
rtx_jit_sources.inc list) and the same options, so errors that only the runtime compiler
sees (its own runtime header, no <stdint.h>) show up here. Prints the log, the compile
time and the code object's size.

usage: python tools/hiprtc_check.py --split ns1 PASS      (rtx_api.hip jit_split_spec)
       python tools/hiprtc_check.py --config tsp1080      (rtx_api.hip jit_spec)"""
import ctypes as C
import os
import sys
import time

here = os.path.dirname(os.path.abspath(__file__))
repo = os.path.dirname(here)
sys.path[:0] = [here, repo, os.path.join(repo, "python-raytracer_amd"), os.path.join(repo, "tests")]
import jit_offline  # noqa: E402

csrc = os.path.join(repo, "python-raytracer_amd", "csrc")
HEADERS = [("rtx_kernels.h", os.path.join(csrc, "rtx_kernels.h")), ("rtx_trace.h", os.path.join(csrc, "rtx_trace.h")),
           ("rtx_fastmath.h", os.path.join(csrc, "rtx_fastmath.h")), ("rtx.h", os.path.join(repo, "include", "rtx.h")),
           ("rtx_split.h", os.path.join(csrc, "rtx_split.h"))]


def main():
    a = sys.argv[1:]
    if a[0] == "--split":
        opts, src = jit_offline.from_split(a[1], int(a[2]))
    else:
        opts, src = jit_offline.from_config(a[1], False)
    rtc = C.CDLL("/opt/rocm/lib/libhiprtc.so")
    prog = C.c_void_p()
    names = (C.c_char_p * len(HEADERS))(*[n.encode() for n, _ in HEADERS])
    texts = (C.c_char_p * len(HEADERS))(*[open(p, "rb").read() for _, p in HEADERS])
    rc = rtc.hiprtcCreateProgram(C.byref(prog), src.encode(), b"rtx_jit_render.hip", len(HEADERS), texts, names)
    assert rc == 0, rc
    copts = (C.c_char_p * len(opts))(*[o.encode() for o in opts])
    t0 = time.time()
    rc = rtc.hiprtcCompileProgram(prog, len(opts), copts)
    dt = time.time() - t0
    n = C.c_size_t()
    rtc.hiprtcGetProgramLogSize(prog, C.byref(n))
    log = C.create_string_buffer(n.value + 1)
    rtc.hiprtcGetProgramLog(prog, log)
    print(log.value.decode(errors="replace")[-4000:])
    if rc == 0:
        rtc.hiprtcGetCodeSize(prog, C.byref(n))
        print("compiled in %.1f s, code object %d bytes" % (dt, n.value))
    else:
        print("FAILED (hiprtc %d) after %.1f s" % (rc, dt))
    rtc.hiprtcDestroyProgram(C.byref(prog))
    sys.exit(0 if rc == 0 else 1)


if __name__ == "__main__":
    main()
