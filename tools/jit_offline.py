"""Compile a scene-specialized kernel offline (no GPU): ISA (.s) and the register/scratch
report. The hiprtc options and source come either from an RTX_JIT_DUMP=1 log that
librtx.so printed on the GPU box, or -- with --config -- straight from the host build of
rtx_api.hip's jit_spec (tests/native/librtx_hostemu.so) for a bench.py config.

usage: python tools/jit_offline.py LOG KERNEL OUT.s [extra hipcc flags...]
       python tools/jit_offline.py --config tsp1080 [--rgb8] OUT.s [extra hipcc flags...]
       python tools/jit_offline.py --split ns1 PASS OUT.s [...]  (a hierarchy config's specialized
           split pass: 0 trace, 1 shadow; rtx_api.hip jit_split_spec)
Environment variables that change the specialization (RTX_JIT_FLAGS, RTX_BINS, ...)
apply in the --config form as they would on the box."""
import ctypes as C
import os
import re
import shlex
import subprocess
import sys
import tempfile

here = os.path.dirname(os.path.abspath(__file__))
repo = os.path.dirname(here)
csrc = os.path.join(repo, "python-raytracer_amd", "csrc")
inc = os.path.join(repo, "include")


def from_log(log, kern):
    lines = open(log).read().split("\n")
    for i, ln in enumerate(lines):
        if ln.startswith("librtx: jit %s:" % kern):
            opts = shlex.split(ln.split(":", 2)[2])
            src = []
            for s in lines[i + 1:]:
                src.append(s)
                if s.startswith("}") and any("render_body" in x for x in src[-3:]):
                    break
            return opts, "\n".join(src) + "\n"
    sys.exit("kernel %s not in %s" % (kern, log))


def from_config(cfg, rgb8):
    sys.path[:0] = [repo, os.path.join(repo, "python-raytracer_amd"), os.path.join(repo, "tests")]
    import bench
    import hostemu
    sc = bench.make_scene(cfg)
    sd = sc.scene_desc()
    cd, _tables = sc.camera_desc()
    f = hostemu.lib().rtx_hostemu_jit_spec
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_char_p, C.c_int64]
    f.restype = C.c_int64
    n = f(C.addressof(sd), C.addressof(cd), 0, 1 if rgb8 else 0, None, 0)
    if n < 0:
        sys.exit("config %s runs the generic kernel (jit_spec %d)" % (cfg, n))
    buf = C.create_string_buffer(int(n) + 1)
    f(C.addressof(sd), C.addressof(cd), 0, 1 if rgb8 else 0, buf, n + 1)
    text = buf.value.decode()
    head, src = text.split("\n\n", 1)
    name, *opts = head.split("\n")
    print("kernel", name)
    return opts, src


def from_split(cfg, pas):
    sys.path[:0] = [repo, os.path.join(repo, "python-raytracer_amd"), os.path.join(repo, "tests")]
    import bench
    import hostemu
    sc = bench.make_scene(cfg)
    sd = sc.scene_desc()
    cd, _tables = sc.camera_desc()
    f = hostemu.lib().rtx_hostemu_jit_split
    f.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_char_p, C.c_int64, C.POINTER(C.c_int64)]
    f.restype = C.c_int64
    cost = C.c_int64()
    jit = 1 if cd.jitter else 0
    n = f(C.addressof(sd), pas, 0, jit, None, 0, C.byref(cost))
    print("csg_cost", cost.value)
    if n < 0:
        sys.exit("config %s runs the precompiled split passes (%d)" % (cfg, n))
    buf = C.create_string_buffer(int(n) + 1)
    f(C.addressof(sd), pas, 0, jit, buf, n + 1, C.byref(cost))
    head, src = buf.value.decode().split("\n\n", 1)
    name, *opts = head.split("\n")
    print("kernel", name)
    return opts, src


def main():
    a = sys.argv[1:]
    if a[0] == "--split":
        opts, src = from_split(a[1], int(a[2]))
        out, extra = a[3], a[4:]
    elif a[0] == "--config":
        cfg = a[1]
        rgb8 = len(a) > 2 and a[2] == "--rgb8"
        a = a[3 if rgb8 else 2:]
        opts, src = from_config(cfg, rgb8)
        out, extra = a[0], a[1:]
    else:
        opts, src = from_log(a[0], a[1])
        out, extra = a[2], a[3:]
    with tempfile.NamedTemporaryFile("w", suffix=".hip", delete=False) as f:
        f.write(src)
        path = f.name
    opts = [o for o in opts if not o.startswith("--offload-arch")]
    base = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "--cuda-device-only", "-I", csrc, "-I", inc] + opts + extra
    subprocess.check_call(base + ["-S", "-o", out, path])
    r = subprocess.run(base + ["-c", "-o", "/tmp/jit_offline.o", "-Rpass-analysis=kernel-resource-usage", path],
                       capture_output=True, text=True)
    for m in re.findall(r"(Function Name: \S+|VGPRs: \d+|ScratchSize \[bytes/lane\]: \d+|Occupancy \[waves/SIMD\]: \d+|SGPRs Spill: \d+|"
                        r"VGPRs Spill: \d+|TotalSGPRs: \d+|LDS Size \[bytes/block\]: \d+)", r.stderr):
        print(m)
    os.unlink(path)


if __name__ == "__main__":
    main()
