"""Compile a scene-specialized kernel offline from an RTX_JIT_DUMP=1 log (the hiprtc options
and source librtx.so printed on the GPU box): ISA (.s) and the register/scratch report.
usage: python tools/jit_offline.py LOG KERNEL OUT.s [extra hipcc flags...]"""
import os
import re
import shlex
import subprocess
import sys
import tempfile

log, kern, out = sys.argv[1:4]
extra = sys.argv[4:]
lines = open(log).read().split("\n")
for i, ln in enumerate(lines):
    if ln.startswith("librtx: jit %s:" % kern):
        opts = shlex.split(ln.split(":", 2)[2])
        src = []
        for s in lines[i + 1:]:
            src.append(s)
            if s.startswith("}") and any("render_body" in x for x in src[-3:]):
                break
        break
else:
    sys.exit("kernel %s not in %s" % (kern, log))
here = os.path.dirname(os.path.abspath(__file__))
csrc = os.path.join(here, "..", "python-raytracer_amd", "csrc")
inc = os.path.join(here, "..", "include")
with tempfile.NamedTemporaryFile("w", suffix=".hip", delete=False) as f:
    f.write("\n".join(src) + "\n")
    path = f.name
opts = [o for o in opts if not o.startswith("--offload-arch")]
base = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "--cuda-device-only", "-I", csrc, "-I", inc] + opts + extra
subprocess.check_call(base + ["-S", "-o", out, path])
r = subprocess.run(base + ["-c", "-o", "/tmp/jit_offline.o", "-Rpass-analysis=kernel-resource-usage", path],
                   capture_output=True, text=True)
for m in re.findall(r"(VGPRs: \d+|ScratchSize \[bytes/lane\]: \d+|Occupancy \[waves/SIMD\]: \d+|SGPRs Spill: \d+|"
                    r"TotalSGPRs: \d+)", r.stderr):
    print(m)
os.unlink(path)
