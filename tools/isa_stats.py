"""Instruction mix of each kernel in a hipcc -S output (device assembly)."""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else "k_render"
for m in re.finditer(r"^(_Z\w+|rtx_jit\w+):\s*(?:;.*)?$", s, re.M):
    name = m.group(1)
    if pat not in name:
        continue
    end = s.find(".Lfunc_end", m.end())
    body = s[m.end():end]
    ins = [l.split()[0] for l in body.split("\n") if l.startswith("\t") and l.strip() and not l.strip().startswith((".", ";"))]
    c = Counter(ins)
    f64 = sum(v for k, v in c.items() if "f64" in k)
    meta = re.search(r"\.name:\s+" + re.escape(name) + r"\n(.*?)\.\.\.|- \.args:.*?\.name:\s+" + re.escape(name), s, re.S)
    print("%-70s instrs %5d  f64 %4d  writelane %3d readlane %3d  s_load %3d  global_load %3d  scratch %d" % (
        name[:70], len(ins), f64, c["v_writelane_b32"], c["v_readlane_b32"],
        sum(v for k, v in c.items() if k.startswith("s_load")), sum(v for k, v in c.items() if k.startswith("global_load")),
        sum(v for k, v in c.items() if "scratch" in k)))
    if "-v" in sys.argv:
        print("   ", c.most_common(40))
