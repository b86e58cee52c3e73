"""The longest waves of a wave timeline (tools/wave_timeline.py --npz, taken with the tile
schedule and the XCD block order off -- RTX_TILE_SCHED=0 RTX_XCD_MAP=0 -- so wave w renders
tile w in row-major order) with their
tiles: (tile row, tile column), duration, and the tile's primary-ray mesh face count from
the host emulation's bins. usage: python tools/timeline_tiles.py wt.npz config [top]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "python-raytracer_amd"), os.path.join(REPO, "tests")]

import bench  # noqa: E402
import hostemu  # noqa: E402

z = np.load(sys.argv[1])
cfg = sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 20
s, e = z["start_us"], z["end_us"]
dur = e - s
sc = bench.make_scene(cfg)
tx = (sc.vc.width + 7) // 8
b = hostemu.bins(sc)
nf = b[1].ravel() if b is not None else None
order = np.argsort(-dur)[:top]
print("waves", len(dur), "median %.2f us, p99 %.2f, max %.2f" % (np.median(dur), np.percentile(dur, 99), dur.max()))
for w in order:
    ty, tc = divmod(int(w), tx)
    print("wave %6d tile (%3d, %3d) %8.2f us  start %7.2f  bin faces %s" %
          (w, ty, tc, dur[w], s[w], int(nf[w]) if nf is not None and w < len(nf) else "-"))
long = dur > 4 * np.median(dur)
print("waves > 4x median:", int(long.sum()))
if nf is not None:
    print("  of them with mesh faces in their bin:", int((nf[: len(dur)][long] > 0).sum()))
