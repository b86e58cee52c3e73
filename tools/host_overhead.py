"""Host cost of one render call (Python -> ctypes -> rtx_render -> launch) on the GPU box:
wall time per call for launches too short to hide it (a few rows), next to the full frame."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "python-raytracer_amd")]
import torch  # noqa: E402
import bench  # noqa: E402

sc = bench.make_scene("tsp1080")
H, W = sc.vc.height, sc.vc.width
fb = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
u8 = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda")
for label, kw in (("full fp32", dict(out=fb)), ("8 rows fp32", dict(row0=0, nrows=8, out=fb[:8])),
                  ("135 rows uint8", dict(row0=0, nrows=135, out=u8[:135])),
                  ("8 rows uint8", dict(row0=0, nrows=8, out=u8[:8]))):
    for _ in range(20):
        sc.render_device(**kw)
    torch.cuda.synchronize()
    n = 2000
    t0 = time.perf_counter()
    for _ in range(n):
        sc.render_device(**kw)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("%-16s issue %.2f us/call, wall %.2f us/call (kernel %s)" % (label, (t1 - t0) / n * 1e6, (t2 - t0) / n * 1e6,
                                                                       sc.last_kernel), flush=True)
