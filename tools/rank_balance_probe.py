"""Per-rank render time of one batched group (N frames of the rank's rows, one launch) for
every rank of N = 2, 4, 8 on TwoSpheresPlane 1080p: the slowest rank sets the multi-GPU
frame rate. Row blocks (np.array_split) vs interleaved 8-row groups, both batched."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "python-raytracer_amd")]
import torch  # noqa: E402
import bench  # noqa: E402
from rtx.scene import group_rows, split_rows  # noqa: E402

sc = bench.make_scene(sys.argv[1] if len(sys.argv) > 1 else "tsp1080")
H, W = sc.vc.height, sc.vc.width
st = torch.cuda.current_stream()
for n in (1, 2, 4, 8):
    res = {}
    for mode in ("blocks", "groups"):
        us = []
        for k in range(n):
            if mode == "blocks":
                r0, nr = split_rows(H, n, k)
                out = torch.empty((n, nr, W, 3), dtype=torch.uint8, device="cuda")
                fn = lambda: sc.render_frames(out, row0=r0, nrows=nr)  # noqa: E731
                per = n
            else:
                nr = len(group_rows(H, n, k))
                out = torch.empty((n, nr, W, 3), dtype=torch.uint8, device="cuda")
                fn = lambda: sc.render_frames(out, groups=(k, n))  # noqa: E731
                per = n
            fn()
            torch.cuda.synchronize()
            us.append(bench.kernel_ms(fn, 50, st) * 1e3 / per)
        res[mode] = us
    print("N=%d  blocks max %.2f mean %.2f us/frame %s | groups max %.2f mean %.2f" % (
        n, max(res["blocks"]), sum(res["blocks"]) / n, ["%.1f" % u for u in res["blocks"]],
        max(res["groups"]), sum(res["groups"]) / n), flush=True)
