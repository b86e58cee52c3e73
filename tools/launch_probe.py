"""Per-launch fixed cost of the one-sample kernels: one full frame per launch against N full
frames in one batched launch (rtx_render_frames, gridDim.y = N), uint8 output both ways,
timed with HIP events over 200 repetitions. usage: python tools/launch_probe.py [config ...]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "python-raytracer_amd")]
import torch  # noqa: E402
import bench  # noqa: E402

REPS = 200


def per_frame_us(fn, n):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(REPS):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / (REPS * n)


for cfg in sys.argv[1:] or ["tsp1080"]:
    sc = bench.make_scene(cfg)
    H, W = sc.vc.height, sc.vc.width
    one = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda")
    line = ["%s single %.2f us" % (cfg, per_frame_us(lambda: sc.render_device(out=one), 1))]
    for n in (2, 4, 8):
        out = torch.empty((n, H, W, 3), dtype=torch.uint8, device="cuda")
        line.append("x%d %.2f" % (n, per_frame_us(lambda: sc.render_frames(out), n)))
    print(", ".join(line), "(us per frame; kernel %s)" % sc.last_kernel, flush=True)
