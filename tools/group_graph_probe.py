"""What one rank does per group at N ranks (bench.py --gpus N, FrameExchange): N renders of
its 1080/N-row uint8 block of TwoSpheresPlane 1080p. Time per frame for the renders launched
eagerly, as one sequential HIP graph, and as one graph whose N renders are independent
branches (fork over side streams inside the capture, so the kernels may run concurrently
and fill the GPU that one 1/N-frame launch leaves partly idle), and as ONE launch of N
frames (rtx_render_frames, gridDim.y = N)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "python-raytracer_amd")]
import torch  # noqa: E402
import bench  # noqa: E402
from rtx.scene import split_rows  # noqa: E402

sc = bench.make_scene(sys.argv[1] if len(sys.argv) > 1 else "tsp1080")
H, W = sc.vc.height, sc.vc.width
REPS = 200


def per_frame_us(fn, n):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(REPS):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / (REPS * n) * 1e6


for n in (1, 2, 4, 8):
    r0, nr = split_rows(H, n, 0)
    out = torch.empty((n, nr, W, 3), dtype=torch.uint8, device="cuda")

    def eager():
        for j in range(n):
            sc.render_device(row0=r0, nrows=nr, out=out[j])
    eager()
    torch.cuda.synchronize()
    g_seq = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g_seq, capture_error_mode="thread_local"):
        eager()
    side = [torch.cuda.Stream() for _ in range(min(n, 4))]
    g_par = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g_par, capture_error_mode="thread_local"):
        main = torch.cuda.current_stream()
        for s in side:
            s.wait_stream(main)
        for j in range(n):
            s = side[j % len(side)]
            with torch.cuda.stream(s):
                sc.render_device(row0=r0, nrows=nr, out=out[j], stream=s)
        for s in side:
            main.wait_stream(s)
    def batched():
        sc.render_frames(out, row0=r0, nrows=nr)
    print("N=%d rows %d: eager %.2f us/frame, graph sequential %.2f, graph %d branches %.2f, one batched launch %.2f"
          % (n, nr, per_frame_us(eager, n), per_frame_us(g_seq.replay, n), len(side), per_frame_us(g_par.replay, n),
             per_frame_us(batched, n)), flush=True)
