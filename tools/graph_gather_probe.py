"""Host issue cost of one sharded frame (render + gather to rank 0) per step, in a one-rank
RCCL group on the box (rtx.distributed.FrameGraph with the gather issued at world 1):
eager Python calls, one HIP graph replay per frame (step), and the frames launched from C
(run: rtx_graph_launch). Also checks that every variant delivers the eager frame's bytes.
usage: python tools/graph_gather_probe.py [config] [steps]"""
import json
import os
import socket
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "python-raytracer_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "tsp1080"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    torch.cuda.set_device(0)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s.getsockname()[1]))
    s.close()
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from rtx.distributed import FrameGraph
    sc = bench.make_scene(cfg)
    out = {"config": cfg, "steps": steps}
    for mode in ("eager", "graph"):
        fg = FrameGraph(sc, 0, 1, graph=(mode == "graph"), collective_at_one=True)
        for _ in range(50):
            fg.step()
        torch.cuda.synchronize()
        if mode == "eager":
            ref = fg.frame().clone()
        fg.g.recv.zero_()
        t0 = time.perf_counter()
        for _ in range(steps):
            fg.step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        r = {"host_us_per_frame": round((t1 - t0) / steps * 1e6, 3),
             "wall_us_per_frame": round((t2 - t0) / steps * 1e6, 3),
             "frame_equal": bool(torch.equal(fg.frame(), ref)), "graph": fg.graph is not None}
        fg.g.recv.zero_()
        t0 = time.perf_counter()
        fg.run(steps)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        r["run"] = {"host_us_per_frame": round((t1 - t0) / steps * 1e6, 3),
                    "wall_us_per_frame": round((t2 - t0) / steps * 1e6, 3),
                    "frame_equal": bool(torch.equal(fg.frame(), ref))}
        out[mode] = r
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(200):
        sc.render_device(out=fg.g.block, stream=st)
    e1.record(st)
    torch.cuda.synchronize()
    out["render_rgb8_us"] = round(e0.elapsed_time(e1) / 200 * 1e3, 3)
    out["kernel"] = sc.last_kernel
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
