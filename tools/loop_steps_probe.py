"""Fixed cost of bench.py's N > 1 value loop against its length, in a one-rank RCCL group:
the time per frame of `steps` frames issued by FrameGraph.run (graph launches from C),
bracketed as bench.timed does (barrier + synchronize on both sides), for several `steps`;
beside it the same for a graph of the render alone (no collective) and for eager frames.
usage: python tools/loop_steps_probe.py [config]"""
import json
import os
import socket
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "python-raytracer_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "tsp1080"
    torch.cuda.set_device(0)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s.getsockname()[1]))
    s.close()
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from rtx.distributed import FrameGraph
    sc = bench.make_scene(cfg)
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream()
    out = {"config": cfg}
    variants = {"graph+gather": dict(collective_at_one=True), "graph render only": dict(collective_at_one=False),
                "eager+gather": dict(collective_at_one=True, graph=False)}
    for name, kw in variants.items():
        fg = FrameGraph(sc, 0, 1, device=dev, **kw)
        for _ in range(5):
            fg.step()
        fg.run(16, st)
        torch.cuda.synchronize()
        bench.clock_warmup(lambda: fg.run(8, st), 0.2, torch.cuda.synchronize)
        rows = {}
        for steps in (8, 20, 64, 200, 2000):
            t = bench.timed(lambda: fg.run(steps, st), 1, True)
            rows[steps] = round(t / steps * 1e6, 3)
        out[name] = rows
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
