"""Minimal render loop for rocprofv3 runs: N + 1 frames of a bench config on cuda:0, every
one with the product's (scene-specialized) kernels: compiles wait inside the first render
(RTX_JIT_ASYNC=0), so no generic-kernel frame mixes into the counters."""
import argparse
import os
import sys

os.environ.setdefault("RTX_JIT_ASYNC", "0")  # (read when librtx.so loads)

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "python-raytracer_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--config", default="tsp1080")
p.add_argument("--iters", type=int, default=10)
a = p.parse_args()
torch.cuda.set_device(0)
sc = bench.make_scene(a.config)
fb = torch.empty((sc.vc.height, sc.vc.width, 3), dtype=torch.float32, device="cuda")
sc.render_device(out=fb)
assert sc.jit_wait() == 0  # (the specialized kernels: the profiled frames are the product's)
for _ in range(a.iters):
    sc.render_device(out=fb)
torch.cuda.synchronize()
print("done", a.config, a.iters)
