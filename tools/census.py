"""Ray/test census of a bench config on cuda:0: device counters per primary sample (the
counting kernel counts per active lane, so triangle tests are the wave-level work)."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "python-raytracer_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--config", default="tm1080")
a = p.parse_args()
torch.cuda.set_device(0)
sc = bench.make_scene(a.config)
W, H = sc.vc.width, sc.vc.height
fb = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
cnt = torch.zeros(16, dtype=torch.int64, device="cuda")
sc.render_device(out=fb, counters=cnt)
c = cnt.cpu().numpy()
n = W * H * sc.samples_per_pixel
print("%s casts/sample %.4f shadow/sample %.4f shade/sample %.4f tri_tests/sample %.3f" % (
    a.config, c[:10].sum() / n, c[10] / n, c[11] / n, c[12] / n))
