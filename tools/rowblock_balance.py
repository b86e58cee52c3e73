"""Load balance of the multi-GPU row partition, measured on one GPU: each rank's row
block (np.array_split(arange(H), N)[r]) rendered alone and timed; prints max/mean per N.
usage: python tools/rowblock_balance.py [--config dof4k] [--reps 3] [--interleave]"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "python-raytracer_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from rtx.scene import split_rows  # noqa: E402,F401


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="dof4k")
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--interleave", action="store_true", help="interleaved 8-row groups (rtx_render_groups)")
    a = p.parse_args()
    sc = bench.make_scene(a.config)
    H = sc.vc.height
    sc.render_device(row0=0, nrows=8)  # compile / warm
    torch.cuda.synchronize()
    out = {"config": a.config, "interleave": a.interleave}
    for n in (2, 4, 8):
        ts = []
        for r in range(n):
            r0, nr = split_rows(H, n, r)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                if a.interleave:
                    sc.render_device(groups=(r, n))
                else:
                    sc.render_device(row0=r0, nrows=nr)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / a.reps)
        mean = sum(ts) / n
        out[str(n)] = {"ms": [round(t, 4) for t in ts], "max_over_mean": round(max(ts) / mean, 3)}
        print(n, out[str(n)], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
