"""Tile dispatch orders from a measured wave timeline (experiment).

  python tools/tile_order.py order WT.npz OUT.bin [--sim]
      longest-measured-first order of the frame's 8x8 tiles (int32 per tile, the file
      RTX_TILE_PERM_FILE reads); --sim prints a list-scheduling estimate of the frame span
      for the row-major and the new order (slots = resident waves per SIMD x SIMDs)
  python tools/tile_order.py check CONFIG OUT.bin
      renders the config with and without the order (GPU): identical framebuffers
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def simulate(dur, order, slots):
    """Greedy list scheduling: waves start in `order`, each on the first free slot."""
    import heapq
    free = [0.0] * slots
    heapq.heapify(free)
    end = 0.0
    for w in order:
        t = heapq.heappop(free)
        t1 = t + float(dur[w])
        end = max(end, t1)
        heapq.heappush(free, t1)
    return end


def main():
    if sys.argv[1] == "order":
        z = np.load(sys.argv[2])
        dur = (z["end_us"] - z["start_us"]).astype(np.float64)
        order = np.argsort(-dur, kind="stable").astype(np.int32)
        order.tofile(sys.argv[3])
        if "--sim" in sys.argv:
            for per_simd in (5, 6, 7):
                slots = 1024 * per_simd
                a = simulate(dur, np.arange(len(dur)), slots)
                b = simulate(dur, order, slots)
                print("slots %d/SIMD: row-major %.2f us, longest first %.2f us" % (per_simd, a, b))
        print("order of %d tiles -> %s" % (len(order), sys.argv[3]))
    elif sys.argv[1] == "check":
        sys.path[:0] = [REPO, os.path.join(REPO, "python-raytracer_amd")]
        import torch
        import bench
        cfg, path = sys.argv[2], sys.argv[3]
        torch.cuda.set_device(0)
        out = []
        for use in (False, True):
            if use:
                os.environ["RTX_TILE_PERM_FILE"] = path
            else:
                os.environ.pop("RTX_TILE_PERM_FILE", None)
            sc = bench.make_scene(cfg)
            fb = torch.empty((sc.vc.height, sc.vc.width, 3), dtype=torch.float32, device="cuda")
            sc.render_device(out=fb)
            torch.cuda.synchronize()
            out.append(fb.clone())
            print(cfg, "perm" if use else "row-major", sc.last_kernel)
        assert torch.equal(out[0], out[1]), "tile order changed the frame"
        print(cfg, "identical frames")


if __name__ == "__main__":
    main()
