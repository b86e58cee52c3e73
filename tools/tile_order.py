"""Tile dispatch orders from a measured wave timeline (tools/wave_timeline.py --npz).

  python tools/tile_order.py order WT.npz OUT.bin [--sim]
      longest-measured-first order of the frame's 8x8 tiles (int32 per tile); --sim prints
      a list-scheduling estimate of the frame span for the row-major and the new order
      (slots = resident waves per SIMD x SIMDs). The library builds the same order itself
      (rtx_api.hip tile_schedule); round 4 first measured it with orders from this tool
      (profiles/r04/tile_order/).
"""
import sys

import numpy as np


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


if __name__ == "__main__":
    main()
