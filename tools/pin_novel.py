#!/usr/bin/env python3
"""Pins the oracle's hierarchy + texture restatement against the reference's published
NovelScene renders (TEST INFRASTRUCTURE: runs the oracle, CPU only).

The published renders used an unseeded np.random jitter, so the comparison is
statistical: the oracle renders column strips (np.array_split(arange(W), tasks)[k]) with
seeded noise and each strip is compared with the same columns of renders/<name>.png.

    python tools/pin_novel.py NovelScene1 64 all        # every strip (8 processes)
    python tools/pin_novel.py NovelScene2 64 16,32,40
"""
import sys
import time
from multiprocessing import Pool

import numpy as np
from PIL import Image

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402

REPO = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))


def run(args):
    name, tasks, k = args
    d, base = O.load_bundle(name)
    sc = O.OracleScene(d, base)
    W, H = sc.width, sc.height
    b, e = divmod(W, tasks)
    ncol = b + (1 if k < e else 0)
    c0 = k * b + min(k, e)
    noise = np.random.RandomState(k).rand(ncol * H * sc.spp_rays * 3)
    return k, c0, O.to_png_array(sc.render(k, tasks, noise=noise))


def main():
    name, tasks = sys.argv[1], int(sys.argv[2])
    ks = list(range(tasks)) if sys.argv[3] == "all" else [int(x) for x in sys.argv[3].split(",")]
    ref = np.asarray(Image.open("%s/tests/golden/published/%s.png" % (REPO, name)).convert("RGB"))
    t = time.time()
    tot_abs = tot_sum = tot_exact = tot_n = 0.0
    with Pool(8) as pool:
        for k, c0, png in pool.imap(run, [(name, tasks, k) for k in ks]):
            d = png.astype(int) - ref[:, c0:c0 + png.shape[1]].astype(int)
            ex = (np.abs(d).max(axis=2) == 0)
            tot_abs += np.abs(d).sum(); tot_sum += d.sum(); tot_exact += ex.sum(); tot_n += ex.size
            print("strip %3d cols %4d..%4d  mean|d| %.4f  bias %+.4f  identical %.4f  max %d"
                  % (k, c0, c0 + png.shape[1] - 1, np.abs(d).mean(), d.mean(), ex.mean(), np.abs(d).max()), flush=True)
    print("%s: %d strips, mean|d| %.4f LSB, bias %+.4f, identical pixels %.4f  (%.0f s)"
          % (name, len(ks), tot_abs / (3 * tot_n), tot_sum / (3 * tot_n), tot_exact / tot_n, time.time() - t))


if __name__ == "__main__":
    main()
