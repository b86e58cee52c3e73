"""CLI mirror of provided/glue.py:11-27: stitch numpy strips (k.npy, sorted by k) along
the column axis, rot90, truncating uint8 conversion, PNG."""
import argparse
import os

import numpy as np


def glue(directory):
    files = os.listdir(directory)
    files.sort(key=lambda x: int(x.split(".")[0]))
    arrays = [np.load(os.path.join(directory, f)) for f in files]
    image = np.concatenate(arrays, axis=0)
    image = np.rot90(image, k=1, axes=(0, 1))
    return (image * 255).astype(np.uint8)


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--outfile", type=str, default="out.png")
    p.add_argument("--dir", type=str)
    a = p.parse_args(argv)
    from PIL import Image
    Image.fromarray(glue(a.dir)).save(a.outfile)


if __name__ == "__main__":
    main()
