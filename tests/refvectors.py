"""Loader for the golden vectors the reference's own code produced
(tests/golden/refvectors/*.npz, written by tests/golden/make_refvectors.py in the build
container; the reference itself never travels)."""
import glob
import hashlib
import json
import os

import numpy as np

DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "refvectors")


def names(kind):
    return sorted(os.path.basename(p)[len(kind) + 1:-4] for p in glob.glob(os.path.join(DIR, kind + "_*.npz")))


def load(kind, name):
    with np.load(os.path.join(DIR, "%s_%s.npz" % (kind, name)), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def scene(fx):
    return json.loads(str(fx["scene_json"]))


def noise(fx):
    """The reference's np.random.rand() stream of a jittered render case (None if not
    jittered): regenerated from the seed and checked against the recorded digest."""
    seed = int(fx["noise_seed"])
    if seed < 0:
        return None
    s = np.random.RandomState(seed).rand(int(fx["noise_count"]))
    assert hashlib.sha256(s.tobytes()).hexdigest() == str(fx["noise_digest"]), "noise stream digest"
    return s


def hits(fx, ti, k, i):
    """Every hit obj k's intersect returned for ray i at time index ti:
    (t, normal, position, material) arrays."""
    off = fx["t%d_obj%d_off" % (ti, k)]
    a, b = int(off[i]), int(off[i + 1])
    return tuple(fx["t%d_obj%d_%s" % (ti, k, f)][a:b] for f in ("t", "normal", "position", "mat"))
