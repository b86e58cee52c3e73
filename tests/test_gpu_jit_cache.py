"""The scene-specialized kernels of one-sample flat scenes carry the scene's records as
literals (csrc/rtx_api.hip jit_baked_records), so each new set of record values compiles
its own kernel. Those modules and their code objects must not accumulate: a module no
scene holds is unloaded beyond $RTX_JIT_IDLE_BAKED idle ones, and the disk cache keeps at
most $RTX_JIT_DISK_BAKED baked code objects. Each re-created scene still renders
bit-identical to the oracle."""
import os

import numpy as np
import pytest

from common import assert_parity, oracle_render_dict, product_scene_dict
from common import OPTS

pytestmark = pytest.mark.gpu


def test_baked_kernels_are_bounded(tmp_path, monkeypatch):
    import torch
    from rtx import _native as N
    from rtx.io import bundled_scene_dict
    assert torch.cuda.is_available()
    cache = tmp_path / "jit"
    cache.mkdir(mode=0o700)
    os.chmod(cache, 0o700)
    monkeypatch.setattr(OPTS, "jit_cache", str(cache))
    monkeypatch.setattr(OPTS, "jit_idle_baked", "1")
    monkeypatch.setattr(OPTS, "jit_disk_baked", "2")
    lib = N.load()
    base = lib.rtx_jit_modules()
    d = bundled_scene_dict("TwoSpheresPlane", resolution=(32, 24), spp=(1, None))  # one sample: baked records
    d.pop("__base_dir__", None)
    counts = []
    for k in range(5):
        d["materials"][0]["diffuse"] = [0.1 + 0.15 * k, 0.5, 0.25]  # new record values: a new baked kernel
        sc = product_scene_dict(d)
        img = sc.render()
        assert sc.last_kernel.startswith("rtx_jit_render_"), sc.last_kernel
        assert_parity(img, oracle_render_dict(d), "baked k=%d" % k)
        counts.append(lib.rtx_jit_modules())
        sc.invalidate()  # rtx_scene_destroy: the scene lets go of its kernel
    assert max(counts) <= base + 2, (base, counts)  # the live one + one idle
    assert lib.rtx_jit_modules() <= base + 1, (base, lib.rtx_jit_modules())
    baked = [f for f in os.listdir(cache) if f.startswith("rtx_b_") and f.endswith(".co")]
    assert 1 <= len(baked) <= 2, sorted(os.listdir(cache))
    # a scene whose module was unloaded loads (or compiles) it again and renders the same
    d["materials"][0]["diffuse"] = [0.1, 0.5, 0.25]
    sc = product_scene_dict(d)
    img = sc.render()
    assert np.array_equal(img, oracle_render_dict(d))
