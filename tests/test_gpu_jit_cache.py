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


@pytest.mark.parametrize("name,res", [("TwoSpheresPlane", (1920, 1080)), ("MirrorRefraction", (160, 90)),
                                      ("TorusMesh", (96, 96))])
def test_async_compile_renders_generic_then_specialized(name, res, tmp_path, monkeypatch):
    """Option jit_async (the product default; this suite pins 0 in conftest.py): with a cold
    code-object cache the first frames launch the precompiled generic kernel while hiprtc
    compiles on a host thread, and after rtx_jit_wait the specialized kernel renders.
    Every frame -- fp32 and the fused uint8 path -- is bit-identical to the oracle, and the
    first frame does not wait for the compile."""
    import time
    import torch
    from rtx.io import bundled_scene_dict
    cache = tmp_path / "jit"
    cache.mkdir(mode=0o700)
    os.chmod(cache, 0o700)
    monkeypatch.setattr(OPTS, "jit_cache", str(cache))
    monkeypatch.setattr(OPTS, "jit_async", "1")
    d = bundled_scene_dict(name, resolution=res, spp=(1, None))
    d.pop("__base_dir__", None)
    d["lights"][0]["power"] = 0.6180339887  # record values no earlier test compiled
    sc = product_scene_dict(d)
    ref = oracle_render_dict(d)
    t0 = time.perf_counter()
    img = sc.render()
    first_s = time.perf_counter() - t0
    first = sc.last_kernel
    assert first.startswith("k_render_"), first
    assert_parity(img, ref, name + " generic")
    assert first_s < 0.2, first_s  # (a compile takes ~0.3 s)
    want8 = (np.rot90(ref, k=1, axes=(0, 1)) * 255).astype(np.uint8)
    assert np.array_equal(sc.render_rgb8(), want8)
    assert sc.jit_wait() == 0
    img = sc.render()
    assert sc.last_kernel.startswith("rtx_jit_render_"), sc.last_kernel
    assert_parity(img, ref, name + " specialized")
    assert np.array_equal(sc.render_rgb8(), want8)
    assert sc.last_kernel.startswith("rtx_jit_render_") and "_rgb8" in sc.last_kernel, sc.last_kernel
    torch.cuda.synchronize()
