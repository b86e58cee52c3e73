"""Shared helpers for the parity tests."""
import numpy as np

from oracle import oracle as O


def oracle_render(name, res=None, subimage=0, tasks=1, noise=None, tallies=False, **edits):
    d, base = O.load_bundle(name)
    if res is not None:
        d["resolution"] = list(res)
    for k, v in edits.items():
        if k == "flat_shaded":
            for g in d["objects"]:
                if g["type"] == "mesh":
                    g["flat_shaded"] = v
        else:
            d[k] = v
    return O.OracleScene(d, base).render(subimage, tasks, noise=noise, tallies=tallies)


def product_scene(name, res=None, **edits):
    import rtx
    from rtx.io import bundled_scene_dict
    d = bundled_scene_dict(name, resolution=res)
    for k, v in edits.items():
        if k == "flat_shaded":
            for g in d["objects"]:
                if g["type"] == "mesh":
                    g["flat_shaded"] = v
        else:
            d[k] = v
    return rtx.load_scene(d, verbose=False)


def compare(img, ref):
    """Parity statistics of a rendered float image against the oracle's."""
    assert img.shape == ref.shape, (img.shape, ref.shape)
    d = np.abs(img - ref).max(axis=2)
    png = np.abs(O.to_png_array(img).astype(int) - O.to_png_array(ref).astype(int)).max(axis=2)
    return dict(frac_diff=float((d > 0).mean()), max_abs=float(d.max()), mean_abs=float(d.mean()),
                png_frac_diff=float((png > 0).mean()), png_max=int(png.max()))


# Parity bar (north_star: "within a stated fp32 tolerance of the reference"): the fp32
# framebuffer must be bit-identical to the oracle's -- every deterministic case asserts
# frac_diff == 0. No tolerance is left: `x ** hardness` (rtx_trace.h spec_pow) is held to
# libm pow bit for bit by tests/test_pow.py.
def assert_parity(img, ref, what=""):
    s = compare(img, ref)
    assert s["frac_diff"] == 0.0, "%s parity (exact): %s" % (what, s)
    return s


def oracle_render_dict(data, subimage=0, tasks=1, noise=None, tallies=False):
    import os
    base = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets")
    return O.OracleScene(data, base).render(subimage, tasks, noise=noise, tallies=tallies)


def product_scene_dict(data):
    import copy
    import os
    import rtx
    d = copy.deepcopy(data)
    d["__base_dir__"] = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets")
    return rtx.load_scene(d, verbose=False)


class _Options:
    """The library options (rtx.set_option / rtx.get_option) as attributes, so a test can
    set one for its own duration with monkeypatch.setattr(OPTS, "bins", "0"): the old value
    is read back and restored at teardown. The host emulation (tests/hostemu.py) includes
    the library's source and has its own copy of the options: it gets the same value when
    the test module has imported it."""

    def __getattr__(self, name):
        import rtx
        return rtx.get_option(name)

    def __setattr__(self, name, value):
        import sys
        import rtx
        rtx.set_option(name, value)
        he = sys.modules.get("hostemu")  # (imported by the host-emulation tests only)
        if he is not None:
            he.set_option(name, value)


OPTS = _Options()
