"""The reference-side binding on the MI355X: scenes built by the reference's own parser
(reference-shaped objects, tests/refobjects.py) rendered through rtx.Scene.from_reference
— the stub INTEGRATION.md §B puts into provided/scene.py's Scene.render — must be
bit-identical to the oracle for the same JSON."""
import numpy as np
import pytest
import torch

import refobjects as R
import rtx
from common import assert_parity, oracle_render

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _device():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    torch.cuda.set_device(0)


@pytest.mark.parametrize("name", R.names())
def test_reference_scene_renders_like_the_oracle(name):
    ref, res = R.load(name)
    edits = {}
    noise = None
    if ref.jitter:  # the reference's RNG is unseeded: replay one seeded stream on both sides
        W, H = res
        noise = np.random.RandomState(7).rand(W * H * ref.vc.dof_samples * ref.samples * 3)
    bound = rtx.Scene.from_reference(ref)
    bound.jitter_noise = noise
    img = bound.render()
    assert bound.last_kernel, "no kernel launched"
    s = assert_parity(img, oracle_render(name, res, noise=noise, **edits), name)
    assert s["frac_diff"] == 0.0


def test_reference_scene_strips_like_main_py():
    """main.py --subimage k --tasks N through the binding (provided/main.py:26-28)."""
    ref, res = R.load("MirrorRefraction")
    bound = rtx.Scene.from_reference(ref)
    for k in range(3):
        assert_parity(bound.render(k, 3), oracle_render("MirrorRefraction", res, subimage=k, tasks=3))
