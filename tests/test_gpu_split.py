"""The hierarchy/texture scenes rendered by the three split passes on the MI355X
(csrc/rtx_split.h, RTX_SPLIT=1): chains of closest hits -> shade-point records, shadow
rays per record -> occlusion masks, lighting + unwinding + the ordered mean. Bit-identical
to the oracle (with its ray tallies) and to the one-kernel form."""
import numpy as np
import pytest
import torch

from common import assert_parity, oracle_render, oracle_render_dict, product_scene, product_scene_dict

pytestmark = pytest.mark.gpu

CASES = [
    ("NovelScene1", (256, 128), {"AA": {"jitter": False, "samples": 1}}),
    ("NovelScene1", (96, 48), {"AA": {"jitter": False, "samples": 4}}),
    ("NovelScene2", (128, 64), {"AA": {"jitter": False, "samples": 1}}),
    ("NovelScene2", (48, 24), {"AA": {"jitter": False, "samples": 2}}),
]


@pytest.fixture
def split(monkeypatch):
    monkeypatch.setenv("RTX_SPLIT", "1")


@pytest.mark.parametrize("name,res,edits", CASES)
def test_split_matches_oracle(name, res, edits, split):
    sc = product_scene(name, res, **edits)
    img = sc.render()
    assert sc.last_kernel.startswith("k_split_"), sc.last_kernel
    assert_parity(img, oracle_render(name, res, **edits), name)


@pytest.mark.parametrize("seed", range(24))
def test_split_random_hierarchy_scenes(seed, split):
    from scenegen import random_hier_scene
    d = random_hier_scene(seed, res=(64, 48), mesh=(seed % 4 == 0))
    sc = product_scene_dict(d)
    assert_parity(sc.render(), oracle_render_dict(d), "hier seed %d" % seed)
    assert sc.last_kernel.startswith("k_split_"), sc.last_kernel


def test_split_tallies_match_oracle(split):
    name, res, edits = "NovelScene2", (64, 32), {"AA": {"jitter": False, "samples": 1}}
    sc = product_scene(name, res, **edits)
    fb = torch.empty((res[1], res[0], 3), dtype=torch.float32, device="cuda")
    cnt = torch.zeros(16, dtype=torch.int64, device="cuda")
    sc.render_device(out=fb, counters=cnt)
    c = cnt.cpu().numpy()
    ref, tl = oracle_render(name, res, tallies=True, **edits)
    assert list(c[:10]) == tl[:10]
    assert c[10] == tl[11] and c[11] == tl[12]


def test_split_small_chunks_and_row_groups(split, monkeypatch):
    """Many chunks (RTX_SPLIT_RECORDS small) and interleaved 8-row groups: the same frame."""
    monkeypatch.setenv("RTX_SPLIT_RECORDS", "4000")
    name, res, edits = "NovelScene1", (80, 40), {"AA": {"jitter": False, "samples": 2}}
    sc = product_scene(name, res, **edits)
    ref = oracle_render(name, res, **edits)
    assert_parity(sc.render(), ref, name)
    full = torch.empty((res[1], res[0], 3), dtype=torch.float32, device="cuda")
    sc.render_device(out=full)
    from rtx.scene import group_rows
    for k in range(3):
        rows = group_rows(res[1], 3, k)
        part = torch.empty((len(rows), res[0], 3), dtype=torch.float32, device="cuda")
        sc.render_device(out=part, groups=(k, 3))
        assert torch.equal(part, full[torch.as_tensor(rows, device="cuda")])


def test_split_equals_one_kernel_full_novel_scene1(monkeypatch):
    """NovelScene1's full config (2048x1024 AA32, Philox jitter): the split passes and the
    one-kernel form give the same bytes."""
    sc = product_scene("NovelScene1")
    H, W = sc.vc.height, sc.vc.width
    a = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    b = torch.empty_like(a)
    monkeypatch.setenv("RTX_SPLIT", "0")
    sc.render_device(out=a)
    one = sc.last_kernel
    monkeypatch.setenv("RTX_SPLIT", "1")
    sc.render_device(out=b)
    torch.cuda.synchronize()
    assert one.startswith("k_render_ext") and sc.last_kernel.startswith("k_split_"), (one, sc.last_kernel)
    assert torch.equal(a, b), float((a != b).float().mean())


@pytest.mark.parametrize("seed", range(2))
def test_split_many_roots_bins_and_grids(seed, split, monkeypatch):
    """40 hierarchy roots and 20 flat spheres (beyond the 32 root bits and 16 sphere bits
    of the bins and shadow-grid cells), lens camera with Philox jitter: the split passes
    with bins and grids == without == the oracle."""
    from scenegen import many_roots_scene
    from oracle import philox as PH
    d = many_roots_scene(seed, res=(96, 64))
    sc = product_scene_dict(d)
    a = sc.render_device().clone()
    assert sc.last_kernel.startswith("k_split_"), sc.last_kernel
    monkeypatch.setenv("RTX_BINS", "0")
    monkeypatch.setenv("RTX_DSGRID", "0")
    b = product_scene_dict(d).render_device().clone()
    assert torch.equal(a, b)
    img = np.ascontiguousarray(np.transpose(a.cpu().numpy()[::-1], (1, 0, 2))).astype(np.float64)
    noise = PH.jitter_noise(sc.seed, 0, 96, 64, sc.vc.dof_samples, sc.samples)
    assert_parity(img, oracle_render_dict(d, noise=noise), "many roots seed %d" % seed)
