"""The hierarchy/texture scenes rendered by the three split passes on the MI355X
(csrc/rtx_split.h, RTX_SPLIT=1): chains of closest hits -> shade-point records, shadow
rays per record -> occlusion masks, lighting + unwinding + the ordered mean. Bit-identical
to the oracle (with its ray tallies) and to the one-kernel form. The trace and shadow passes
run specialized on the scene's CSG trees (option jit_csg, rtx_trace.h namespace csg) where
the scene qualifies, the precompiled passes otherwise: both are the split path."""
import numpy as np
import pytest
import torch

from common import assert_parity, oracle_render, oracle_render_dict, product_scene, product_scene_dict
from common import OPTS

pytestmark = pytest.mark.gpu

CASES = [
    ("NovelScene1", (256, 128), {"AA": {"jitter": False, "samples": 1}}),
    ("NovelScene1", (96, 48), {"AA": {"jitter": False, "samples": 4}}),
    ("NovelScene2", (128, 64), {"AA": {"jitter": False, "samples": 1}}),
    ("NovelScene2", (48, 24), {"AA": {"jitter": False, "samples": 2}}),
]


SPLIT = ("k_split_", "rtx_jit_split_")  # the split passes: precompiled, or specialized on the trees


@pytest.fixture
def split(monkeypatch):
    monkeypatch.setattr(OPTS, "split", "1")


@pytest.mark.parametrize("name,res,edits", CASES)
def test_split_matches_oracle(name, res, edits, split):
    sc = product_scene(name, res, **edits)
    img = sc.render()
    assert sc.last_kernel.startswith(SPLIT), sc.last_kernel
    assert_parity(img, oracle_render(name, res, **edits), name)


@pytest.mark.parametrize("seed", range(24))
def test_split_random_hierarchy_scenes(seed, split, monkeypatch):
    """Random hierarchy scenes (every fourth with a mesh): every third seed with the passes
    specialized on its trees (a compile each), the others with the precompiled passes."""
    from scenegen import random_hier_scene
    monkeypatch.setattr(OPTS, "jit_csg", "1" if seed % 3 == 0 else "0")
    d = random_hier_scene(seed, res=(64, 48), mesh=(seed % 4 == 0))
    sc = product_scene_dict(d)
    assert_parity(sc.render(), oracle_render_dict(d), "hier seed %d" % seed)
    assert sc.last_kernel.startswith("rtx_jit_split_" if seed % 3 == 0 else "k_split_"), sc.last_kernel


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
    """Many chunks (RTX_SPLIT_BYTES small) and interleaved 8-row groups: the same frame."""
    monkeypatch.setattr(OPTS, "split_bytes", str(4000 * 40))
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
    monkeypatch.setattr(OPTS, "split", "0")
    sc.render_device(out=a)
    one = sc.last_kernel
    monkeypatch.setattr(OPTS, "split", "1")
    sc.render_device(out=b)
    torch.cuda.synchronize()
    assert one.startswith("k_render_ext") and sc.last_kernel.startswith(SPLIT), (one, sc.last_kernel)
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
    assert sc.last_kernel.startswith(SPLIT), sc.last_kernel
    monkeypatch.setattr(OPTS, "bins", "0")
    monkeypatch.setattr(OPTS, "dsgrid", "0")
    b = product_scene_dict(d).render_device().clone()
    assert torch.equal(a, b)
    img = np.ascontiguousarray(np.transpose(a.cpu().numpy()[::-1], (1, 0, 2))).astype(np.float64)
    noise = PH.jitter_noise(sc.seed, 0, 96, 64, sc.vc.dof_samples, sc.samples)
    assert_parity(img, oracle_render_dict(d, noise=noise), "many roots seed %d" % seed)


@pytest.mark.parametrize("ratio,budget", [("0", None), ("0.02", str(3000 * 40)), ("0.3", None)])
def test_split_pool_overflow_redo(ratio, budget, split, monkeypatch):
    """A deeper-record pool smaller than the chains need: hits that find it full mark their
    blocks, and the one-kernel form renders those again after pass C (render_body_spp with
    L.redo) -- the frame is the oracle's, bit for bit, on frames with many mirrors."""
    from scenegen import random_hier_scene
    monkeypatch.setattr(OPTS, "split_ratio", ratio)
    if budget:
        monkeypatch.setattr(OPTS, "split_bytes", budget)
    for seed in (3, 5):
        d = random_hier_scene(seed, res=(40, 30))
        d["materials"] = [dict(m, type="mirror", tint=m.get("tint", 0.3)) if i % 2 == 0 else m
                          for i, m in enumerate(d["materials"])]
        sc = product_scene_dict(d)
        img = sc.render()
        assert sc.last_kernel.startswith(SPLIT), sc.last_kernel
        assert_parity(img, oracle_render_dict(d), "pool overflow %s seed %d" % (ratio, seed))


def test_split_pool_learns_and_frames_repeat(split):
    """The learned pool (no fixed ratio): the first frame may redo blocks, later frames size
    the pool from the first's counters; every frame is the same bytes."""
    name, res, edits = "NovelScene1", (160, 80), {"AA": {"jitter": False, "samples": 2}}
    sc = product_scene(name, res, **edits)
    frames = []
    for _ in range(4):
        frames.append(sc.render_device().clone())
        torch.cuda.synchronize()
    for f in frames[1:]:
        assert torch.equal(f, frames[0])
    img = np.ascontiguousarray(np.transpose(frames[0].cpu().numpy()[::-1], (1, 0, 2))).astype(np.float64)
    assert_parity(img, oracle_render(name, res, **edits), name)


def test_split_renders_on_two_streams(split):
    """Renders of one hierarchy scene on two streams share its record buffers: the library
    orders them (each waits for the other's last split render), so both frames are right."""
    name, res, edits = "NovelScene2", (96, 48), {"AA": {"jitter": False, "samples": 2}}
    sc = product_scene(name, res, **edits)
    ref = sc.render_device().clone()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = []
    for k in range(6):
        st = s1 if k % 2 == 0 else s2
        o = torch.empty_like(ref)
        sc.render_device(out=o, stream=st)
        outs.append(o)
    torch.cuda.synchronize()
    for o in outs:
        assert torch.equal(o, ref)


@pytest.mark.filterwarnings("ignore:The CUDA Graph is empty")  # (the refused capture's graph)
def test_split_capture_needs_a_first_render(split):
    """Graph capture of a hierarchy scene whose record buffer does not exist yet is refused
    (the library does not allocate inside a capture); after one eager render the capture
    works and its replays give the eager frame."""
    from rtx._native import RtxError
    name, res, edits = "NovelScene1", (64, 32), {"AA": {"jitter": False, "samples": 2}}
    sc = product_scene(name, res, **edits)
    sc._set_camera(0, 1)
    out = torch.empty((res[1], res[0], 3), dtype=torch.float32, device="cuda")
    st = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with pytest.raises(RtxError):
        with torch.cuda.graph(g, stream=st):
            sc.render_device(out=out, stream=st)
    ref = sc.render_device().clone()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        sc.render_device(out=out, stream=st)
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


@pytest.mark.parametrize("case", ["ns1", "ns1_full", "ns2", "random", "many_roots"])
def test_split_csg_specialized_equals_precompiled(case, split, monkeypatch):
    """The trace and shadow passes specialized on the scene's CSG trees (node fields and
    matrices as literals, the traversals unrolled: rtx_api.hip jit_csg_tables) give the
    precompiled passes' bytes: NovelScene1/2 (NovelScene1 also at its full 2048x1024 AA32
    Philox config), random hierarchy scenes with and without a mesh, 40 roots."""
    from scenegen import many_roots_scene, random_hier_scene
    if case == "random":
        ds = [random_hier_scene(seed, res=(64, 48), mesh=(seed % 2 == 0)) for seed in (1, 2, 9, 12)]
        make = [lambda d=d: product_scene_dict(d) for d in ds]
    elif case == "many_roots":
        make = [lambda: product_scene_dict(many_roots_scene(1, res=(96, 64)))]
    elif case == "ns1_full":
        make = [lambda: product_scene("NovelScene1")]
    else:
        name = "NovelScene1" if case == "ns1" else "NovelScene2"
        make = [lambda: product_scene(name, (128, 64), AA={"jitter": True, "samples": 4})]
    for mk in make:
        frames, kernels = [], []
        for on in ("1", "0"):
            monkeypatch.setattr(OPTS, "jit_csg", on)
            sc = mk()
            frames.append(sc.render_device().clone())
            kernels.append(sc.last_kernel)
        torch.cuda.synchronize()
        assert kernels[0].startswith("rtx_jit_split_") and kernels[1].startswith("k_split_"), kernels
        assert torch.equal(frames[0], frames[1]), float((frames[0] != frames[1]).float().mean())
