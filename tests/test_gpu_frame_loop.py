"""The multi-GPU frame loops (rtx.distributed.FrameExchange, FramePipeline) with their
DEFAULT device renderers on the MI355X, in a one-rank RCCL (nccl) process group: every
frame they deliver must be the reference's published PNG bytes (provided/main.py:30-34;
renders/TwoSpheresPlane.png, renders/MirrorRefraction.png). The exchange logic between
ranks (slots, split sizes, reordering) is the same code the gloo tests run with 1-4 CPU
ranks (tests/test_multirank.py); one GPU per rank means the box can host one rank."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

from common import product_scene

pytestmark = pytest.mark.gpu

PUB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "published")


def _png(name):
    from PIL import Image
    return np.asarray(Image.open(os.path.join(PUB, name + ".png")).convert("RGB"))


@pytest.fixture(scope="module")
def pg():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    torch.cuda.set_device(0)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield
    dist.destroy_process_group()


@pytest.mark.parametrize("name,interleave", [("TwoSpheresPlane", True), ("MirrorRefraction", False),
                                             ("MirrorRefraction", True)])
def test_frame_exchange_default_renderer_delivers_published_frames(pg, name, interleave):
    sc = product_scene(name)
    want = _png(name)
    from rtx.distributed import FrameExchange
    ex = FrameExchange(sc, 0, 1, interleave=interleave)
    assert ex.render_frames is not None  # the batched launch, not an injected renderer
    got = []
    for _ in range(5):
        got += [(k, f.clone()) for k, f in ex.step()]
    got += [(k, f.clone()) for k, f in ex.flush()]
    assert [k for k, _ in got] == list(range(5))
    for k, f in got:
        assert f.dtype == torch.uint8 and tuple(f.shape) == want.shape
        assert np.array_equal(f.cpu().numpy(), want), (name, k, sc.last_kernel)


@pytest.mark.parametrize("name,interleave", [("TwoSpheresPlane", False), ("MirrorRefraction", True)])
def test_frame_pipeline_default_renderer_delivers_published_frames(pg, name, interleave):
    sc = product_scene(name)
    want = _png(name)
    from rtx.distributed import FramePipeline
    pipe = FramePipeline(sc, 0, 1, interleave=interleave)
    frames = []
    for _ in range(4):
        f = pipe.step()
        frames.append(None if f is None else f.clone())
    frames.append(pipe.flush().clone())
    assert frames[0] is None and len(frames) == 5
    for k, f in enumerate(frames[1:]):
        assert np.array_equal(f.cpu().numpy(), want), (name, k, sc.last_kernel)


def test_frame_exchange_graph_mode_recaptures_after_camera_change(pg):
    """graph=True bakes the camera upload's device pointers into the HIP graphs: a camera
    change re-records them instead of replaying freed tables."""
    from rtx.distributed import FrameExchange
    sc = product_scene("TwoSpheresPlane", (96, 72))

    def render_block(out, rows, k):
        sc.render_device(groups=(0, 1), out=out)
    ex = FrameExchange(sc, 0, 1, render_block=render_block, graph=True)
    got = [(k, f.clone()) for _ in range(2) for k, f in ex.step()]  # frames 0, 1 submitted (0 returned)
    assert ex.graph and ex.graphs[0] is not None
    want_a = sc.render_rgb8()
    sc.vc.set_camera([1.0, 2.5, 6.0], [0.0, 0.5, 0.0], [0.0, 1.0, 0.0], 40)
    got += [(k, f.clone()) for _ in range(2) for k, f in ex.step()]  # frames 2, 3: the new camera
    got += [(k, f.clone()) for k, f in ex.flush()]
    want_b = sc.render_rgb8()
    assert [k for k, _ in got] == [0, 1, 2, 3]
    assert not np.array_equal(want_a, want_b)
    for k, f in got:
        assert np.array_equal(f.cpu().numpy(), want_a if k < 2 else want_b), k


@pytest.mark.parametrize("name,interleave", [("TwoSpheresPlane", None), ("MirrorRefraction", None),
                                             ("MirrorRefraction", True)])
def test_frame_graph_replays_render_and_gather(pg, name, interleave):
    """bench.py's N > 1 value loop (rtx.distributed.FrameGraph): this rank's render, the RCCL
    gather (issued even at world 1: collective_at_one) and -- for interleaved rows -- rank
    0's reorder, recorded once as a HIP graph and replayed per frame (step) or launched
    from C (run, rtx_graph_launch). Every frame is the published PNG; the graph is
    recorded again after a camera change."""
    from rtx.distributed import FrameGraph
    sc = product_scene(name)
    want = _png(name)
    fg = FrameGraph(sc, 0, 1, interleave=interleave, collective_at_one=True)
    # by default one-sample frames (MirrorRefraction) in contiguous blocks, multi-sample ones
    # (the published TwoSpheresPlane: 3 samples) in interleaved groups, reordered in the graph
    assert fg.interleave == (interleave is True or sc.samples_per_pixel > 1)
    for _ in range(3):
        fg.step()
    torch.cuda.synchronize()
    assert fg.graph is not None, sc.last_kernel
    assert np.array_equal(fg.frame().cpu().numpy(), want)
    for n in (4, 11):  # one-frame launches; one 8-frame graph launch + 3 one-frame ones
        fg.g.recv.zero_()
        if fg.out is not None:
            fg.out.zero_()
        fg.run(n)
        torch.cuda.synchronize()
        assert np.array_equal(fg.frame().cpu().numpy(), want), n
    assert fg.graphk is not None and fg.kmax == 8
    first = fg.graph
    # a camera change uploads new tables: the next step records a new graph
    sc.vc.set_camera([1.0, 2.5, 6.0], [0.0, 0.5, 0.0], [0.0, 1.0, 0.0], 40)
    fg.step()
    torch.cuda.synchronize()
    assert fg.graph is not first
    moved = product_scene(name)
    moved.vc.set_camera([1.0, 2.5, 6.0], [0.0, 0.5, 0.0], [0.0, 1.0, 0.0], 40)
    assert np.array_equal(fg.frame().cpu().numpy(), moved.render_rgb8())


def test_frame_graph_falls_back_to_eager_when_recording_fails(pg, monkeypatch):
    """A backend that cannot record its collective into a graph: every rank agrees (an
    all_reduce outside the capture) to issue the frames eagerly, with a warning, and the
    frames are still the published PNG."""
    import contextlib
    from rtx.distributed import FrameGraph

    @contextlib.contextmanager
    def refuses(*a, **k):
        raise RuntimeError("operation not permitted when stream is capturing (simulated)")
        yield
    sc = product_scene("MirrorRefraction")
    want = _png("MirrorRefraction")
    fg = FrameGraph(sc, 0, 1, collective_at_one=True)
    monkeypatch.setattr(torch.cuda, "graph", refuses)
    with pytest.warns(UserWarning, match="eagerly"):
        fg.step()
    assert not fg.graph_on and fg.graph is None
    fg.run(3)
    torch.cuda.synchronize()
    assert np.array_equal(fg.frame().cpu().numpy(), want)
