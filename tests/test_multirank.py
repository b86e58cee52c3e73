"""World-size-2 gloo tests of the multi-rank frame path (row blocks + gather) on CPU,
with the tests-only host build of the device source standing in for each rank's GPU."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, name, res, out_q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), os.path.join(os.path.dirname(here), "python-raytracer_amd"), here):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import hostemu
    from common import product_scene
    from rtx.distributed import render_frame
    sc = product_scene(name, res)

    # each rank renders only its own rows (host build of the device code standing in
    # for this rank's GPU), in the layout rtx_render / rtx_render_groups write
    def rows(row0, nrows):
        return torch.from_numpy(hostemu.render_rows(sc, np.arange(row0, row0 + nrows), threads=2))

    def group(rws):  # interleaved 8-row groups: the given image rows
        return torch.from_numpy(hostemu.render_rows(sc, rws, threads=2))

    for dtype in (torch.float32, torch.uint8):
        frame = render_frame(sc, rank, world, render_rows=rows, dtype=dtype)
        if rank == 0:
            out_q.put((str(dtype), frame.numpy()))
        frame = render_frame(sc, rank, world, render_rows=group, dtype=dtype, interleave=True)
        if rank == 0:
            out_q.put(("interleaved " + str(dtype), frame.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def _pipeline_worker(rank, world, port, name, res, nframes, interleave, out_q):
    """bench.py's multi-GPU frame loop (rtx.distributed.FramePipeline: render this rank's
    interleaved groups, uint8, async gather, previous frame finished while the next one
    renders) with the host emulation as each rank's renderer."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), os.path.join(os.path.dirname(here), "python-raytracer_amd"), here):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import hostemu
    from common import product_scene
    from rtx.distributed import FramePipeline, to_rgb8
    sc = product_scene(name, res)

    cache, count = {}, [0]

    def render_block(out, rows):  # the fused uint8 render, emulated: fp32 rows, then main.py's conversion
        if "rows" not in cache:
            cache["rows"] = to_rgb8(torch.from_numpy(hostemu.render_rows(sc, rows, threads=2)))
        out.copy_(cache["rows"] + count[0])  # frame k's rows + k (uint8 wraps): frames differ
        count[0] += 1
    pipe = FramePipeline(sc, rank, world, device=torch.device("cpu"), render_block=render_block, interleave=interleave)

    def keep(f):  # a returned frame may be a view of a reused buffer: copy it at once
        return None if f is None else f.clone()
    frames = [keep(pipe.step()) for _ in range(nframes)] + [keep(pipe.flush())]
    if rank == 0:
        assert frames[0] is None and all(f is not None for f in frames[1:])
        out_q.put([f.numpy() for f in frames[1:]])
    else:
        assert all(f is None for f in frames)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,res,interleave", [(1, (40, 23), True), (2, (40, 23), True), (3, (33, 26), True),
                                                  (2, (40, 24), False), (3, (20, 13), False)])
def test_frame_pipeline_gathers_every_frame(world, res, interleave):
    from common import oracle_render
    from oracle import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipeline_worker, args=(r, world, port, "MirrorRefraction", res, 3, interleave, q))
             for r in range(world)]
    for p in procs:
        p.start()
    frames = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = O.to_png_array(oracle_render("MirrorRefraction", res))
    assert len(frames) == 3
    for k, f in enumerate(frames):
        assert np.array_equal(f, (want.astype(np.int64) + k).astype(np.uint8)), k


def _exchange_worker(rank, world, port, name, res, nframes, interleave, out_q):
    """bench.py's N > 1 frame loop (rtx.distributed.FrameExchange: frame k sharded over the
    ranks and gathered to rank k mod N, N frames per all_to_all) with the host emulation as
    each rank's renderer. Frame k's rows are the scene's plus k (mod 256), so a frame that
    reaches the wrong owner or slot fails the comparison."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), os.path.join(os.path.dirname(here), "python-raytracer_amd"), here):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import hostemu
    from common import product_scene
    from rtx.distributed import FrameExchange, to_rgb8
    sc = product_scene(name, res)
    cache = {}

    def render_block(out, rows, k):
        if "rows" not in cache:
            cache["rows"] = to_rgb8(torch.from_numpy(hostemu.render_rows(sc, rows, threads=2)))
        out.copy_(cache["rows"] + k)  # uint8 wraps
    ex = FrameExchange(sc, rank, world, device=torch.device("cpu"), render_block=render_block, interleave=interleave)
    got = []  # frames are views of a receive buffer: keep copies (the buffer is reused)
    for _ in range(nframes):
        got += [(k, f.clone().numpy()) for k, f in ex.step()]
    got += [(k, f.clone().numpy()) for k, f in ex.flush()]
    out_q.put((rank, got))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,res,interleave,nframes", [(1, (40, 23), True, 3), (1, (40, 24), False, 2),
                                                          (2, (40, 23), True, 5), (3, (33, 26), True, 7),
                                                          (2, (40, 24), False, 4), (3, (20, 13), False, 2),
                                                          (4, (24, 20), False, 9), (4, (24, 41), True, 8),
                                                          (4, (16, 20), True, 6)])  # rank 3 has no rows
def test_frame_exchange_delivers_every_frame_to_its_owner(world, res, interleave, nframes):
    from common import oracle_render
    from oracle import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exchange_worker, args=(r, world, port, "MirrorRefraction", res, nframes, interleave, q))
             for r in range(world)]
    for p in procs:
        p.start()
    per_rank = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = O.to_png_array(oracle_render("MirrorRefraction", res))
    seen = []
    for r, frames in per_rank.items():
        for k, f in frames:
            assert k % world == r, (k, r)
            assert np.array_equal(f, (want.astype(np.int64) + k).astype(np.uint8)), (k, r)
            seen.append(k)
    assert sorted(seen) == list(range(nframes))


@pytest.mark.parametrize("world,res", [(2, (40, 23)), (3, (17, 10))])
def test_gather_row_blocks(world, res):
    from common import oracle_render
    from oracle import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, "MirrorRefraction", res, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(4))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = oracle_render("MirrorRefraction", res)
    fb_ref = np.transpose(ref, (1, 0, 2))[::-1].astype(np.float32)
    assert np.array_equal(got["torch.float32"], fb_ref)
    assert np.array_equal(got["torch.uint8"], O.to_png_array(ref))
    assert np.array_equal(got["interleaved torch.float32"], fb_ref)
    assert np.array_equal(got["interleaved torch.uint8"], O.to_png_array(ref))


@pytest.mark.parametrize("height", [1, 7, 8, 9, 23, 64, 181, 1080, 2160])
def test_interleaved_groups_partition_the_rows(height):
    """group_rows (Python) and rtx_group_rows (C ABI, host-only) agree, and the ranks'
    8-row groups partition the image rows."""
    from rtx import _native as N
    from rtx.scene import group_rows
    lib = N.load()
    for n in (1, 2, 3, 4, 5, 8):
        parts = [group_rows(height, n, k) for k in range(n)]
        assert np.array_equal(np.sort(np.concatenate(parts)), np.arange(height))
        for k in range(n):
            assert lib.rtx_group_rows(height, k, n) == len(parts[k])
            assert np.all(np.diff(parts[k]) > 0)
    assert lib.rtx_group_rows(height, 3, 3) == -1 and lib.rtx_group_rows(height, -1, 2) == -1


def test_glue_reassembles_strips(tmp_path):
    """rtx.glue over render(k, N) strips == full render (provided/glue.py semantics)."""
    import hostemu
    from common import product_scene
    from oracle import oracle as O
    from rtx.glue import glue
    sc = product_scene("TwoSpheresPlane", (37, 20))
    for k in range(4):
        img, _ = hostemu.render(sc, k, 4)
        np.save(tmp_path / ("%d.npy" % k), img)
    full, _ = hostemu.render(sc)
    assert np.array_equal(glue(str(tmp_path)), O.to_png_array(full))
