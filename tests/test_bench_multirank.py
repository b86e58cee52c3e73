"""bench.py's N > 1 measurement (measure_sharded: one sharded frame per step, gathered to
rank 0 and awaited; the FrameExchange and FramePipeline streams beside it) run end to
end on world-size-2 and -3 gloo groups, with the tests-only host build of the device
source standing in for each rank's GPU: barriers, max-over-ranks timing and the three
frame loops in the order the bench runs them, and the delivered frame checked against the
oracle's PNG bytes."""
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


def _worker(rank, world, port, res, steps, out_q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), os.path.join(os.path.dirname(here), "python-raytracer_amd"), here):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    import hostemu
    from common import product_scene
    from rtx.distributed import to_rgb8
    sc = product_scene("MirrorRefraction", res)
    cache = {}
    calls = [0]

    def rows_u8(rows):
        key = tuple(int(r) for r in rows)
        if key not in cache:
            cache[key] = to_rgb8(torch.from_numpy(hostemu.render_rows(sc, np.asarray(rows), threads=2)))
        calls[0] += 1
        return cache[key]

    def render_rows(out, rows):  # the value loop (rtx.distributed.FrameGraph): this rank's rows
        out.copy_(rows_u8(rows))

    def render_block(out, rows):  # FramePipeline
        out.copy_(rows_u8(rows))

    def render_block_k(out, rows, k):  # FrameExchange
        out.copy_(rows_u8(rows))
    mg, frame = bench.measure_sharded(sc, rank, world, steps, 2, True, torch.device("cpu"), sync=lambda: None,
                                      render_rows=render_rows, render_block=render_block,
                                      render_block_k=render_block_k, graph=False)
    # the scaling config's sharded frame beside the value (here the same scene stands in)
    mg["scaling_config"] = bench.sharded_config_field("dof4k", sc, rank, world, 2, 1, True, torch.device("cpu"),
                                                      sync=lambda: None, render_rows=render_rows)
    out_q.put((rank, mg, None if frame is None else frame.clone().numpy(), calls[0]))
    dist.barrier()
    dist.destroy_process_group()


def bench_root_shares(world):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.dirname(here))
    import bench
    return bench.root_shares(world)


@pytest.mark.parametrize("world,res", [(2, (40, 23)), (3, (33, 26))])
def test_bench_sharded_frame_loop(world, res):
    from common import oracle_render
    from oracle import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    steps = 4
    procs = [ctx.Process(target=_worker, args=(r, world, port, res, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (mg, f, n)) for r, mg, f, n in (q.get(timeout=240) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = O.to_png_array(oracle_render("MirrorRefraction", res))
    mg0, frame0, _ = got[0]
    assert np.array_equal(frame0, want)  # the value loop's last frame, on rank 0
    for r in range(1, world):
        assert got[r][1] is None
        # every rank reports the same max-over-ranks times
        assert got[r][0]["frame_s"] == mg0["frame_s"]
        assert got[r][0]["throughput"]["frame_ms"] == mg0["throughput"]["frame_ms"]
    assert mg0["frame_s"] > 0 and mg0["frame_ms"] == round(mg0["frame_s"] * 1e3 / steps, 5)
    W, H = res
    assert mg0["throughput"]["Mrays_s"] > 0 and mg0["gather_to_rank0"]["Mrays_s"] > 0
    # one-sample frames: contiguous blocks, rank 0's share tuned over the candidate shares
    # (every rank agrees: the timings are maxima over ranks); every row rendered once
    loop = mg0["frame_loop"]
    assert loop["partition"].startswith("contiguous") and not loop["graph"]  # (gloo: eager)
    tuned = loop["root_share_tuning"]
    assert [e["share"] for e in tuned] == bench_root_shares(world)
    x = min(tuned, key=lambda e: e["frame_us"])["root_rows"]
    assert mg0["rows_per_rank"][0] == x and sum(mg0["rows_per_rank"]) == H
    assert all(n > 0 for n in mg0["rows_per_rank"])
    for r in range(1, world):
        assert got[r][0]["frame_loop"]["root_share_tuning"] == tuned
    # the fields the 1 -> N comparison needs: the scaling config's sharded frame at N > 1 ...
    sc_f = mg0["scaling_config"]
    assert sc_f["config"] == "dof4k" and sc_f["frame_ms"] > 0 and sc_f["Mrays_s"] > 0
    for r in range(1, world):
        assert got[r][0]["scaling_config"]["frame_ms"] == sc_f["frame_ms"]  # max over ranks


def test_bench_n1_line_has_rgb8_frame():
    """... and at N = 1 the uint8 frame (the bytes every N > 1 rank renders) beside the
    fp32 one: bench.rgb8_field with the host emulation's uint8 frame and a wall timer."""
    import sys
    import time
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), os.path.join(os.path.dirname(here), "python-raytracer_amd"), here):
        sys.path.insert(0, p)
    import bench
    import hostemu
    from common import product_scene, oracle_render
    from oracle import oracle as O
    from rtx.distributed import to_rgb8
    res = (24, 16)
    sc = product_scene("TwoSpheresPlane", res)
    out = {}

    def frame_u8():
        out["f"] = to_rgb8(torch.from_numpy(hostemu.render_rows(sc, np.arange(res[1]), threads=2)))

    def timer(fn, n):
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        return (time.perf_counter() - t0) * 1e3 / n
    f = bench.rgb8_field(frame_u8, 2, timer, res[0], res[1], 1, lambda: "hostemu")
    assert f["frame_ms"] > 0 and f["Mrays_s"] > 0 and f["kernel"] == "hostemu"
    assert np.array_equal(out["f"].numpy(), O.to_png_array(oracle_render("TwoSpheresPlane", res)))
