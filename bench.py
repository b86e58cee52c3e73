#!/usr/bin/env python3
"""Benchmark of the MI355X render path (BASELINE.json metric: Mrays/sec + frame ms,
TwoSpheresPlane 1920x1080 @1/2/4/8 GPUs).

The unit is the reference's: primary samples W*H*aa*dof*|times| per second (its tqdm bar,
provided/scene.py:45,71). One step = one 1920x1080 1-spp frame of TwoSpheresPlane.
N = 1: the frame is rendered into the fp32 framebuffer on one GPU.
N > 1 ("scaling": "strong", the north star's 1 -> 8-GPU tile scaling): ONE frame per step,
sharded across the ranks -- each renders its interleaved 8-row groups straight to uint8
on its GPU -- and gathered to rank 0 by one RCCL gather, awaited before the next frame
(measure_sharded). Reported beside it: the frame-stream throughput of one static scene
state (rtx.distributed.FrameExchange, "throughput"), every frame gathered to rank 0 in a
double-buffered stream ("gather_to_rank0") and the frame-parallel rate (each rank its own
frame, "weak_scaling"). DepthOfField 4K (--config dof4k) is the render-bound scaling
config; the TwoSpheresPlane 1080p frame is the metric's.

Launch: python bench.py [--steps K --warmup W]          (N = 1)
        python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "python-raytracer_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "Mrays/sec + frame ms, TwoSpheresPlane 1920×1080 @1/2/4/8 GPUs"
METRIC_OTHER = "Mrays/sec + frame ms, %s"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)

CONFIGS = {
    # name: (bundled scene, resolution, (aa, dof) or None, description)
    "tsp1080": ("TwoSpheresPlane", (1920, 1080), (1, None), "TwoSpheresPlane 1920x1080 1spp (primary + shadow rays)"),
    "tm1080": ("TorusMesh", (1920, 1080), (1, None), "TorusMesh 1920x1080 1spp (128-triangle mesh)"),
    "mr1080": ("MirrorRefraction", (1920, 1080), (1, None), "MirrorRefraction 1920x1080 1spp (reflect/refract chains)"),
    "dof4k": ("DepthOfField", (3840, 2160), (2, 32), "DepthOfField 3840x2160 AA2 x DOF32 = 64spp, jittered"),
    "ns1": ("NovelScene1", (2048, 1024), None, "NovelScene1 2048x1024 AA32 jittered (CSG hierarchies + textures)"),
    "ns2": ("NovelScene2", (1024, 512), None,
            "NovelScene2 1024x512 AA2 x DOF15 x 16 motion times, jittered (CSG hierarchies + textures)"),
    "blob1080": ("blob", (1920, 1080), None,
                 "81,920-face smooth mesh 1920x1080 1spp (bunny-sized stand-in; reference bunny.obj is absent)"),
}
# The render-bound config beside the metric's at N > 1.
SCALING_CONFIG = "dof4k"
# CPU-baseline sub-sampling for the configs whose full frame takes minutes on one core:
# the first of N column strips (np.array_split(arange(W), N)[0]) per repeat.
CPU_STRIPS = {"tm1080": 16, "dof4k": 16, "ns1": 32, "ns2": 128, "blob1080": 64}


def scene_dict(cfg):
    """(scene dict, asset dir) of a config: a bundled scene, or the synthetic large mesh."""
    name, res, spp, _ = CONFIGS[cfg]
    if name == "blob":
        sys.path.insert(0, os.path.join(REPO, "tests"))
        from scenegen import blob_obj, blob_scene
        path = os.path.join("/tmp", "rtx_blob6_%d.obj" % os.getpid())
        if not os.path.exists(path):
            blob_obj(path, level=6)
        return blob_scene(path, res), os.path.dirname(path)
    from rtx.io import bundled_scene_dict
    d = bundled_scene_dict(name, resolution=res, spp=spp)
    base = d.pop("__base_dir__")
    return d, base


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--config", default="tsp1080", choices=sorted(CONFIGS))
    p.add_argument("--cpu-seconds", type=float, default=10.0,
                   help="budget of the C-restatement CPU line (0 = skip both CPU lines)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--clock-warmup-s", type=float, default=0.3,
                   help="untimed sustained rendering before the warm-up steps, so the GPU clocks settle")
    p.add_argument("--force-dist", action="store_true", help="initialise torch.distributed even for one rank (tests)")
    p.add_argument("--pipeline", action="store_true",
                   help="run the multi-GPU frame loop (sharded frames + RCCL exchange) even at N = 1 (rehearsal)")
    p.add_argument("--no-graph", action="store_true",
                   help="N > 1: launch each frame's render from Python instead of one HIP graph per group")
    p.add_argument("--pmc-json", default=None,
                   help="tools/pmc_summary.py output for this config (default profiles/pmc_<config>.json)")
    return p.parse_args()


def pmc_traffic(path):
    """HBM bytes per launch measured by rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE in
    separate passes, gfx950 FETCH correction) — see tools/pmc_session.sh."""
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get("hbm_bytes_per_launch"), path
    except (OSError, ValueError):
        return None, None


# VALU issue ceiling: 1024 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU instruction
# (MI355X_MICROARCH.md: a SIMD issues a wave64 v_fma_f32 over 2 cycles).
VALU_PEAK_GINST_S = 1024 * 2.4 / 2.0


def pmc_valu(path):
    """VALU wave-instructions per launch from the same PMC summary (SQ_INSTS_VALU)."""
    try:
        with open(path) as f:
            return json.load(f)["counters_per_dispatch"]["SQ_INSTS_VALU"]
    except (OSError, ValueError, KeyError, TypeError):
        return None


def make_scene(cfg):
    import rtx
    d, base = scene_dict(cfg)
    if cfg == "dof4k":
        d["AA"] = {"jitter": True, "samples": CONFIGS[cfg][2][0]}
    d["__base_dir__"] = base
    return rtx.load_scene(d, verbose=False)


def cpu_threads():
    """Host threads for the CPU baseline: the GPU box's CPU share (16 per GPU), or fewer
    cores when the machine has them; RTX_CPU_THREADS overrides."""
    n = os.environ.get("RTX_CPU_THREADS")
    if n:
        return max(1, int(n))
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    return max(1, min(16, avail))


def cpu_baseline_native(cfg, budget_s, threads=None):
    """The oracle (C restatement of the reference) on the same workload, as the reference
    parallelises it: column strips (scene.py:35-37 `np.array_split`, render.nu's tasks),
    one strip per host thread (ctypes releases the GIL; every oracle_render call builds
    its own scene). Whole frames (or the config's fixed sub-sample) repeated until the
    budget is used."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle as O
    name, res, spp, _ = CONFIGS[cfg]
    d, base = scene_dict(cfg)
    osc = O.OracleScene(d, base)
    W, H = res
    P = threads or cpu_threads()
    frac = CPU_STRIPS.get(cfg, 1)  # render the first 1/frac of the columns
    tasks = P * frac
    strips = [len(c) for c in np.array_split(np.arange(W), tasks)[:P]]
    noises = [None] * P
    if osc.jitter:
        rs = np.random.RandomState(0)
        noises = [rs.rand(nc * H * osc.spp_rays * 3) for nc in strips]
    ncol = sum(strips)

    def one(k):
        osc.render(k, tasks, noise=noises[k])

    nsamp = 0
    frames = 0
    with ThreadPoolExecutor(P) as ex:
        t0 = time.perf_counter()
        while True:
            list(ex.map(one, range(P)))
            nsamp += ncol * H * osc.n_samples
            frames += 1
            if time.perf_counter() - t0 >= budget_s:
                break
        dt = time.perf_counter() - t0
    if frac == 1:
        sample = "full %dx%d frame(s)" % (W, H)
    else:
        sample = "columns 0..%d of %dx%d (1/%d of the frame)" % (ncol - 1, W, H, frac)
    return {"value": nsamp / dt / 1e6, "unit": "Mrays/s", "cores": P, "kind": "port (C restatement)",
            "sample": "%s x %d repeats in %.1f s; %d column strips (np.array_split, as render.nu) on %d host "
                      "threads (oracle/rtx_oracle.c, gcc -O2)" % (sample, frames, dt, P, P)}


# Python-loop baseline: rows j = j0, j0 + R, j0 + 2R, ... (reference row index) of the
# full-width frame, (R, j0[, C]) per config; every row for the 1080p configs whose whole
# frame fits the budget. NovelScene1 (CSG + textures, ~270 samples/s per process): its
# middle row. C: only the first C columns of each process's strip -- NovelScene2 (480
# samples per pixel) and the 81,920-face mesh (a Python loop over every face per ray).
PY_ROW_STRIDE = {"tsp1080": (1, 0), "mr1080": (1, 0), "tm1080": (16, 0), "dof4k": (270, 0), "ns1": (1024, 512),
                 "ns2": (512, 256, 4), "blob1080": (1080, 540, 6)}
_PY = {}


def _py_init(cfg):
    from oracle import oracle as O
    from oracle import pyloop as PL
    d, base = scene_dict(cfg)
    osc = O.OracleScene(d, base)
    _PY["scene"] = PL.PyLoopScene(osc)
    _PY["spp"] = osc.n_samples
    _PY["jitter"] = osc.jitter


def _py_strip(args):
    """One np.array_split column strip (render.nu's --subimage k --tasks N process)."""
    k, tasks, rows, cols = args
    sc = _PY["scene"]
    ncol = len(np.array_split(np.arange(sc.width), tasks)[k])
    if cols is not None:
        ncol = min(ncol, cols)
    noise = np.random.RandomState(k).rand(ncol * len(rows) * sc.samples * sc.dof_samples * 3) if _PY["jitter"] else None
    t0 = time.perf_counter()
    sc.render(k, tasks, rows=rows, noise=noise, cols=cols)
    return ncol * len(rows) * _PY["spp"], time.perf_counter() - t0


def cpu_baseline(cfg, processes=None):
    """The reference's Python render loop (oracle/pyloop.py: per pixel, sample, ray and
    object Python calls, PyGLM's fp32 on numpy scalars; bit-identical to the C oracle,
    tests/test_pyloop.py) on the host, parallelised as the reference does it: P processes,
    one np.array_split column strip each (provided/scene.py:36-37, render.nu). Runs before
    the GPU is initialised (forked workers)."""
    import multiprocessing as mp
    if cfg not in PY_ROW_STRIDE:
        return None
    _, res, _, _ = CONFIGS[cfg]
    W, H = res
    P = processes or cpu_threads()
    stride, j0 = PY_ROW_STRIDE[cfg][:2]
    cols = PY_ROW_STRIDE[cfg][2] if len(PY_ROW_STRIDE[cfg]) > 2 else None
    rows = list(range(j0, H, stride))
    with mp.get_context("fork").Pool(P, initializer=_py_init, initargs=(cfg,)) as pool:
        pool.map(_py_init, [cfg] * P)  # every worker built its scene before the clock starts
        t0 = time.perf_counter()
        res_ = pool.map(_py_strip, [(k, P, rows, cols) for k in range(P)], chunksize=1)
        dt = time.perf_counter() - t0
    nsamp = sum(r[0] for r in res_)
    cpu = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next(line.split(":", 1)[1].strip() for line in f if line.startswith("model name"))
    except (OSError, StopIteration):
        pass
    sample = "full %dx%d frame" % (W, H) if stride == 1 else \
        "rows %s (%d of %d) of the %dx%d frame" % (", ".join(str(r) for r in rows[:3]) + (", ..." if len(rows) > 3 else ""),
                                                   len(rows), H, W, H)
    if cols is not None:
        sample += ", the first %d columns of each process's strip" % cols
    return {"value": nsamp / dt / 1e6, "unit": "Mrays/s", "cores": P, "kind": "port",
            "sample": "%s, %d samples in %.1f s; %d processes, one np.array_split column strip each (as render.nu); "
                      "oracle/pyloop.py: the reference's per-sample Python loop, bit-identical to the C oracle; "
                      "host CPU %s" % (sample, nsamp, dt, P, cpu)}


def kernel_ms(fn, n, stream):
    """Average duration of fn() over n calls from HIP events on the launch stream (events
    bracket the whole run: per-call events would insert gaps between launches)."""
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(n):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def clock_warmup(fn, seconds, sync):
    """Untimed frames until `seconds` of sustained GPU work have run, before the W warm-up
    steps: the MI355X raises its clocks only under sustained load. TSP 1080p measured
    26.3 us per frame after 10 warm-up frames and 23.9 us after 4,000 (~0.1 s), with the same
    kernel (profiles/r03/warm/). Returns (frames, seconds)."""
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(16):
            fn()
        sync()
        n += 16
    return n, time.perf_counter() - t0


def max_over_ranks(x, use_dist, device="cuda"):
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    if use_dist:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def cuda_sync():
    torch.cuda.synchronize()


def timed(fn, steps, use_dist, sync=cuda_sync, device="cuda"):
    """Wall time of `steps` calls of fn, bracketed by barrier + synchronize on both sides;
    the max over ranks is the job's time. Each rank's clock stops when its own work is done;
    the closing barrier keeps every rank inside the bracket."""
    if use_dist:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    sync()
    t1 = time.perf_counter()
    if use_dist:
        dist.barrier()
    return max_over_ranks(t1 - t0, use_dist, device)


def root_shares(world):
    """Candidate shares of the frame's rows for rank 0 in the value loop's uneven blocks
    (rtx.distributed.BlockGather): from an even split up to 0.9 -- every rank keeps rows."""
    c = [1.0 / world, 1.5 / world, 2.0 / world, 3.0 / world, 0.5, 0.6, 0.7, 0.8, 0.9]
    return sorted(set(round(x, 4) for x in c if 1.0 / world - 1e-9 <= x <= 0.9))


def sharded_frame(sc, rank, world, steps, warmup, use_dist, device, sync=cuda_sync, stream=None, render_rows=None,
                  graph=True, collective_at_one=False, tune=True):
    """ONE frame sharded over the ranks per step (the N > 1 value; rtx.distributed.FrameGraph):
    every step renders this rank's rows of the frame straight to uint8 (fused, one launch),
    gathers them to rank 0 (one RCCL collective) and, for interleaved rows, puts them in
    image order on rank 0 -- recorded once as a HIP graph and replayed per frame, so a frame
    costs one graph launch of host time. Frames are stream-ordered: each frame's gather
    completes before the next frame renders. No batching and no overlap across frames: the
    latency of one frame, the reference's one-frame-per-run strip render + glue
    (render.nu:10-15, provided/glue.py:17-27). The timed loop issues its frames from C,
    frames_per_graph per graph launch (FrameGraph.run).
    Partition: one-sample frames in contiguous row blocks, rank 0's share TUNED before the
    timed region (tune, N > 1): rank 0's own rows cross no link while every other row is
    carried into rank 0 by the collective, so the frame is fastest when rank 0 renders more
    than 1/N of it; each candidate share (root_shares) is timed over
    the same loop (max over ranks, so every rank picks the same one). Multi-sample frames
    (render-bound): interleaved 8-row groups, one gather, reordered on rank 0.
    Returns (seconds for `steps` frames, max over ranks; rank 0's last frame [H, W, 3];
    the loop's description)."""
    from rtx.distributed import FrameGraph
    H = sc.vc.height
    blocks = sc.samples_per_pixel == 1
    tuning, root_rows = [], None

    def build(x):
        return FrameGraph(sc, rank, world, dst=0, device=device, render_block=render_rows, graph=graph,
                          collective_at_one=collective_at_one, root_rows=x)
    if tune and blocks and world > 1:
        m = max(4, min(steps, 100))
        for share in root_shares(world):
            x = min(max(int(round(share * H)), 1), H - (world - 1))
            fg = build(x)
            for _ in range(max(1, min(warmup, 3))):
                fg.step()
            fg.run(2 * fg.kmax if fg.graph_on else 1, stream)
            sync()
            t = timed(lambda: fg.run(m, stream), 1, use_dist, sync, device) / m
            tuning.append({"root_rows": x, "share": share, "frame_us": round(t * 1e6, 3)})
            del fg
        root_rows = min(tuning, key=lambda e: e["frame_us"])["root_rows"]
    fg = build(root_rows)
    for _ in range(warmup):
        fg.step()
    fg.run(2 * fg.kmax if fg.graph_on else 1, stream)  # (records and warms the multi-frame graph too)
    sync()
    # the timed region: `steps` frames, issued from C (rtx_graph_launch, fg.kmax frames per
    # graph launch; each frame rendered, gathered and reordered before the next starts)
    s = timed(lambda: fg.run(steps, stream), 1, use_dist, sync, device)
    # host issue per frame (outside the timed region): the clock stopped before the device
    # finishes, for run() and for one Python step() per frame
    t0 = time.perf_counter()
    fg.run(steps, stream)
    t1 = time.perf_counter()
    sync()
    t2 = time.perf_counter()
    for _ in range(steps):
        fg.step()
    t3 = time.perf_counter()
    sync()
    last = fg.frame()
    nrows = [len(r) for r in fg.g.rows]
    if fg.interleave:
        part = "interleaved 8-row groups, one gather to rank 0, reordered there"
    elif fg.root_rows is not None:
        part = ("contiguous row blocks, rank 0 renders rows 0-%d itself (its share tuned over %d candidates), "
                "the others np.array_split the rest; one all_to_all_single with uneven splits brings them to rank 0 "
                "in image order" % (fg.root_rows - 1, len(tuning)))
    else:
        part = "contiguous row blocks (np.array_split), one gather to rank 0"
    info = {"graph": fg.graph is not None, "frames_per_graph": fg.kmax if fg.graphk is not None else 1,
            "rows_per_rank": nrows if len(nrows) <= 16 else [min(nrows), max(nrows)],
            "partition": part, "in_order": bool(fg.g.in_order),
            "host_issue_us_per_frame": round((t1 - t0) * 1e6 / steps, 3),
            "host_issue_step_us_per_frame": round((t3 - t2) * 1e6 / steps, 3)}
    if tuning:
        info["root_share_tuning"] = tuning
    return s, (last.clone() if last is not None else None), info


def sharded_config_field(cfg, sc, rank, world, steps, warmup, use_dist, device, sync=cuda_sync, stream=None,
                         render_rows=None):
    """The scaling config's sharded frame beside the metric's (DESIGN.md section 7:
    DepthOfField 4K is render-bound at every N, TwoSpheresPlane 1080p is link-bound at
    N = 2): the same one-frame-per-step loop as the value, on `sc`."""
    s, _, _ = sharded_frame(sc, rank, world, steps, warmup, use_dist, device, sync, stream, render_rows)
    W, H = sc.vc.width, sc.vc.height
    return {"config": cfg, "workload": CONFIGS[cfg][3], "steps": steps, "frame_ms": round(s * 1e3 / steps, 5),
            "Mrays_s": round(W * H * sc.samples_per_pixel * steps / s / 1e6, 3),
            "note": "one frame per step sharded over the N ranks (uint8 rows) and gathered to rank 0, awaited: "
                    "the value's loop on the render-bound scaling config"}


def measure_sharded(sc, rank, world, steps, warmup, use_dist, device, sync=cuda_sync, stream=None,
                    render_rows=None, render_block=None, render_block_k=None, graph=True, collective_at_one=False):
    """The N > 1 measurements (bench.py's multi-GPU leg; at N = 1 with --pipeline a
    rehearsal). Renderers default to the HIP kernels on this rank's GPU; the CPU tests
    inject the host emulation (tests/test_bench_multirank.py).

    - value: ONE frame sharded over the ranks, frame by frame (sharded_frame).
    - throughput: the frame stream of one static scene state (rtx.distributed.FrameExchange:
      frame k to rank k mod N, N frames per batched launch and per all_to_all, overlapped).
    - gather_to_rank0: the same stream with every frame gathered to rank 0 (FramePipeline).
    Returns a dict (times are the max over ranks) and, on rank 0, the last frame of the
    value loop ([H, W, 3] uint8)."""
    from rtx.distributed import FrameExchange, FramePipeline
    H, W = sc.vc.height, sc.vc.width
    spp = sc.samples_per_pixel
    frame_s, last_frame, loop = sharded_frame(sc, rank, world, steps, warmup, use_dist, device, sync, stream,
                                              render_rows, graph=graph, collective_at_one=collective_at_one)

    def run_frames(loop, n):
        if use_dist:
            dist.barrier()
        sync()
        t0 = time.perf_counter()
        for _ in range(n):
            loop.step()
        loop.flush()
        sync()
        t1 = time.perf_counter()
        if use_dist:
            dist.barrier()
        return max_over_ranks(t1 - t0, use_dist, device)
    ex = FrameExchange(sc, rank, world, device=device, render_block=render_block_k, graph=graph)
    for _ in range(warmup):
        ex.step()
    ex.flush()
    sync()
    stream_s = run_frames(ex, steps)
    pipe = FramePipeline(sc, rank, world, device=device, render_block=render_block)
    for _ in range(warmup):
        pipe.step()
    pipe.flush()
    rank0_s = run_frames(pipe, steps)

    def rate(s):
        return round(W * H * spp * steps / s / 1e6, 3)
    out = {
        "frame_s": frame_s,
        "frame_ms": round(frame_s * 1e3 / steps, 5),
        "rows_per_rank": loop["rows_per_rank"],
        "partition": loop["partition"],
        "collective": "one RCCL collective per frame bringing the ranks' uint8 rows to rank 0, stream-ordered",
        "frame_loop": dict(loop, note="render + gather + reorder recorded as a HIP graph (FrameGraph): the timed "
                                      "frames issued from C, frames_per_graph frames per graph launch "
                                      "(host_issue_us_per_frame); host_issue_step: one Python step() per frame"),
        "throughput": {
            "frame_ms": round(stream_s * 1e3 / steps, 5), "Mrays_s": rate(stream_s),
            "launch": ("one batched launch per group of N frames (rtx_render_groups_frames)" if ex.render_frames
                       else "one HIP graph of the group's N renders per group" if ex.graph else "eager"),
            "note": "frame-stream throughput of one static scene state (rtx.distributed.FrameExchange): frame k "
                    "sharded over the N ranks and gathered to rank k mod N; a group of N frames rendered in ONE "
                    "batched launch per rank and exchanged by one all_to_all, overlapped with the next group"},
        "gather_to_rank0": {
            "frame_ms": round(rank0_s * 1e3 / steps, 5), "Mrays_s": rate(rank0_s),
            "note": "FramePipeline: every frame gathered to rank 0, double-buffered (its ingress bounds the rate)"},
        "headline": "value = ONE frame sharded over the N ranks (uint8 rows, fused) and gathered to rank 0, "
                    "frame by frame (one HIP graph launch each), stream-ordered: no batching or overlap across frames",
    }
    return out, last_frame


def rgb8_field(render_u8, steps, timer, W, H, spp, kernel):
    """The N = 1 frame into uint8 (main.py's PNG bytes from the fused kernel,
    rtx_render_rgb8): the output every N > 1 rank renders, so the 1 -> N ratio can be taken
    on the same bytes. timer(fn, n) -> ms per call (HIP events on the launch stream)."""
    ms = timer(render_u8, steps)
    return {"frame_ms": round(ms, 5), "Mrays_s": round(W * H * spp / ms / 1e3, 3), "kernel": kernel(),
            "note": "the same frame rendered straight to uint8 (rtx_render_rgb8, 3 B/pixel), as each rank does "
                    "at N > 1; HIP events over the same number of launches"}


def roofline(bytes_alg, kern_ms, rows_frac, pmc_path):
    """The dominant kernel's roofline. The bound is VALU issue: the megakernel keeps its rays
    in registers and moves little more than its framebuffer, so the counters show issue,
    not HBM, as the limiter. achieved = SQ_INSTS_VALU per launch
    (rocprofv3 PMC pass of the same kernel, committed under profiles/) / the kernel's
    average duration; peak = 1024 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU instruction
    (MI355X_MICROARCH.md). Every instruction is priced at that 2-cycle rate, so frac <= 1
    (fp64, transcendental and VOP3 forms take longer). Beside it: the measured HBM bytes
    (2 x FETCH_SIZE + WRITE_SIZE) against 8 TB/s (frac_hbm), and SURVEY.md 8(d)'s
    algorithmic byte model (model_frac: SoA ray records this kernel never stores)."""
    secs = kern_ms * 1e-3
    traffic, src = pmc_traffic(pmc_path)
    valu = pmc_valu(pmc_path) if src else None
    if src:
        src = os.path.relpath(src, REPO)
    roof = {"bound": "valu", "achieved": None, "peak": VALU_PEAK_GINST_S, "unit": "G wave64 VALU instructions/s",
            "frac": None, "traffic": None,
            "traffic_unit": "HBM bytes/launch (rocprofv3 PMC: 2 x FETCH_SIZE + WRITE_SIZE)", "source": src,
            "model_bytes_per_launch": int(bytes_alg),
            "model_frac": round(bytes_alg / secs / 1e9 / HBM_PEAK_GBS, 5),
            "model": "SURVEY.md 8(d): 32 B x ray segments + 12 B x pixels per frame, priced at 8 TB/s: the SoA "
                     "ray records of a wavefront design, which this megakernel keeps in registers (not a bound)"}
    if valu:
        v = valu * rows_frac
        ach = v / secs / 1e9
        roof.update(achieved=round(ach, 2), frac=round(ach / VALU_PEAK_GINST_S, 5), valu_insts_per_launch=int(v),
                    issue_floor_us=round(v / VALU_PEAK_GINST_S / 1e3, 3))
    else:
        roof["note"] = "no PMC summary for this config: the VALU fraction is unmeasured"
    if traffic is not None:
        traffic = int(round(traffic * rows_frac))
        roof.update(traffic=traffic, achieved_hbm_GBs=round(traffic / secs / 1e9, 2),
                    frac_hbm=round(traffic / secs / 1e9 / HBM_PEAK_GBS, 5))
    return roof


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            sys.exit("--gpus %d needs torch.distributed.run with %d processes" % (a.gpus, a.gpus))
    cpu = {}
    if world == 1 and not a.no_cpu_baseline and a.cpu_seconds > 0:
        # host baselines first, before this process touches the GPU (the Python loop forks)
        cpu["cpu_baseline"] = cpu_baseline(a.config)
        cpu["cpu_baseline_native"] = cpu_baseline_native(a.config, a.cpu_seconds)
        if cpu["cpu_baseline"] is None:  # configs without a Python-loop sample: C restatement only
            cpu["cpu_baseline"] = cpu.pop("cpu_baseline_native")
    torch.cuda.set_device(local)
    use_dist = world > 1 or a.force_dist or a.pipeline
    if use_dist:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import rtx  # noqa: F401

    # setup cost, outside the timed region (the reference re-parses and re-renders per
    # main.py run, provided/main.py:25-34): host parse, rtx_scene_create (records, mesh
    # BVH, light grids), rtx_camera_set (tables, primary-ray bins) and the first frame
    # (scene-specialized kernel: hiprtc compile, or a load from the on-disk cache)
    jit_dir = os.environ.get("RTX_JIT_CACHE") or "/tmp/rtx_jit_%d" % os.getuid()

    def n_cached():
        try:
            return len(os.listdir(jit_dir))
        except OSError:
            return 0
    tc = time.perf_counter()
    torch.zeros(1, device="cuda")  # the process's HIP context (not a scene cost)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sc = make_scene(a.config)
    t1 = time.perf_counter()
    sc.native()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    sc._set_camera(0, 1)
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    W, H = sc.vc.width, sc.vc.height
    spp = sc.samples_per_pixel
    stream = torch.cuda.current_stream()
    fb = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    cached0 = n_cached()
    t4 = time.perf_counter()
    sc.render_device(out=fb)
    torch.cuda.synchronize()
    t5 = time.perf_counter()
    first_kernel = sc.last_kernel
    sc.jit_wait()  # the specialized kernel (compiling on a host thread since the first frame)
    sc.render_device(out=fb)
    torch.cuda.synchronize()
    t6 = time.perf_counter()
    if first_kernel.startswith(("rtx_jit_render_", "rtx_jit_split_")):
        how = "specialized kernel, compiled (hiprtc)" if n_cached() > cached0 else \
            "specialized kernel, code object from the disk cache"
    else:
        how = "generic kernel %s while the specialized one compiles on a host thread (%s)" % (
            first_kernel, "hiprtc" if n_cached() > cached0 else "code object from the disk cache")
    setup = {"hip_context_ms": round((t0 - tc) * 1e3, 3), "parse_ms": round((t1 - t0) * 1e3, 3),
             "scene_create_ms": round((t2 - t1) * 1e3, 3), "camera_set_ms": round((t3 - t2) * 1e3, 3),
             "first_frame_ms": round((t5 - t4) * 1e3, 3), "first_frame_kernel": how,
             "specialized_ready_ms": round((t6 - t4) * 1e3, 3), "specialized_kernel": sc.last_kernel,
             "note": "outside the timed region; first_frame_ms includes one render; specialized_ready_ms: from the "
                     "first frame's start to the end of the first frame with the specialized kernel"}

    # ray-segment census for the algorithmic byte model (separate counting launch)
    cnt = torch.zeros(16, dtype=torch.int64, device="cuda")
    sc.render_device(out=fb, counters=cnt)
    c = cnt.cpu().numpy()
    sc.jit_wait()  # (no compile left running on a host thread during the timed regions)
    cast_rays = int(c[:10].sum())
    shadow_rays = int(c[10])
    segments = cast_rays + shadow_rays
    b_alg = 32 * segments + 12 * W * H  # 32 B per segment + 12 B/pixel fp32 RGB

    def full_frame():
        sc.render_device(out=fb, stream=stream)

    extra = {}
    if world == 1 and not a.pipeline:
        # N = 1: one step = one whole frame into the fp32 framebuffer
        fb8 = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda")

        def frame_u8():
            sc.render_device(out=fb8, stream=stream)
        frame_u8()  # the uint8 variant of the specialized kernel, compiled before any timing
        sc.jit_wait()
        warm = clock_warmup(full_frame, a.clock_warmup_s, torch.cuda.synchronize)
        for _ in range(a.warmup):
            full_frame()
        torch.cuda.synchronize()
        wall_s = timed(full_frame, a.steps, use_dist)
        kern_ms = kernel_ms(full_frame, a.steps, stream)  # the render kernel alone, same launches
        kernel = sc.last_kernel
        clock_warmup(frame_u8, min(0.1, a.clock_warmup_s), torch.cuda.synchronize)  # (its own, right before it)
        for _ in range(a.warmup):
            frame_u8()
        extra["rgb8"] = rgb8_field(frame_u8, a.steps, lambda fn, n: kernel_ms(fn, n, stream), W, H, spp,
                                   lambda: sc.last_kernel)
        rows_frac = 1.0
        scaling, parallelism = "strong", "single GPU"
    else:
        # N > 1 (north star): one step = ONE frame sharded across the ranks (uint8 rows
        # rendered by every rank) and gathered to rank 0, awaited, frame by frame
        dev = torch.device("cuda", local)
        from rtx.distributed import rank_rows, row_block
        interleave = spp > 1  # the value loop's partition (rtx.distributed.FrameGraph)
        my_rows = rank_rows(H, world, rank, interleave)
        r0, nr = row_block(H, world, rank)
        warm_out = torch.empty((max(len(my_rows), 1), W, 3), dtype=torch.uint8, device="cuda")

        def rank_render(out):
            if interleave:
                sc.render_device(groups=(rank, world), out=out, stream=stream)
            else:
                sc.render_device(row0=r0, nrows=nr, out=out, stream=stream)

        def own_rows():  # clock warm-up on this rank's own rows (no collective)
            if len(my_rows):
                rank_render(warm_out[:len(my_rows)])
        own_rows()
        sc.jit_wait()  # (the specialized kernel compiles on a host thread meanwhile)
        warm = clock_warmup(own_rows, a.clock_warmup_s, torch.cuda.synchronize)
        mg, _ = measure_sharded(sc, rank, world, a.steps, a.warmup, use_dist, dev, stream=stream,
                                graph=not a.no_graph, collective_at_one=a.pipeline)
        wall_s = mg.pop("frame_s")
        # breakdown (outside the timed region): this rank's render alone, fp32 (the kernel
        # the roofline below prices) and uint8 (the one the frame loop runs), from HIP events
        rank_fb = torch.empty((max(len(my_rows), 1), W, 3), dtype=torch.float32, device="cuda")

        def fp32_rows():
            if len(my_rows):
                rank_render(rank_fb[:len(my_rows)])
        fp32_rows()  # (its first call may compile the fp32 variant of the specialized kernel)
        sc.jit_wait()
        torch.cuda.synchronize()
        kern_ms = max_over_ranks(kernel_ms(fp32_rows, a.steps, stream), use_dist)
        kernel = sc.last_kernel
        render_ms = max_over_ranks(kernel_ms(own_rows, a.steps, stream), use_dist)
        mg["render_ms_per_rank"] = round(kern_ms, 5)
        mg["render_rgb8_ms_per_rank"] = round(render_ms, 5)
        mg["kernel_rgb8"] = sc.last_kernel
        rows_frac = len(my_rows) / H
        extra["multi_gpu"] = mg
        # secondary: weak scaling (each rank renders its own whole frame per step)
        for _ in range(3):
            full_frame()
        weak_s = timed(full_frame, a.steps, use_dist)
        extra["weak_scaling"] = {"Mrays_s": round(world * W * H * spp * a.steps / weak_s / 1e6, 3),
                                 "ms_per_step": round(weak_s * 1e3 / a.steps, 5),
                                 "note": "frame-parallel: each rank renders its own whole frame, no collective"}
        if a.config != SCALING_CONFIG:  # the render-bound scaling config's sharded frame beside it
            sc2 = make_scene(SCALING_CONFIG)  # (its warm-up frames compile its kernel)
            extra["scaling_config"] = sharded_config_field(SCALING_CONFIG, sc2, rank, world, min(a.steps, 10), 2,
                                                           use_dist, dev, stream=stream)
        scaling, parallelism = "strong", "rows x %d ranks + one RCCL gather to rank 0 per frame" % world
    ms_per_step = wall_s * 1e3 / a.steps
    value = W * H * spp * a.steps / wall_s / 1e6

    if rank == 0:
        roof = roofline(b_alg * rows_frac, kern_ms, rows_frac,
                        a.pmc_json or os.path.join(REPO, "profiles", "pmc_%s.json" % a.config))
        out = {
            "metric": METRIC if a.config == "tsp1080" else METRIC_OTHER % CONFIGS[a.config][3],
            "value": round(value, 3), "unit": "Mrays/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "clock_warmup": {"frames": warm[0], "seconds": round(warm[1], 3),
                                                 "note": "untimed sustained rendering before the warm-up steps "
                                                         "(GPU clocks settle; rank-local at N > 1)"},
            "ms_per_step": round(ms_per_step, 5), "higher_is_better": True, "scaling": scaling,
            "vs_baseline": None, "dtype": "fp32 vectors + fp64 scalars (reference numerics)", "data": "synthetic",
            "config": {"workload": CONFIGS[a.config][3], "width": W, "height": H, "spp": spp,
                       "frames_per_step": 1, "parallelism": parallelism},
            "frame_ms": round(kern_ms, 5), "kernel": kernel,
            "segments_per_frame": segments, "cast_rays_per_frame": cast_rays, "shadow_rays_per_frame": shadow_rays,
            "roofline": roof,
        }
        out["setup_ms"] = setup
        out.update(extra)
        out.update(cpu)
        print(json.dumps(out), flush=True)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
