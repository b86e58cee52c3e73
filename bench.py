#!/usr/bin/env python3
"""Benchmark of the MI355X render path (BASELINE.json metric: Mrays/sec + frame ms,
TwoSpheresPlane 1920x1080).

One step = one 1920x1080 1-spp frame of TwoSpheresPlane rendered by each rank (the
primary sample is the reference's unit: its tqdm bar counts W*H*aa*dof*|times|,
provided/scene.py:45,71). With N ranks the job renders N frames per step, one per GPU
(frame-parallel weak scaling; no data-path collective). ``--rowblock`` additionally times
the north-star strong-scaling form: one frame split across ranks (interleaved 8-row groups,
which balance sky and ground rows) and gathered to rank 0 over RCCL.

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
    p.add_argument("--rowblock", action="store_true", help="also time row-block + RCCL gather of one frame")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget (0 = skip)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--force-dist", action="store_true", help="initialise torch.distributed even for one rank (tests)")
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


def cpu_baseline(cfg, budget_s, threads=None):
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
    return {"value": nsamp / dt / 1e6, "unit": "Mrays/s", "cores": P, "kind": "port",
            "sample": "%s x %d repeats in %.1f s; %d column strips (np.array_split, as render.nu) on %d host "
                      "threads (oracle/rtx_oracle.c, gcc -O2)" % (sample, frames, dt, P, P)}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            sys.exit("--gpus %d needs torch.distributed.run with %d processes" % (a.gpus, a.gpus))
    torch.cuda.set_device(local)
    use_dist = world > 1 or a.force_dist
    if use_dist:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import rtx  # noqa: F401
    from rtx.scene import group_rows

    sc = make_scene(a.config)
    W, H = sc.vc.width, sc.vc.height
    spp = sc.samples_per_pixel
    stream = torch.cuda.current_stream()
    fb = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")

    # ray-segment census for the algorithmic byte model (separate counting launch)
    cnt = torch.zeros(16, dtype=torch.int64, device="cuda")
    sc.render_device(out=fb, counters=cnt)
    c = cnt.cpu().numpy()
    cast_rays = int(c[:10].sum())
    shadow_rays = int(c[10])
    segments = cast_rays + shadow_rays
    b_alg = 32 * segments + 12 * W * H  # 32 B per segment + 12 B/pixel fp32 RGB

    for _ in range(a.warmup):
        sc.render_device(out=fb)
    torch.cuda.synchronize()

    # HIP events on the launch stream bracket the whole timed region (events between
    # launches would insert ~10 us gaps on ROCm); kernel time = elapsed / steps.
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if use_dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(a.steps):
        sc.render_device(out=fb, stream=stream)
    e1.record(stream)
    torch.cuda.synchronize()
    # each rank's clock stops when its own K frames are done; the closing barrier keeps
    # every rank inside the bracket and the max over ranks below is the job's time
    t1 = time.perf_counter()
    if use_dist:
        dist.barrier()
    wall = torch.tensor([t1 - t0], dtype=torch.float64, device="cuda")
    kern = torch.tensor([e0.elapsed_time(e1) / a.steps], dtype=torch.float64, device="cuda")
    if use_dist:
        dist.all_reduce(wall, op=dist.ReduceOp.MAX)
        dist.all_reduce(kern, op=dist.ReduceOp.MAX)
    wall_s = float(wall.item())
    kern_ms = float(kern.item())
    ms_per_step = wall_s * 1e3 / a.steps
    samples_per_step = world * W * H * spp
    value = samples_per_step * a.steps / wall_s / 1e6

    rowblock = None
    if a.rowblock and use_dist:
        from rtx.distributed import render_frame
        for _ in range(3):
            render_frame(sc, rank, world, dtype=torch.uint8, interleave=True)
        torch.cuda.synchronize()
        dist.barrier()
        r0 = time.perf_counter()
        nrb = max(5, a.steps // 2)
        for _ in range(nrb):
            render_frame(sc, rank, world, dtype=torch.uint8, interleave=True)
        torch.cuda.synchronize()
        dist.barrier()
        rb = torch.tensor([time.perf_counter() - r0], dtype=torch.float64, device="cuda")
        dist.all_reduce(rb, op=dist.ReduceOp.MAX)
        rb_ms = float(rb.item()) * 1e3 / nrb
        rowblock = {"ms_per_frame": rb_ms, "Mrays_s": W * H * spp / rb_ms / 1e3, "scaling": "strong",
                    "gather": "uint8 interleaved 8-row groups (rtx_render_groups) to rank 0 "
                              "(torch.distributed.gather, RCCL)",
                    "rows_per_rank": max(len(group_rows(H, world, r)) for r in range(world))}

    if rank == 0:
        achieved = b_alg / (kern_ms * 1e-3) / 1e9
        traffic, traffic_src = pmc_traffic(a.pmc_json or os.path.join(REPO, "profiles", "pmc_%s.json" % a.config))
        if traffic is not None:
            traffic = int(round(traffic))
            traffic_src = os.path.relpath(traffic_src, REPO)
        out = {
            "metric": METRIC if a.config == "tsp1080" else METRIC_OTHER % CONFIGS[a.config][3], "value": round(value, 3), "unit": "Mrays/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms_per_step, 5), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp32 vectors + fp64 scalars (reference numerics)", "data": "synthetic",
            "config": {"workload": CONFIGS[a.config][3], "width": W, "height": H, "spp": spp,
                       "frames_per_step": world,
                       "parallelism": "frame-parallel (one frame per rank per step)" if world > 1 else "single GPU"},
            "frame_ms": round(kern_ms, 5),
            "segments_per_frame": segments, "cast_rays_per_frame": cast_rays, "shadow_rays_per_frame": shadow_rays,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "traffic_unit": "bytes/launch (rocprofv3 PMC)", "traffic_source": traffic_src,
                         "model": "B_alg = 32 B x ray segments + 12 B x pixels per frame (SURVEY.md 8d) / kernel time",
                         "bytes_alg_per_frame": b_alg},
        }
        valu = pmc_valu(os.path.join(REPO, traffic_src)) if traffic_src else None
        if valu:
            ach = valu / (kern_ms * 1e-3) / 1e9
            # the kernel's second bound: VALU issue (the path computes; the HBM model
            # above charges algorithmic ray traffic that stays in registers). frac prices
            # every instruction at the 2-cycle fp32 rate (fp64, transcendental and VOP3
            # forms take longer, so 1.0 is not reachable)
            out["valu"] = {"insts_per_launch": int(valu), "achieved": round(ach, 1), "peak": VALU_PEAK_GINST_S,
                           "unit": "G wave64-instructions/s", "frac": round(ach / VALU_PEAK_GINST_S, 4),
                           "source": traffic_src}
        if rowblock:
            out["rowblock"] = rowblock
        if world == 1 and not a.no_cpu_baseline and a.cpu_seconds > 0:
            out["cpu_baseline"] = cpu_baseline(a.config, a.cpu_seconds)
        print(json.dumps(out), flush=True)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
