"""Wave timeline of one frame (experiment): every wave of a scene-specialized kernel built
with RTX_WAVE_LOG records its start and end (s_memrealtime, 100 MHz) and hardware ids
(rtx_kernels.h WaveClock). Prints the frame's span, wave durations, how many waves are
resident over the frame (per SIMD), the ramp-up and the drain.

usage (GPU box): python tools/wave_timeline.py --config tsp1080 [--json out.json]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "python-raytracer_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--config", default="tsp1080")
p.add_argument("--frames", type=int, default=2000)
p.add_argument("--json", default=None)
p.add_argument("--npz", default=None, help="per-wave start/end (us) and hardware ids, for schedule simulations")
a = p.parse_args()
os.environ["RTX_JIT_FLAGS"] = (os.environ.get("RTX_JIT_FLAGS", "") + " -DRTX_WAVE_LOG=1").strip()
torch.cuda.set_device(0)
import bench  # noqa: E402

sc = bench.make_scene(a.config)
W, H = sc.vc.width, sc.vc.height
n_waves = ((W + 7) // 8) * ((H + 7) // 8)
log = torch.zeros(4 * n_waves + 4096, dtype=torch.int64, device="cuda")
os.environ["RTX_WAVE_LOG_PTR"] = str(log.data_ptr())
fb = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
sc.render_device(out=fb)
torch.cuda.synchronize()
assert sc.last_kernel.startswith("rtx_jit_render_"), sc.last_kernel
for _ in range(a.frames):  # clocks settle
    sc.render_device(out=fb)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
sc.render_device(out=fb)
e1.record()
torch.cuda.synchronize()
ev_us = e0.elapsed_time(e1) * 1e3
L = log[:4 * n_waves].view(n_waves, 4).cpu().numpy().astype(np.int64)
t0, t1, hw, xcc = L[:, 0], L[:, 1], L[:, 2], L[:, 3]
assert (t1 >= t0).all() and (t0 > 0).all(), "log incomplete"
base = t0.min()
s = (t0 - base) * 0.01  # us
e = (t1 - base) * 0.01
dur = e - s
span = e.max()
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
se = (hw >> 13) & 7
xc = xcc & 15
n_simd = len(set(zip(xc.tolist(), se.tolist(), cu.tolist(), simd.tolist())))
grid = np.linspace(0, span, 201)
resident = np.array([((s <= t) & (e > t)).sum() for t in grid]) / max(n_simd, 1)
peak = resident.max()
ramp = grid[np.argmax(resident >= 0.9 * peak)]
drain_start = grid[len(grid) - 1 - np.argmax(resident[::-1] >= 0.9 * peak)]
out = {
    "config": a.config, "kernel": sc.last_kernel, "waves": int(n_waves), "simds_seen": int(n_simd),
    "event_us": round(ev_us, 3), "span_us": round(float(span), 3),
    "wave_us": {"mean": round(float(dur.mean()), 3), "p10": round(float(np.percentile(dur, 10)), 3),
                "median": round(float(np.median(dur)), 3), "p90": round(float(np.percentile(dur, 90)), 3),
                "max": round(float(dur.max()), 3)},
    "resident_waves_per_simd": {"peak": round(float(peak), 2), "mean": round(float(resident.mean()), 2)},
    "ramp_us_to_90pct": round(float(ramp), 3), "drain_us_from_90pct": round(float(span - drain_start), 3),
    "last_start_us": round(float(s.max()), 3),
    "per_xcc_span_us": {int(x): [round(float(s[xc == x].min()), 3), round(float(e[xc == x].max()), 3)]
                        for x in sorted(set(xc.tolist()))},
    "resident_profile": [round(float(r), 2) for r in resident[::10]],
    "start_profile_us": [round(float(np.percentile(s, q)), 3) for q in (1, 10, 25, 50, 75, 90, 99, 100)],
}
print(json.dumps(out))
if a.npz:
    np.savez_compressed(a.npz, start_us=s.astype(np.float32), end_us=e.astype(np.float32), xcc=xc.astype(np.int8),
                        se=se.astype(np.int8), cu=cu.astype(np.int8), simd=simd.astype(np.int8),
                        tiles_x=np.int32((W + 7) // 8))
if a.json:
    with open(a.json, "w") as f:
        json.dump(out, f, indent=1)
