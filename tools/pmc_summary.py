"""Summarise a tools/pmc_session.sh run: counters of the render kernels per frame, and
HBM traffic per frame = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes (FETCH_SIZE/WRITE_SIZE
are KiB; on gfx950 FETCH_SIZE reads half the bytes of a wide stream -- MI355X_MICROARCH.md
§HBM -- so it is doubled).

A frame is one launch of the flat scenes' render kernel, or -- hierarchy scenes, split
passes (csrc/rtx_split.h) -- every chunk's trace / shadow / shade launch: per-frame values
sum the kernels' per-dispatch averages times their dispatches per frame, and "kernels"
breaks them down. bench.py reads counters_per_dispatch (= per frame) and
hbm_bytes_per_launch (= per frame).

usage: python tools/pmc_summary.py gpurun_out/<tag> <config> [frames=6] > profiles/rNN/pmc_<config>.json
(frames: tools/prof_driver.py renders --iters + 1, all with the specialized kernels)
"""
import csv
import glob
import json
import os
import sys

d, cfg = sys.argv[1], sys.argv[2]
frames = int(sys.argv[3]) if len(sys.argv) > 3 else 6  # tools/prof_driver.py --iters 5 (pmc_session.sh) + 1
RENDER = ("k_render", "rtx_jit_render", "k_split_", "rtx_jit_split_", "k_mesh_chunks")
per = {}  # kernel -> counter -> [values per dispatch]
for f in sorted(glob.glob(os.path.join(d, "p*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if not any(x in k for x in RENDER):
            continue
        per.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
kernels = {}
frame = {}
for k, cs in per.items():
    n = max(len(v) for v in cs.values())
    avg = {c: sum(v) / len(v) for c, v in cs.items()}
    kernels[k] = {"dispatches": n, "per_dispatch": avg}
    for c, v in cs.items():  # this counter's dispatches (one pass each) averaged, times dispatches per frame
        frame[c] = frame.get(c, 0.0) + sum(v) / len(v) * (len(v) / frames)
main = max(kernels, key=lambda k: kernels[k]["per_dispatch"].get("SQ_WAVE_CYCLES", 0) * kernels[k]["dispatches"]) \
    if kernels else None
out = {"config": cfg, "kernel": main, "frames": frames, "counters_per_dispatch": frame,
       "note": "counters_per_dispatch: per frame (every render dispatch of one frame summed)"}
if len(kernels) > 1:
    out["kernels"] = kernels
if "FETCH_SIZE" in frame and "WRITE_SIZE" in frame:
    out["hbm_bytes_per_launch"] = (2 * frame["FETCH_SIZE"] + frame["WRITE_SIZE"]) * 1024
    out["hbm_bytes_note"] = "(2*FETCH_SIZE + WRITE_SIZE) KiB per frame; FETCH doubled per MI355X_MICROARCH.md gfx950 note"
if "SQ_WAVES" in frame and "SQ_INSTS_VALU" in frame:
    out["valu_insts_per_wave"] = frame["SQ_INSTS_VALU"] / frame["SQ_WAVES"]
    out["salu_insts_per_wave"] = frame.get("SQ_INSTS_SALU", 0) / frame["SQ_WAVES"]
print(json.dumps(out, indent=1))
