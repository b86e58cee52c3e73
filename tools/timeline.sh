#!/bin/bash
# Wave timelines of configs (tools/wave_timeline.py) with the RTX_WAVE_LOG tools library,
# built beforehand: tools/build_lib_variant.sh wavelog -DRTX_WAVE_LOG=1 -DRTX_TOOLS_BUILD.
# CONFIGS as bench.py names them; outputs under gpurun_out/$TAG/wt_<config>.{json,npz}.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-timeline}
mkdir -p "$OUT"
for c in ${CONFIGS:-tsp1080}; do
  RTX_LIB_OVERRIDE=$PWD/_abl/librtx_wavelog.so timeout -k 10 180 python tools/wave_timeline.py --config $c \
    --frames ${FRAMES:-500} --json "$OUT/wt_$c.json" --npz "$OUT/wt_$c.npz" > "$OUT/wt_$c.log" 2>&1 || { tail "$OUT/wt_$c.log"; exit 1; }
  tail -4 "$OUT/wt_$c.log"
done
