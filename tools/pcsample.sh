#!/bin/bash
# PC sampling of the render kernel (host-trap method) for hotspot analysis.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-pcs}
mkdir -p "$OUT"
export TMPDIR=/tmp
rocprofv3 -L > "$OUT/list.txt" 2>&1 || true
grep -i -A3 "pc.sampl" "$OUT/list.txt" | head -40
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method ${METHOD:-host_trap} --pc-sampling-unit ${UNIT:-time} \
  --pc-sampling-interval ${INTERVAL:-1} -d "$OUT/pcs" -o pcs --output-format csv -- python3 tools/prof_driver.py --config ${CFG:-tsp1080} --iters 50 > "$OUT/pcs.log" 2>&1
rc=$?; echo "rc=$rc"; tail -20 "$OUT/pcs.log"; ls -la "$OUT/pcs" 2>/dev/null
