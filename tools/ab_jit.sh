#!/bin/bash
# A/B of scene-specialized kernel variants without rebuilding librtx: each variant is
# "name|hiprtc flags" (RTX_JIT_FLAGS, appended after the library's forwarded macros, so
# -D overrides win). usage: CONFIGS="tm1080" VARIANTS="base|;noshadow|-DRTX_ABLATE=1" bash tools/ab_jit.sh
# Ablation variants are cost probes, not parity-correct.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-abjit}
mkdir -p "$OUT"
IFS=';' read -ra VS <<< "${VARIANTS:-base|}"
for c in ${CONFIGS:-tsp1080}; do
  st=50; [ $c = dof4k ] && st=10
  for v in "${VS[@]}"; do
    name=${v%%|*}; flags=${v#*|}
    RTX_JIT_FLAGS="$flags" timeout -k 10 120 python bench.py --config $c --steps $st --warmup 3 --no-cpu-baseline > "$OUT/${c}_$name.json" 2> "$OUT/${c}_$name.err" || { tail -5 "$OUT/${c}_$name.err"; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/${c}_$name.json')); print('%-8s %-12s %9.2f us  %s' % ('$c', '$name', d['frame_ms']*1e3, d['kernel']))"
  done
done
