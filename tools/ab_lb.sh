#!/bin/bash
# Occupancy-bound A/B of the scene-specialized kernels: RTX_JIT_FLAGS overrides the
# forwarded RTX_LB_WAVES per run (bench frame_ms, DOF 4K and the 1-spp configs).
set -u
mkdir -p gpurun_out/lb
for c in ${CONFIGS:-dof4k tsp1080 tm1080 mr1080}; do
  for w in ${WAVES:-5 4 3}; do
    st=50; [ $c = dof4k ] && st=10
    RTX_JIT_FLAGS="-DRTX_LB_WAVES(M,S)=$w" timeout -k 10 120 python bench.py --config $c --steps $st --warmup 3 --no-cpu-baseline > gpurun_out/lb/${c}_w$w.json 2>gpurun_out/lb/${c}_w$w.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/lb/${c}_w$w.json'));print('$c waves=$w', d['frame_ms'], d['kernel'])"
  done
done
