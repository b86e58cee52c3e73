#!/bin/bash
# Light grids (shadow rays of point lights against the mesh, rtx_api.hip light_grids):
# exactness tests on the MI355X, then frame times with and without (RTX_LGRID=0).
set -u
mkdir -p gpurun_out/lgrid
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "light_grids or large_mesh or TorusMesh or random_scenes or primary_bins" > gpurun_out/lgrid/tests.log 2>&1 || { tail -30 gpurun_out/lgrid/tests.log; exit 1; }
tail -2 gpurun_out/lgrid/tests.log
run() {  # run TAG CONFIG STEPS [env...]
  local tag=$1 c=$2 st=$3; shift 3
  env "$@" timeout -k 10 200 python bench.py --config $c --steps $st --warmup 3 --no-cpu-baseline \
    > gpurun_out/lgrid/$tag.json 2> gpurun_out/lgrid/$tag.err || { tail gpurun_out/lgrid/$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/lgrid/$tag.json'));print('$tag', d['frame_ms'], d['kernel'])"
}
for c in ${CONFIGS:-tm1080 blob1080}; do
  run ${c}_grid $c 50
  run ${c}_walk $c 50 RTX_LGRID=0
done
