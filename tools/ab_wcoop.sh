#!/bin/bash
# Wave-cooperative large-mesh variant (-DRTX_WCOOP=1: one ray per wave, faces across
# lanes) against the default one-ray-per-lane kernel: exactness tests, then frame times
# of the 81,920-face blob at 1080p (binned primaries, and the BVH walk with RTX_BINS=0)
# and TorusMesh with every mesh on the cooperative path.
set -u
mkdir -p gpurun_out/wcoop
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "wave_cooperative or large_mesh" > gpurun_out/wcoop/tests.log 2>&1 || { tail -30 gpurun_out/wcoop/tests.log; exit 1; }
tail -2 gpurun_out/wcoop/tests.log
run() {  # run TAG CONFIG STEPS [env...]
  local tag=$1 c=$2 st=$3; shift 3
  env "$@" timeout -k 10 200 python bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline \
    > gpurun_out/wcoop/$tag.json 2> gpurun_out/wcoop/$tag.err || { tail gpurun_out/wcoop/$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/wcoop/$tag.json'));print('$tag', d['frame_ms'], d['kernel'])"
}
run blob_lane blob1080 20
run blob_coop blob1080 20 RTX_JIT_FLAGS=-DRTX_WCOOP=1
run blob_walk_lane blob1080 20 RTX_BINS=0
run blob_walk_coop blob1080 20 RTX_BINS=0 RTX_JIT_FLAGS=-DRTX_WCOOP=1
run tm_lane tm1080 50
run tm_coop tm1080 50 "RTX_JIT_FLAGS=-DRTX_WCOOP=1 -DRTX_WCOOP_MIN=1"
