#!/bin/bash
# Block-size A/B with matching kernels: each variant library is built with
# -DRTX_BLOCK_FLAT=<n> (host launch geometry) and forwards that macro to the
# scene-specialized hiprtc kernels, so the launched kernel and the grid agree.
# Build the variants first (CPU side):
#   hipcc <Makefile HIPFLAGS> -shared -DRTX_BLOCK_FLAT=<n> -o _abl/librtx_blk<n>.so \
#     csrc/rtx_api.hip csrc/rtx_kern_ext_m0.hip csrc/rtx_kern_ext_m1.hip -lhiprtc
set -u
mkdir -p gpurun_out/blk
for c in ${CONFIGS:-tsp1080 tm1080 mr1080 dof4k}; do
  st=50; [ $c = dof4k ] && st=10
  for v in default ${BLOCKS:-64 128}; do
    if [ $v = default ]; then unset RTX_LIB_OVERRIDE; else export RTX_LIB_OVERRIDE=$PWD/_abl/librtx_blk$v.so; fi
    timeout -k 10 120 python bench.py --config $c --steps $st --warmup 3 --no-cpu-baseline \
      > gpurun_out/blk/${c}_$v.json 2> gpurun_out/blk/${c}_$v.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/blk/${c}_$v.json'));print('$c block=$v', d['frame_ms'], d['kernel'])"
  done
done
