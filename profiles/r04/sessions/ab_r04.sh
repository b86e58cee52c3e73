#!/bin/bash
# Round-4 A/Bs on one box (frame time per variant, interleaved twice): persistent waves
# (RTX_PERSIST = resident waves per SIMD the grid is sized for) on the one-sample configs,
# and MirrorRefraction's occupancy (frame levels in LDS x waves/SIMD bound).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r04ab}; mkdir -p $O
run() {  # run NAME CONFIG [env assignments...]
  local n=$1 c=$2; shift 2
  local st=100; [ $c = dof4k ] && st=10
  env "$@" timeout -k 10 120 python bench.py --config $c --steps $st --warmup 5 --no-cpu-baseline \
    > $O/${c}_$n.json 2> $O/${c}_$n.err || { echo "FAIL $c $n"; tail -5 $O/${c}_$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/${c}_$n.json'));print('$c $n', d['frame_ms'], d['kernel'])"
}
for rep in 1 2; do
  for c in ${PCONFIGS:-tsp1080 mr1080 tm1080}; do
    run base$rep $c
    for w in ${PWAVES:-4 6 8}; do run p$w.$rep $c RTX_PERSIST=$w; done
  done
  run base$rep mr1080
  run l8w6.$rep mr1080 "RTX_JIT_FLAGS=-URTX_LB_WAVES -DRTX_LB_WAVES(MESH,SEC)=6 -DRTX_FRAME_LDS_LEVELS=8"
  run l7w7.$rep mr1080 "RTX_JIT_FLAGS=-URTX_LB_WAVES -DRTX_LB_WAVES(MESH,SEC)=7 -DRTX_FRAME_LDS_LEVELS=7"
done
echo AB_DONE
