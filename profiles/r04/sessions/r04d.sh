#!/bin/bash
# Round-4 session d: measured longest-first tile orders (wave timeline -> order -> A/B).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04d; mkdir -p $O
export TMPDIR=/tmp
for c in ${CFGS:-tsp1080 mr1080 tm1080 dof4k}; do
  fr=2000; [ $c = dof4k ] && fr=40
  timeout -k 10 200 python tools/wave_timeline.py --config $c --frames $fr --json $O/wt_$c.json --npz $O/wt_$c.npz > $O/wt_$c.log 2>&1 || { echo "wt $c failed"; tail -5 $O/wt_$c.log; exit 1; }
  python tools/tile_order.py order $O/wt_$c.npz $O/order_$c.bin --sim || exit 1
  timeout -k 10 200 python tools/tile_order.py check $c $O/order_$c.bin > $O/check_$c.log 2>&1 || { echo "check $c failed"; tail -5 $O/check_$c.log; exit 1; }
  tail -1 $O/check_$c.log
done
for rep in 1 2; do
  for c in ${CFGS:-tsp1080 mr1080 tm1080 dof4k}; do
    st=100; [ $c = dof4k ] && st=10
    for v in 0 1; do
      if [ $v = 1 ]; then export RTX_TILE_PERM_FILE=$O/order_$c.bin; else unset RTX_TILE_PERM_FILE; fi
      timeout -k 10 200 python bench.py --config $c --steps $st --warmup 5 --no-cpu-baseline > $O/${c}_p$v.$rep.json 2> $O/${c}_p$v.$rep.err || { echo "FAIL $c p$v"; tail -5 $O/${c}_p$v.$rep.err; exit 1; }
      python -c "import json;d=json.load(open('$O/${c}_p$v.$rep.json'));print('$c perm=$v', d['frame_ms'], d['kernel'])"
    done
  done
done
unset RTX_TILE_PERM_FILE
echo SESSION_D_DONE
