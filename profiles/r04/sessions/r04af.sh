#!/bin/bash
# Round-4 session af: plane self tests with the per-call check gated on a wave vote --
# MirrorRefraction with them (RTX_SELF_SKIP=2) and without, TSP and TM default vs off.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04af; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py \
  -k "config_size or random or counters" > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for cv in mr1080:2 mr1080:0 tsp1080:1 tsp1080:0 tm1080:1 tm1080:0; do
    c=${cv%%:*}; v=${cv#*:}
    RTX_SELF_SKIP=$v timeout -k 10 200 python bench.py --config $c --steps 100 --warmup 3 --no-cpu-baseline \
      > $O/${c}_s$v.$rep.json 2> $O/${c}_s$v.$rep.err || { echo FAIL $c $v; tail -5 $O/${c}_s$v.$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$O/${c}_s$v.$rep.json'));print('$c self=$v.$rep', d['frame_ms'])"
  done
done
echo R04AF_DONE
