#!/bin/bash
# Round-4 session ad: plane self-test skip -- GPU parity, then TSP/MR/TM/DOF frame times
# with and without the self skips (RTX_SELF_SKIP=0), interleaved twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04ad; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_refvectors.py \
  > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do
  for c in tsp1080 mr1080 tm1080 dof4k; do
    st=100; [ $c = dof4k ] && st=10
    for v in skip noskip; do
      e=""; [ $v = noskip ] && e="RTX_SELF_SKIP=0"
      env $e timeout -k 10 200 python bench.py --config $c --steps $st --warmup 3 --no-cpu-baseline \
        > $O/${c}_$v$rep.json 2> $O/${c}_$v$rep.err || { echo FAIL $c $v; tail -5 $O/${c}_$v$rep.err; exit 1; }
      python -c "import json;d=json.load(open('$O/${c}_$v$rep.json'));print('$c $v$rep', d['frame_ms'], d['kernel'])"
    done
  done
done
echo R04AD_DONE
