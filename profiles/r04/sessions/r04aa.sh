#!/bin/bash
# Round-4 session aa: box self-test skip -- parity (shadow grids, Philox DOF frames, full
# 4K frame with and without grids), then DepthOfField 4K with and without the skip
# (RTX_SELF_SKIP=0), interleaved twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04aa; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py \
  -k "dir_shadow or philox or lens_bins or random or box" > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do
  for v in skip noskip; do
    e=""; [ $v = noskip ] && e="RTX_SELF_SKIP=0"
    env $e timeout -k 10 200 python bench.py --config dof4k --steps 10 --warmup 3 --no-cpu-baseline \
      > $O/dof4k_$v$rep.json 2> $O/dof4k_$v$rep.err || { echo FAIL $v; tail -5 $O/dof4k_$v$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$O/dof4k_$v$rep.json'));print('dof4k $v$rep', d['frame_ms'], d['kernel'])"
  done
done
echo R04AA_DONE
