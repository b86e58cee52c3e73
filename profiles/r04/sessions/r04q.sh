#!/bin/bash
# Round-4 session q: lens cameras' thick primary-ray bins -- parity, then DepthOfField 4K
# frame time with and without them (interleaved twice).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04q; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py \
  -k "lens_bins or philox or primary_bins" > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for rep in 1 2; do
  for v in lens nolens; do
    e=""; [ $v = nolens ] && e="RTX_LENS_BINS=0"
    env $e timeout -k 10 200 python bench.py --config dof4k --steps 10 --warmup 3 --no-cpu-baseline \
      > $O/dof_$v$rep.json 2> $O/dof_$v$rep.err || { echo FAIL $v; tail -5 $O/dof_$v$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$O/dof_$v$rep.json'));print('dof $v$rep', d['frame_ms'], d['kernel'])"
  done
done
echo R04Q_DONE
