#!/bin/bash
# Round-4 session t: primary-ray bins of hierarchy roots and moving objects, shadow grids
# with hierarchy roots (both per camera) -- parity, then frame times with both, without the
# bins (RTX_BINS=0) and without the shadow grids (RTX_DSGRID=0), interleaved twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04t; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_split.py \
  -k "dir_shadow or bins or random or philox_frames or split" > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for rep in 1 2; do
  for c in ${CONFIGS:-ns1 ns2 dof4k mr1080}; do
    st=100; [ $c = dof4k ] && st=10; [ $c = ns1 ] && st=5; [ $c = ns2 ] && st=3
    for v in all nobins nogrid; do
      e=""; [ $v = nobins ] && e="RTX_BINS=0"; [ $v = nogrid ] && e="RTX_DSGRID=0"
      env $e timeout -k 10 200 python bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline \
        > $O/${c}_$v$rep.json 2> $O/${c}_$v$rep.err || { echo FAIL $c $v; tail -5 $O/${c}_$v$rep.err; exit 1; }
      python -c "import json;d=json.load(open('$O/${c}_$v$rep.json'));print('$c $v$rep', d['frame_ms'], d['kernel'])"
    done
  done
done
echo R04T_DONE
