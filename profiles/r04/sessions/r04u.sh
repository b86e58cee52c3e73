#!/bin/bash
# Round-4 session u: shadow grids only where they pay (no grid for a few spheres alone):
# parity, MirrorRefraction frame time with the default and with RTX_DSGRID_MIN=1, then the
# DepthOfField 4K cost probes (tools/r04s.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04u; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_parity.py \
  -k "dir_shadow or config_size" > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do
  for v in default grid; do
    e=""; [ $v = grid ] && e="RTX_DSGRID_MIN=1"
    env $e timeout -k 10 200 python bench.py --config mr1080 --steps 100 --warmup 3 --no-cpu-baseline \
      > $O/mr1080_$v$rep.json 2> $O/mr1080_$v$rep.err || { echo FAIL $v; tail -5 $O/mr1080_$v$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$O/mr1080_$v$rep.json'));print('mr1080 $v$rep', d['frame_ms'], d['kernel'])"
  done
done
bash tools/r04s.sh
