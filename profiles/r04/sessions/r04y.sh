#!/bin/bash
# Round-4 session y: cost probe -- shading points on a box skip that box's shadow test
# (RTX_ABLATE=22; not exact by design), DepthOfField 4K, interleaved twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04y; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for v in 0 22; do
    if [ $v = 0 ]; then unset RTX_JIT_FLAGS; else export RTX_JIT_FLAGS="-DRTX_ABLATE=$v"; fi
    timeout -k 10 200 python bench.py --config dof4k --steps 10 --warmup 3 --no-cpu-baseline > $O/dof_a$v.$rep.json 2> $O/dof_a$v.$rep.err || { echo FAIL $v; tail -5 $O/dof_a$v.$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$O/dof_a$v.$rep.json'));print('dof ablate=$v.$rep', d['frame_ms'])"
  done
done
echo R04Y_DONE
