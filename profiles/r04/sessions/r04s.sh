#!/bin/bash
# Round-4 session s: DepthOfField 4K cost probes after the lens bins and shadow grids
# (RTX_ABLATE, results not exact by design), and its PMC counters.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04s; mkdir -p $O
export TMPDIR=/tmp
for v in 0 8 15 1 3 5 17 20 19 0; do
  if [ $v = 0 ]; then unset RTX_JIT_FLAGS; else export RTX_JIT_FLAGS="-DRTX_ABLATE=$v"; fi
  timeout -k 10 200 python bench.py --config dof4k --steps 10 --warmup 3 --no-cpu-baseline > $O/dof_a$v.json 2> $O/dof_a$v.err || { echo FAIL $v; tail -5 $O/dof_a$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/dof_a$v.json'));print('dof ablate=$v', d['frame_ms'])"
done
unset RTX_JIT_FLAGS
for v in 10 0; do
  if [ $v = 0 ]; then unset RTX_JIT_FLAGS; else export RTX_JIT_FLAGS="-DRTX_ABLATE=$v"; fi
  timeout -k 10 200 python bench.py --config ns1 --steps 5 --warmup 2 --no-cpu-baseline > $O/ns1_a$v.json 2> $O/ns1_a$v.err || { echo FAIL ns1 $v; tail -5 $O/ns1_a$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/ns1_a$v.json'));print('ns1 ablate=$v', d['frame_ms'])"
done
echo R04S_DONE
