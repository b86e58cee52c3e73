#!/bin/bash
# Round-4 session k: DepthOfField 4K cost probes (RTX_ABLATE, results not exact by design).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04k; mkdir -p $O
export TMPDIR=/tmp
for v in 0 7 17 19 20 21 15 0; do
  if [ $v = 0 ]; then unset RTX_JIT_FLAGS; else export RTX_JIT_FLAGS="-DRTX_ABLATE=$v"; fi
  timeout -k 10 200 python bench.py --config dof4k --steps 10 --warmup 3 --no-cpu-baseline > $O/dof_a$v.json 2> $O/dof_a$v.err || { echo FAIL $v; tail -5 $O/dof_a$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/dof_a$v.json'));print('dof ablate=$v', d['frame_ms'])"
done
