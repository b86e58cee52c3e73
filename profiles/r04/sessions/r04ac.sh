#!/bin/bash
# Round-4 session ac: cost probe -- camera hits on a plane skip that plane's shadow test
# (RTX_ABLATE=23, wave-level; not exact by design): DepthOfField 4K, TSP, MR.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04ac; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for c in dof4k tsp1080 mr1080; do
    st=100; [ $c = dof4k ] && st=10
    for v in 0 23; do
      if [ $v = 0 ]; then unset RTX_JIT_FLAGS; else export RTX_JIT_FLAGS="-DRTX_ABLATE=$v"; fi
      timeout -k 10 200 python bench.py --config $c --steps $st --warmup 3 --no-cpu-baseline > $O/${c}_a$v.$rep.json 2> $O/${c}_a$v.$rep.err || { echo FAIL $c $v; tail -5 $O/${c}_a$v.$rep.err; exit 1; }
      python -c "import json;d=json.load(open('$O/${c}_a$v.$rep.json'));print('$c ablate=$v.$rep', d['frame_ms'])"
    done
  done
done
echo R04AC_DONE
