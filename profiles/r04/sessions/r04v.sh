#!/bin/bash
# Round-4 session v: shadow-grid resolution (GS, default 256 512 1024) (RTX_DSGRID_G) on DepthOfField 4K and
# NovelScene1/2, interleaved twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04v; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for c in dof4k ns1 ns2; do
    st=10; [ $c = ns1 ] && st=5; [ $c = ns2 ] && st=2
    for g in ${GS:-256 512 1024}; do
      RTX_DSGRID_G=$g timeout -k 10 200 python bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline \
        > $O/${c}_g$g.$rep.json 2> $O/${c}_g$g.$rep.err || { echo FAIL $c $g; tail -5 $O/${c}_g$g.$rep.err; exit 1; }
      python -c "import json;d=json.load(open('$O/${c}_g$g.$rep.json'));print('$c G=$g.$rep', d['frame_ms'])"
    done
  done
done
echo R04V_DONE
