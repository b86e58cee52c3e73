#!/bin/bash
# Round-4 session e: the full GPU suite with the measured tile schedule and split passes
# on by default, then the configs' bench lines (schedule on / off).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04e; mkdir -p $O
export TMPDIR=/tmp
TAG=r04e STEPS="tests smoke" bash tools/session.sh || exit 1
for rep in 1 2; do
  for c in tsp1080 mr1080 tm1080; do
    for v in 1 0; do
      RTX_TILE_SCHED=$v timeout -k 10 200 python bench.py --config $c --steps 100 --warmup 5 --no-cpu-baseline > $O/${c}_ts$v.$rep.json 2> $O/${c}_ts$v.$rep.err || { echo "FAIL $c ts$v"; tail -5 $O/${c}_ts$v.$rep.err; exit 1; }
      python -c "import json;d=json.load(open('$O/${c}_ts$v.$rep.json'));print('$c sched=$v', d['frame_ms'], d['kernel'])"
    done
  done
done
echo SESSION_E_DONE
