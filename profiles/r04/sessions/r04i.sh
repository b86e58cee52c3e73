#!/bin/bash
# Round-4 session i: raised issue priority for deep reflect/refract chains (MR), and the
# split kernels' counters (NovelScene1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04i; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for v in none 1 2 3; do
    if [ $v = none ]; then unset RTX_JIT_FLAGS; else export RTX_JIT_FLAGS="-DRTX_DEEP_PRIO=$v"; fi
    timeout -k 10 200 python bench.py --config mr1080 --steps 100 --warmup 5 --no-cpu-baseline > $O/mr_p$v.$rep.json 2> $O/mr_p$v.$rep.err || { echo FAIL; tail -5 $O/mr_p$v.$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$O/mr_p$v.$rep.json'));print('mr prio=$v', d['frame_ms'], d['kernel'])"
  done
done
unset RTX_JIT_FLAGS
TAG=r04i STEPS="pmc" CONFIGS="ns1" bash tools/session.sh
