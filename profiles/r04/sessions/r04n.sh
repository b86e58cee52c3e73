#!/bin/bash
# Round-4 session n: host-computed origin terms of primary rays (RTX_PRIM_ORIGIN).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04n; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_refvectors.py tests/test_gpu_jit_cache.py -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/pytest.log; [ $rc = 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
for rep in 1 2; do
  for c in tsp1080 mr1080 tm1080; do
    for v in 1 0; do
      RTX_PRIM_ORIGIN=$v timeout -k 10 200 python bench.py --config $c --steps 200 --warmup 5 --no-cpu-baseline > $O/${c}_po$v.$rep.json 2> $O/${c}_po$v.$rep.err || { echo "FAIL $c po$v"; tail -5 $O/${c}_po$v.$rep.err; exit 1; }
      python -c "import json;d=json.load(open('$O/${c}_po$v.$rep.json'));print('$c prim=$v', d['frame_ms'], d['kernel'])"
    done
  done
done
