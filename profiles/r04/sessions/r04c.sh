#!/bin/bash
# Round-4 session c: the split hierarchy passes (tests, NovelScene A/B), then session b.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_jit_cache.py -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > $O/pytest_split.log 2>&1
rc=$?; echo "split tests rc=$rc"; tail -5 $O/pytest_split.log; [ $rc = 0 ] || exit 1
for rep in 1 2; do
  for c in ns1 ns2; do
    st=10; [ $c = ns2 ] && st=4
    for v in 0 1; do
      RTX_SPLIT=$v timeout -k 10 300 python bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline > $O/${c}_s$v.$rep.json 2> $O/${c}_s$v.$rep.err || { echo "FAIL $c $v"; tail -5 $O/${c}_s$v.$rep.err; exit 1; }
      python -c "import json;d=json.load(open('$O/${c}_s$v.$rep.json'));print('$c split=$v', d['frame_ms'], d['kernel'])"
    done
  done
done
for rep in 1 2; do
  for c in tsp1080 mr1080 tm1080; do
    for v in 0 1; do
      RTX_KP_BYVAL=$v timeout -k 10 120 python bench.py --config $c --steps 100 --warmup 5 --no-cpu-baseline > $O/${c}_kv$v.$rep.json 2> $O/${c}_kv$v.$rep.err || { echo "FAIL $c kv$v"; tail -5 $O/${c}_kv$v.$rep.err; exit 1; }
      python -c "import json;d=json.load(open('$O/${c}_kv$v.$rep.json'));print('$c byval=$v', d['frame_ms'], d['kernel'])"
    done
  done
done
bash tools/r04b.sh
