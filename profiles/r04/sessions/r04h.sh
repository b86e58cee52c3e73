#!/bin/bash
# Round-4 session h: hierarchy tests after the wave-uniform traversal indices and the
# surface-free shadow enumerations; NovelScene1/2 split vs one-kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04h; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py tests/test_gpu_refvectors.py -x -q -p no:cacheprovider \
  -k "split or hier or Novel or novel or box or kat or refvector or render_" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/pytest.log; [ $rc = 0 ] || exit 1
for rep in 1 2; do
  for c in ns1 ns2; do
    st=10; [ $c = ns2 ] && st=4
    for v in 1 0; do
      RTX_SPLIT=$v timeout -k 10 300 python bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline > $O/${c}_s$v.$rep.json 2> $O/${c}_s$v.$rep.err || { echo "FAIL $c $v"; tail -5 $O/${c}_s$v.$rep.err; exit 1; }
      python -c "import json;d=json.load(open('$O/${c}_s$v.$rep.json'));print('$c split=$v', d['frame_ms'], d['kernel'])"
    done
  done
done
TAG=r04h STEPS="rocprof_configs" CONFIGS="ns1" bash tools/session.sh > $O/rocprof.log 2>&1
python - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/r04h/ns1_kernel_stats.csv')):
    print('%-50s %5s calls avg %9.1f us' % (r['Name'][:50], r['Calls'], float(r['AverageNs']) / 1e3))
PY
