#!/bin/bash
# Round-4 session j: the stackless shade pass (prev links).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04j; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/pytest.log; [ $rc = 0 ] || exit 1
for rep in 1 2; do
  for c in ns1 ns2; do
    st=10; [ $c = ns2 ] && st=4
    timeout -k 10 300 python bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline > $O/${c}.$rep.json 2> $O/${c}.$rep.err || { echo "FAIL $c"; tail -5 $O/${c}.$rep.err; exit 1; }
    python -c "import json;d=json.load(open('$O/${c}.$rep.json'));print('$c', d['frame_ms'], d['kernel'])"
  done
done
TAG=r04j STEPS="rocprof_configs" CONFIGS="ns1" bash tools/session.sh > $O/rocprof.log 2>&1
python - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/r04j/ns1_kernel_stats.csv')):
    print('%-50s %5s calls avg %9.1f us' % (r['Name'][:50], r['Calls'], float(r['AverageNs']) / 1e3))
PY
