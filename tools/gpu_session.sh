#!/bin/bash
# One GPU session: smoke, GPU tests, PMC counters (tsp1080), bench (with measured
# traffic), extra configs, rocprofv3 kernel trace. Every GPU step has its own time limit;
# the script stops at the first fault/abort/timeout (pytest: exit >= 2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-s1}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name" ; date
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -3 "$OUT/$name.log"
  return $rc
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
if [ -z "${SKIP_TESTS:-}" ]; then
  step pytest_gpu 600 python -m pytest tests -m gpu -q -rf -p no:cacheprovider
  rc=$?; [ $rc -le 1 ] || exit $rc
fi
TAG=$(basename "$OUT")/pmc bash tools/pmc_session.sh > "$OUT/pmc.log" 2>&1 || { tail "$OUT/pmc.log"; exit 1; }
python tools/pmc_summary.py "$OUT/pmc" tsp1080 > "$OUT/pmc_tsp1080.json"
step bench 300 python bench.py --steps 50 --warmup 10 --cpu-seconds ${CPU_SECONDS:-10} --pmc-json "$OUT/pmc_tsp1080.json" || exit 1
for c in ${CONFIGS:-}; do
  step bench_$c 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline || exit 1
done
step rocprof 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --pmc-json "$OUT/pmc_tsp1080.json" || exit 1
echo ALL_DONE
