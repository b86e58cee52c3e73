#!/bin/bash
# Round-end check of this tree on a fresh box: GPU parity suite, smoke, default bench
# (with the CPU baselines) and its rocprofv3 kernel statistics.
set -u
OUT=gpurun_out/${TAG:-r02final}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }; tail -3 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench_default.log 2>&1 || { tail $OUT/bench_default.log; exit 1; }; grep '^{' $OUT/bench_default.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > $OUT/rocprof.log 2>&1 || { tail $OUT/rocprof.log; exit 1; }
echo FINAL_OK
