#!/bin/bash
# Batched-frames check: GPU parity suite (incl. rtx_render_frames), smoke, the group-render
# probe, the frame loop over one RCCL rank and the default bench.
set -u
OUT=gpurun_out/${TAG:-r02s13}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }; tail -3 $OUT/smoke.log
timeout -k 10 200 python tools/group_graph_probe.py > $OUT/group_graph_probe.log 2>&1 || { tail $OUT/group_graph_probe.log; exit 1; }; cat $OUT/group_graph_probe.log
TAG=$(basename $OUT) CONFIGS="tsp1080 dof4k" bash tools/s10_pipeline.sh || exit 1
timeout -k 10 300 python bench.py > $OUT/bench_default.log 2>&1 || { tail $OUT/bench_default.log; exit 1; }; grep '^{' $OUT/bench_default.log | cut -c1-300
