#!/bin/bash
# Batched interleaved groups: GPU parity suite, smoke, per-rank balance probe, the frame
# loop over one RCCL rank.
set -u
OUT=gpurun_out/${TAG:-r02s15}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }; tail -3 $OUT/smoke.log
timeout -k 10 200 python tools/rank_balance_probe.py > $OUT/rank_balance.log 2>&1 || { tail $OUT/rank_balance.log; exit 1; }; cat $OUT/rank_balance.log
TAG=$(basename $OUT) CONFIGS="tsp1080 dof4k" bash tools/s10_pipeline.sh || exit 1
