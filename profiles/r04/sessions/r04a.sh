#!/bin/bash
# Round-4 first GPU session: tests, smoke, default bench, rocprof, persistent-wave parity, A/Bs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r04a STEPS="tests smoke bench rocprof" bash tools/session.sh || exit 1
RTX_PERSIST=6 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider \
  -k "config_size_1080p or render_matches_oracle or philox or interleaved or render_frames" \
  --timeout 120 --timeout-method thread > gpurun_out/r04a/persist_tests.log 2>&1
echo "persist tests rc=$?"; tail -2 gpurun_out/r04a/persist_tests.log
TAG=r04a/ab bash tools/ab_r04.sh > gpurun_out/r04a/ab.log 2>&1; echo "ab rc=$?"; cat gpurun_out/r04a/ab.log
TAG=r04a STEPS="configs" CONFIGS="dof4k" CPU=0 bash tools/session.sh
