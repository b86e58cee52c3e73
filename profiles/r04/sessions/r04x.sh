#!/bin/bash
# Round-4 session x: the split passes at 2^28-record chunks -- split parity tests, then the
# NovelScene1/2 bench lines and kernel statistics.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r04x STEPS="tests configs rocprof_configs" TESTS="tests/test_gpu_split.py tests/test_gpu_parity.py" \
  KEXPR="split or hier or novel or Novel" CONFIGS="ns1 ns2" BSTEPS=10 bash tools/session.sh
