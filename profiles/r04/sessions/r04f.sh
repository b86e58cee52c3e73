#!/bin/bash
# Round-4 session f: kernel statistics of the split passes (NovelScene1/2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r04f STEPS="rocprof_configs" CONFIGS="ns1 ns2" bash tools/session.sh || exit 1
for c in ns1 ns2; do echo "== $c"; cat gpurun_out/r04f/${c}_kernel_stats.csv | cut -d, -f1-4 | head -8; done
