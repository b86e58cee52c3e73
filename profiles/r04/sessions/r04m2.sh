#!/bin/bash
# Round-4 measurement session, part 2: bench lines of every config (with the CPU baselines
# and the PMC summaries of part 1), rocprof kernel statistics per config, the default line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r04m} STEPS="configs rocprof_configs bench rocprof" CONFIGS="${CONFIGS:-tsp1080 mr1080 tm1080 dof4k ns1 ns2 blob1080}" BSTEPS=20 bash tools/session.sh
