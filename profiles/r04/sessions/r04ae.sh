#!/bin/bash
# Round-4 session ae (final numbers): PMC passes of every config, then the bench lines with
# those counts (copied into profiles/ on the box first), rocprof statistics, the default
# line, the full GPU suite and smoke.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
C="tsp1080 mr1080 tm1080 dof4k ns1 ns2 blob1080"
TAG=r04ae STEPS="pmc" CONFIGS="$C" bash tools/session.sh || exit 1
for c in $C; do cp gpurun_out/r04ae/pmc_$c.json profiles/pmc_$c.json; done
TAG=r04ae STEPS="configs rocprof_configs bench rocprof tests smoke" CONFIGS="$C" BSTEPS=20 bash tools/session.sh
