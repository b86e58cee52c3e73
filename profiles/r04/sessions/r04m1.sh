#!/bin/bash
# Round-4 measurement session, part 1: the GPU suite, smoke, and PMC passes of every config.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r04m} STEPS="tests smoke pmc" CONFIGS="tsp1080 mr1080 tm1080 dof4k ns1 ns2 blob1080" bash tools/session.sh
