#!/bin/bash
# Round-4 session b: wave timelines of the specialized kernels; PMC passes of DepthOfField
# (scratch fix) and NovelScene1 (the CSG kernel's first counter profile).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04b; mkdir -p $O
export TMPDIR=/tmp
for c in tsp1080 mr1080 tm1080 dof4k; do
  fr=2000; [ $c = dof4k ] && fr=40
  timeout -k 10 200 python tools/wave_timeline.py --config $c --frames $fr --json $O/wt_$c.json > $O/wt_$c.log 2>&1 || { echo "wt $c failed"; tail -5 $O/wt_$c.log; exit 1; }
  tail -1 $O/wt_$c.log
done
TAG=r04b STEPS="pmc" CONFIGS="dof4k ns1" bash tools/session.sh
