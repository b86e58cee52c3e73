#!/bin/bash
# Round-4: PC sampling (rocprofv3 beta, host trap) of the TwoSpheresPlane kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04p; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
  --pc-sampling-interval 1 -d $O/pcs -o pcs --output-format csv -- python3 tools/prof_driver.py --config tsp1080 --iters 3000 > $O/pcs.log 2>&1
echo "rc=$?"; tail -5 $O/pcs.log; find $O/pcs -type f | head; mkdir -p $O/co; cp /tmp/rtx_jit_$(id -u)/*.co $O/co/ 2>/dev/null; ls $O/co | head
