#!/bin/bash
# GPU: per-launch fixed cost (tools/launch_probe.py) per library variant (LIBS="name=path ...")
set -u
O=gpurun_out/${TAG:-probe}; mkdir -p $O
export TMPDIR=/tmp
for v in ${LIBS:-default=default}; do
  n=${v%%=*}; l=${v#*=}
  if [ "$l" = default ]; then unset RTX_LIB_OVERRIDE; else export RTX_LIB_OVERRIDE=$PWD/$l; fi
  echo "== $n"; timeout -k 10 200 python tools/launch_probe.py ${PCONFIGS:-tsp1080} > $O/probe_$n.log 2>&1 || { tail -3 $O/probe_$n.log; exit 1; }
  grep us $O/probe_$n.log
done
