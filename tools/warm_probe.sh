#!/bin/bash
# Frame time against warm-up length and timed length (GPU clock ramp?), default N = 1 bench.
set -u
O=gpurun_out/${TAG:-warm_probe}; mkdir -p $O
export TMPDIR=/tmp
c=${CFG:-tsp1080}
for v in "10 100" "4000 100" "10 4000" "4000 4000"; do
  set -- $v
  timeout -k 10 200 python bench.py --config $c --steps $2 --warmup $1 --no-cpu-baseline > $O/w$1_s$2.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads([l for l in open('$O/w$1_s$2.log') if l.startswith('{')][0]); print('warmup $1 steps $2', d['frame_ms'], d['ms_per_step'])"
done
