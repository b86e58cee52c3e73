#!/bin/bash
# Frame time per environment variant: VARIANTS="name=VAR=val VAR2=val;name2=..." (empty:
# defaults), CONFIGS as bench.py names them.
set -u
mkdir -p gpurun_out/abe
IFS=';' read -ra VS <<< "${VARIANTS:-base=}"
for c in ${CONFIGS:-tm1080}; do
  st=50; [ $c = dof4k ] && st=10
  for v in "${VS[@]}"; do
    n=${v%%=*}; e=${v#*=}
    env $e timeout -k 10 120 python bench.py --config $c --steps $st --warmup 3 --no-cpu-baseline \
      > gpurun_out/abe/${c}_$n.json 2> gpurun_out/abe/${c}_$n.err || { tail -5 gpurun_out/abe/${c}_$n.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/abe/${c}_$n.json'));print('$c $n', d['frame_ms'], d['kernel'])"
  done
done
