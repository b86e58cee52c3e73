#!/bin/bash
# Frame time per library variant (built beforehand into _abl/, e.g. with other -D knobs):
# VARIANTS="name=_abl/librtx_x.so;name2=default", CONFIGS as bench.py names them.
set -u
mkdir -p gpurun_out/abl
IFS=';' read -ra VS <<< "${VARIANTS:-default=default}"
for c in ${CONFIGS:-ns1}; do
  st=${STEPS:-10}
  for v in "${VS[@]}"; do
    n=${v%%=*}; l=${v#*=}
    if [ "$l" = default ]; then unset RTX_LIB_OVERRIDE; else export RTX_LIB_OVERRIDE=$PWD/$l; fi
    timeout -k 10 200 python bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline \
      > gpurun_out/abl/${c}_$n.json 2> gpurun_out/abl/${c}_$n.err || { tail -5 gpurun_out/abl/${c}_$n.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/abl/${c}_$n.json'));print('$c $n', d['frame_ms'], d['kernel'])"
  done
done
