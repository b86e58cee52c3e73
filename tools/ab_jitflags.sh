#!/bin/bash
# Frame time per scene-specialized kernel variant without rebuilding the library:
# VARIANTS="name=flags;name=flags" (flags go to the jit_flags option, RTX_JIT_FLAGS, e.g.
# "-URTX_ABLATE -DRTX_ABLATE=1"); CONFIGS as bench.py names them. Cost probes (RTX_ABLATE)
# exist only in a tools build of the library: TOOLS_LIB (default _abl/librtx_tools.so,
# built by `tools/build_lib_variant.sh tools -DRTX_TOOLS_BUILD`) is used when present.
set -u
mkdir -p gpurun_out/abj
TL=${TOOLS_LIB:-_abl/librtx_tools.so}
[ -f "$TL" ] && export RTX_LIB_OVERRIDE=$PWD/$TL
IFS=';' read -ra VS <<< "${VARIANTS:-base=}"
for c in ${CONFIGS:-tsp1080 tm1080}; do
  st=50; [ $c = dof4k ] && st=10
  for v in "${VS[@]}"; do
    n=${v%%=*}; f=${v#*=}
    RTX_JIT_FLAGS="$f" timeout -k 10 120 python bench.py --config $c --steps $st --warmup 3 --no-cpu-baseline \
      > gpurun_out/abj/${c}_$n.json 2> gpurun_out/abj/${c}_$n.err || { tail -5 gpurun_out/abj/${c}_$n.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/abj/${c}_$n.json'));print('$c $n', d['frame_ms'], d['kernel'])"
  done
done
