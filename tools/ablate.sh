#!/bin/bash
# Build ablation variants of librtx.so (RTX_ABLATE=1: no shadow tests; 2: no lighting;
# 3: no shading math after the shadow test) and time each on the bench configs.
# Experiment only: results are not parity-correct for N != 0.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ablate}
# ABL_DIR: where the variant libraries live; with PREBUILT=1 they were built beforehand
# (on the CPU container, inside the tree so they travel) and are not rebuilt here
ABL_DIR=${ABL_DIR:-/tmp/rtx_ablate}
mkdir -p "$OUT" "$ABL_DIR"
# VARIANTS: names; FLAGS_<name> gives its hipcc -D flags (default: -DRTX_ABLATE=<name>);
# FLAGS_<name>=none: the built library as is; JFLAGS_<name>: extra flags for the
# scene-specialized (hiprtc) kernels
for n in ${VARIANTS:-0 1 2 3}; do
  fl_var="FLAGS_$n"; fl="${!fl_var:--DRTX_TOOLS_BUILD -DRTX_ABLATE=$n}"
  if [ "$fl" = "none" ]; then cp python-raytracer_amd/rtx/_lib/librtx.so "$ABL_DIR/librtx_$n.so"; continue; fi
  if [ -n "${PREBUILT:-}" ] && [ -f "$ABL_DIR/librtx_$n.so" ]; then continue; fi
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared $fl \
    -o "$ABL_DIR/librtx_$n.so" python-raytracer_amd/csrc/rtx_api.hip python-raytracer_amd/csrc/rtx_kern_ext_m0.hip python-raytracer_amd/csrc/rtx_kern_ext_m1.hip -lhiprtc || exit 1
done
for n in ${VARIANTS:-0 1 2 3}; do
  for c in ${CONFIGS:-tsp1080}; do
    jf_var="JFLAGS_$n"
    env_var="ENV_$n"  # ENV_<name>: extra VAR=value settings for this variant
    env ${!env_var:-} RTX_JIT_FLAGS="${!jf_var:-}" RTX_LIB_OVERRIDE="$ABL_DIR/librtx_$n.so" timeout -k 10 120 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/v${n}_$c.log" 2>&1 || exit 1
    echo "variant $n $c $(python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/v${n}_$c.log') if l.startswith('{')][0]); print('frame_ms', d['frame_ms'])")"
  done
done
