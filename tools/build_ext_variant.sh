#!/bin/bash
# A librtx.so variant whose hierarchy/texture kernels are built with extra flags (or from
# another source tree: SRC=dir holding csrc/), linked with this tree's build/rtx_api.o, into
# _abl/librtx_<name>.so (tools/ab_lib.sh runs it through RTX_LIB_OVERRIDE).
# usage: tools/build_ext_variant.sh NAME [-D...]
set -eu
cd "$(dirname "$0")/.."
name=$1; shift
src=${SRC:-python-raytracer_amd}
out=_abl/build_$name; mkdir -p $out _abl
flags="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wall"
for t in m0 m1; do /opt/rocm/bin/hipcc $flags "$@" -c -o $out/ext_$t.o $src/csrc/rtx_kern_ext_$t.hip & done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o _abl/librtx_$name.so python-raytracer_amd/build/rtx_api.o \
  $out/ext_m0.o $out/ext_m1.o -lhiprtc
echo "_abl/librtx_$name.so"
