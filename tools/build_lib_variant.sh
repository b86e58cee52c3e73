#!/bin/bash
# A whole librtx.so built with extra -D flags (they reach the hiprtc kernels through the
# forwarded library macros), into ${ABL:-_abl}/librtx_<name>.so (_abl/ is not uploaded to the
# GPU box: ABL=_abv for a variant an A/B session loads). usage: tools/build_lib_variant.sh NAME [-D...]
set -eu
cd "$(dirname "$0")/../python-raytracer_amd"
name=$1; shift
abl=${ABL:-_abl}
out=../$abl/build_$name; mkdir -p $out
make -s csrc/rtx_jit_sources.inc
flags="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -fPIC -Wall"
for t in rtx_api rtx_kern_ext_m0 rtx_kern_ext_m1 rtx_bins; do /opt/rocm/bin/hipcc $flags "$@" -c -o $out/$t.o csrc/$t.hip & done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../$abl/librtx_$name.so $out/*.o -lhiprtc
rm -rf $out
echo "$abl/librtx_$name.so"
