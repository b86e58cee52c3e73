#!/bin/bash
# Builds the wavefront experiment into _abl/librtx_wf.so (CPU side; travels with gpurun).
set -eu
cd "$(dirname "$0")/../.."
make -s -C python-raytracer_amd python-raytracer_amd/csrc/rtx_jit_sources.inc 2>/dev/null || make -s -C python-raytracer_amd csrc/rtx_jit_sources.inc
mkdir -p _abl
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -o _abl/librtx_wf.so \
  tools/wavefront/rtx_wavefront.hip python-raytracer_amd/csrc/rtx_kern_ext_m0.hip python-raytracer_amd/csrc/rtx_kern_ext_m1.hip -lhiprtc
