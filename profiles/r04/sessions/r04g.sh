#!/bin/bash
# Round-4 session g: split-pass occupancy variants (NovelScene1/2) and the split kernels' PMC.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
VARIANTS="base=default;b4=_abl/librtx_b4.so;a5b4=_abl/librtx_a5b4.so;base2=default;b4_2=_abl/librtx_b4.so;a5b4_2=_abl/librtx_a5b4.so" \
  CONFIGS="ns1" STEPS=10 bash tools/ab_lib.sh || exit 1
VARIANTS="base=default;b4=_abl/librtx_b4.so;a5b4=_abl/librtx_a5b4.so" CONFIGS="ns2" STEPS=4 bash tools/ab_lib.sh || exit 1
mkdir -p gpurun_out/r04g && cp gpurun_out/abl/*.json gpurun_out/r04g/
TAG=r04g STEPS="pmc" CONFIGS="ns1" bash tools/session.sh
