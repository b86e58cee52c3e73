#!/bin/bash
# Register / scratch / SGPR-spill report of the hierarchy/texture kernels (MESH = false TU)
# and their out-of-line helpers, compiled offline. usage: tools/ext_ru.sh [FILTER] [-D...]
set -eu
cd "$(dirname "$0")/../python-raytracer_amd/csrc"
f=${1:-.}; shift || true
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC --cuda-device-only "$@" -c \
  -Rpass-analysis=kernel-resource-usage -o /tmp/rtx_ext_ru.o rtx_kern_ext_m0.hip 2>&1 |
  grep -oE "(Function Name: \S+|VGPRs: [0-9]+|ScratchSize \[bytes/lane\]: [0-9]+|SGPRs Spill: [0-9]+|Occupancy \[waves/SIMD\]: [0-9]+)" |
  awk '/Function Name/{if(l)print l; l=$3; next}{l=l" "$0}END{print l}' | c++filt | grep -E -- "$f" | sed -E 's/\(rtx::[^)]*\)//' | cut -c1-200
rm -f /tmp/rtx_ext_ru.o
