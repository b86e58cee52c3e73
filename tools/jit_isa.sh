#!/bin/bash
# ISA of a scene-specialized kernel, compiled offline with the options hiprtc gets (see
# tools/jit_resource.sh). usage: tools/jit_isa.sh "<mesh> <sec> <ext> <cnt> <jit>" out.s [-D...]
set -eu
cd "$(dirname "$0")/.."
read -r M S X C J <<< "$1"; out=$2; shift 2
b() { [ "$1" = 1 ] && echo true || echo false; }
src=$(mktemp /tmp/rtx_jit_XXXX.hip)
cat > "$src" <<SRC
#include "$(pwd)/python-raytracer_amd/csrc/rtx_kernels.h"
extern "C" __global__ RTX_RENDER_BOUNDS($(b $M), $(b $S), $(b $X)) void rtx_jit_render(const rtx::KParams* __restrict__ P, const rtx::Launch L) {
  rtx::render_body<$(b $M), $(b $S), $(b $X), $(b $C), $(b $J)>(P, L);
}
SRC
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off --cuda-device-only -S -o "$out" "$src" "$@"
rm -f "$src"
