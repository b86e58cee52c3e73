#!/bin/bash
# Register / scratch / occupancy report of a scene-specialized kernel, compiled offline
# with hipcc from the same headers and options hiprtc gets (print them on the GPU with
# RTX_JIT_DUMP=1). usage: tools/jit_resource.sh "<mesh> <sec> <ext> <cnt> <jit>" [-D... options]
set -eu
cd "$(dirname "$0")/.."
read -r M S X C J <<< "$1"; shift
b() { [ "$1" = 1 ] && echo true || echo false; }
src=$(mktemp /tmp/rtx_jit_XXXX.hip)
cat > "$src" <<SRC
#include "$(pwd)/python-raytracer_amd/csrc/rtx_kernels.h"
extern "C" __global__ RTX_RENDER_BOUNDS($(b $M), $(b $S), $(b $X)) void rtx_jit_render(const rtx::KParams* __restrict__ P, const rtx::Launch L) {
  rtx::render_body<$(b $M), $(b $S), $(b $X), $(b $C), $(b $J)>(P, L);
}
SRC
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off --cuda-device-only -c -o /tmp/rtx_jit_ru.o "$src" \
  -Rpass-analysis=kernel-resource-usage "$@" 2>&1 | grep -E "Function Name|VGPRs:|AGPRs|Occupancy|ScratchSize|SGPRs Spill|VGPRs Spill|LDS Size"
rm -f "$src" /tmp/rtx_jit_ru.o
