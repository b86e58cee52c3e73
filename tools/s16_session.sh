#!/bin/bash
# Secondary-ray frames with register-held materials: GPU parity suite, then MR frame time
# with the packed (3-word) and the 4-word LDS frames, twice.
set -u
OUT=gpurun_out/${TAG:-r02s16}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
CONFIGS="mr1080" VARIANTS="packed=;words4=-URTX_FRAME_MATBITS -DRTX_FRAME_MATBITS=0;packed2=;words4b=-URTX_FRAME_MATBITS -DRTX_FRAME_MATBITS=0" bash tools/ab_jitflags.sh
