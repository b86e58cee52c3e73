#!/bin/bash
# Frame stack split (8 LDS levels + private deep levels): GPU parity suite, then MR frame
# time with 10, 8 and 6 LDS levels, twice.
set -u
OUT=gpurun_out/${TAG:-r02s19}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit 1
CONFIGS="mr1080" VARIANTS="l8=;l10=-URTX_FRAME_LDS_LEVELS -DRTX_FRAME_LDS_LEVELS=10;l6=-URTX_FRAME_LDS_LEVELS -DRTX_FRAME_LDS_LEVELS=6;l8b=;l10b=-URTX_FRAME_LDS_LEVELS -DRTX_FRAME_LDS_LEVELS=10" bash tools/ab_jitflags.sh
