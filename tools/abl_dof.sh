#!/bin/bash
# DOF/TSP cost probes through the scene-specialized kernels only (the library is used as
# built; JFLAGS_<n> go to hiprtc). Experiment only: variants != 0 are not parity-correct.
export FLAGS_0=none FLAGS_4=none FLAGS_nb=none
export JFLAGS_4=-DRTX_ABLATE=4 JFLAGS_nb=-DRTX_FIXED_NB=0
TAG=${TAG:-abl19} VARIANTS="${VARIANTS:-0 4 nb}" CONFIGS="${CONFIGS:-dof4k tsp1080 mr1080}" bash tools/ablate.sh
