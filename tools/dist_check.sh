#!/bin/bash
# Exercise the multi-rank bench path (RCCL init, barrier, all_reduce, the frame pipeline's gather) with
# one rank on a one-GPU box, and the CLI's distributed row-block render.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-dist}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 1 --steps 10 --warmup 3 --pipeline --no-cpu-baseline > "$OUT/bench_dist1.log" 2>&1 || { tail -30 "$OUT/bench_dist1.log"; exit 1; }
grep '^{' "$OUT/bench_dist1.log"
cd python-raytracer_amd && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 \
  -m rtx.main --infile ../tests/golden/tsp_small.json --outfile ../$OUT/tsp_dist.png --distributed --quiet > ../$OUT/cli_dist.log 2>&1 || { tail -30 ../$OUT/cli_dist.log; exit 1; }
python -m rtx.main --infile ../tests/golden/tsp_small.json --outfile ../$OUT/tsp_single.png --quiet > ../$OUT/cli_single.log 2>&1 || { tail -30 ../$OUT/cli_single.log; exit 1; }
python - <<PY
import numpy as np
from PIL import Image
a = np.asarray(Image.open("../$OUT/tsp_dist.png")); b = np.asarray(Image.open("../$OUT/tsp_single.png"))
print("cli distributed == single:", a.shape, bool((a == b).all()))
PY
