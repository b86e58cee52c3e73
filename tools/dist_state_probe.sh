#!/bin/bash
# Does process state change the kernel time? The default N = 1 bench, the same bench inside
# a one-rank torch.distributed (RCCL) process, and again the default (TAG, CFG).
set -u
O=gpurun_out/${TAG:-dist_probe}; mkdir -p $O
export TMPDIR=/tmp
c=${CFG:-tsp1080}
j() { python -c "import json,sys; d=json.loads([l for l in open('$1') if l.startswith('{')][0]); print('$2', d['frame_ms'], d['ms_per_step'], d['kernel'])"; }
timeout -k 10 200 python bench.py --config $c --steps 200 --warmup 10 --no-cpu-baseline > $O/plain1.log 2>&1 || exit 1; j $O/plain1.log plain1
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 \
  bench.py --gpus 1 --force-dist --config $c --steps 200 --warmup 10 --no-cpu-baseline > $O/dist.log 2>&1 || exit 1; j $O/dist.log dist
timeout -k 10 200 python bench.py --config $c --steps 200 --warmup 10 --no-cpu-baseline > $O/plain2.log 2>&1 || exit 1; j $O/plain2.log plain2
