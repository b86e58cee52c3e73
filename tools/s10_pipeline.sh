#!/bin/bash
# Multi-GPU frame loop rehearsed with one RCCL rank (FrameExchange, graph and eager) on
# the 1-GPU box: TwoSpheresPlane 1080p and DepthOfField 4K.
set -u
OUT=gpurun_out/${TAG:-r02s10}; mkdir -p $OUT
for c in ${CONFIGS:-tsp1080 dof4k}; do
  for g in "" "--no-graph"; do
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --steps 30 --warmup 5 --pipeline --no-cpu-baseline --config $c $g > $OUT/bench_pipeline1_$c$g.log 2>&1 || { tail -20 $OUT/bench_pipeline1_$c$g.log; exit 1; }
    grep '^{' $OUT/bench_pipeline1_$c$g.log > $OUT/bench_pipeline1_$c$g.json
    python3 -c "import json; d=json.load(open('$OUT/bench_pipeline1_$c$g.json')); m=d['multi_gpu']; print('$c $g', d['ms_per_step'], m['render_rgb8_ms_per_rank'], m['exchange_ms_per_group'], m['gather_to_rank0']['frame_ms'])"
  done
done
