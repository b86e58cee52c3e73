#!/bin/bash
# Usage: TAG=name CONFIGS="tsp1080 ..." CENSUS="tm1080" bash tools/gpu_check.sh
# parity suite + selected bench configs (+ census)
mkdir -p gpurun_out/${TAG}
timeout -k 10 400 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/$TAG/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/$TAG/pytest.log; [ $rc -eq 0 ] || exit 1
for c in ${CONFIGS:-tsp1080}; do
  timeout -k 10 120 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$TAG/bench_$c.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/$TAG/bench_$c.log') if l.startswith('{')][0]); print('$c frame_ms', d['frame_ms'])"
done
for c in ${CENSUS:-}; do timeout -k 10 120 python tools/census.py --config $c 2>&1 | grep casts; done
