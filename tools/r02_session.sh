#!/bin/bash
# Round-2 GPU session: PMC passes (FETCH_SIZE / WRITE_SIZE / instruction mix) for every
# BASELINE config, then the default bench (N = 1), a bench line per config carrying its
# measured traffic, the multi-GPU frame pipeline rehearsed over RCCL with one rank, and the
# rocprofv3 kernel-trace summary of the default bench. Every GPU step has its own time
# limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r02}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -2 "$OUT/$name.log"
  return $rc
}
CFGS=${CONFIGS:-tsp1080 tm1080 mr1080 dof4k}
# PMC=0: no counter passes (the box stays fresh for timing: DOF measured 7.2 ms on a fresh
# box and 8.2-9.0 ms right after the PMC passes); the bench lines then take their traffic
# from the committed profiles/pmc_<config>.json of the same kernels
if [ "${PMC:-1}" = 1 ]; then
  for c in $CFGS; do
    CFG=$c TAG=$(basename "$OUT")/pmc_$c bash tools/pmc_session.sh > "$OUT/pmc_$c.log" 2>&1 || { tail "$OUT/pmc_$c.log"; exit 1; }
    python tools/pmc_summary.py "$OUT/pmc_$c" $c > "$OUT/pmc_$c.json" || exit 1
  done
else
  for c in $CFGS; do cp profiles/pmc_$c.json "$OUT/pmc_$c.json"; done
fi
[ "${BENCH:-1}" = 1 ] || { echo ALL_DONE; exit 0; }  # BENCH=0: counter passes only
step bench_default 300 python bench.py --pmc-json "$OUT/pmc_tsp1080.json" || exit 1
for c in $CFGS; do
  steps=50; [ $c = dof4k ] && steps=10
  step bench_$c 300 python bench.py --config $c --steps $steps --warmup 3 --no-cpu-baseline --pmc-json "$OUT/pmc_$c.json" || exit 1
done
for c in tsp1080 dof4k; do
  step bench_pipeline1_$c 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29531 bench.py --gpus 1 --steps 30 --warmup 5 --pipeline --no-cpu-baseline --config $c || exit 1
done
step rocprof 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline || exit 1
echo ALL_DONE
