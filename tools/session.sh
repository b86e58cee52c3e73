#!/bin/bash
# One parametrized GPU session (replaces the per-session one-off scripts). Every GPU step
# has its own time limit, and the script stops at the first failure (pytest: exit >= 2 on
# a crash; a failing assertion stops it too unless KEEP_GOING=1).
#
#   TAG=name STEPS="tests smoke bench configs ab pmc rocprof pipeline" bash tools/session.sh
#
# tests     python -m pytest tests -m gpu (TESTS="tests/x.py ..." and KEXPR="a or b" narrow it)
# smoke     __graft_entry__.smoke()
# bench     the default bench line (N = 1, with CPU baselines unless CPU=0)
# configs   bench.py --config C for C in CONFIGS (CPU=1 adds the CPU legs to each line)
# ab        tools/ab_jitflags.sh: VARIANTS="name=jit flags;..." over CONFIGS
# abl       tools/ab_lib.sh: LIBS="name=_abl/librtx_x.so;name2=default" over CONFIGS (ROUNDS times,
#           interleaved)
# pmc       rocprofv3 counter passes (FETCH_SIZE, WRITE_SIZE, instruction mix) per CONFIGS
#           -> $OUT/pmc_<config>.json
# rocprof   rocprofv3 --kernel-trace --stats of the default bench
# rocprof_configs  the same for each of CONFIGS -> $OUT/<config>_kernel_stats.csv
# pipeline  the multi-GPU frame loop over RCCL with one rank (PIPE_CONFIGS)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-session}
mkdir -p "$OUT"
export TMPDIR=/tmp
CFGS=${CONFIGS:-tsp1080 tm1080 mr1080 dof4k}
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name"; date +%T
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -3 "$OUT/$name.log"
  return $rc
}
cpu_flag() { [ "${CPU:-1}" = 1 ] && echo "--cpu-seconds ${CPU_SECONDS:-10}" || echo "--no-cpu-baseline"; }
for s in ${STEPS:-tests smoke bench rocprof}; do
  case $s in
    tests)
      if [ -n "${KEXPR:-}" ]; then kx=(-k "$KEXPR"); else kx=(); fi
      step pytest_gpu ${TESTS_TIMEOUT:-900} python -u -m pytest ${TESTS:-tests} "${kx[@]}" -m gpu -x -q -p no:cacheprovider \
        --timeout 120 --timeout-method thread ${DURATIONS:+--durations=$DURATIONS}
      rc=$?; [ $rc -eq 0 ] || [ "${KEEP_GOING:-0}" = 1 -a $rc -eq 1 ] || exit 1 ;;
    smoke)
      step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    bench)
      step bench_default 400 python bench.py $(cpu_flag) || exit 1
      grep '^{' "$OUT/bench_default.log" > "$OUT/bench_default.json" ;;
    configs)
      for c in $CFGS; do
        pj=""; [ -f "$OUT/pmc_$c.json" ] && pj="--pmc-json $OUT/pmc_$c.json"
        st=${BSTEPS:-20}; wu=3  # (microsecond frames: 300 of them, past the tile schedule's first frames)
        case $c in tsp1080|tm1080|mr1080|blob1080) st=${BSTEPS_FAST:-300}; wu=20 ;; ns2) st=${BSTEPS_NS2:-5} ;; esac
        step bench_$c 600 python bench.py --config $c --steps $st --warmup $wu $(cpu_flag) $pj || exit 1
        grep '^{' "$OUT/bench_$c.log" > "$OUT/bench_$c.json"
      done ;;
    ab)
      CONFIGS="$CFGS" bash tools/ab_jitflags.sh > "$OUT/ab.log" 2>&1 || { tail "$OUT/ab.log"; exit 1; }
      cat "$OUT/ab.log"; mkdir -p "$OUT/ab"; cp gpurun_out/abj/*.json "$OUT/ab/" ;;
    abl)
      for r in $(seq 1 ${ROUNDS:-2}); do
        VARIANTS="$LIBS" CONFIGS="$CFGS" STEPS=${BSTEPS:-10} bash tools/ab_lib.sh > "$OUT/abl_$r.log" 2>&1 || { tail "$OUT/abl_$r.log"; exit 1; }
        cat "$OUT/abl_$r.log"; mkdir -p "$OUT/abl_$r"; cp gpurun_out/abl/*.json "$OUT/abl_$r/"
      done ;;
    pmc)
      for c in $CFGS; do
        CFG=$c TAG="${OUT#gpurun_out/}/pmc_$c" bash tools/pmc_session.sh > "$OUT/pmc_$c.log" 2>&1 || { tail "$OUT/pmc_$c.log"; exit 1; }
        python tools/pmc_summary.py "$OUT/pmc_$c" $c 6 > "$OUT/pmc_$c.json" || exit 1
        python -c "import json;d=json.load(open('$OUT/pmc_$c.json'));c=d['counters_per_dispatch'];print('$c', d['kernel'], 'WRITE_KiB', c.get('WRITE_SIZE'), 'FETCH_KiB', c.get('FETCH_SIZE'), 'hbm_B', d.get('hbm_bytes_per_launch'), 'valu/wave', d.get('valu_insts_per_wave'))"
      done ;;
    rocprof)
      step rocprof 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py \
        --steps 100 --warmup 10 --no-cpu-baseline || exit 1 ;;
    rocprof_configs)  # rocprofv3 kernel statistics of each config's bench run
      for c in $CFGS; do
        st=100; [ $c = dof4k ] && st=10; [ $c = ns1 ] && st=10; [ $c = ns2 ] && st=3
        step rocprof_$c 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$c" -o run --output-format csv -- python3 bench.py \
          --config $c --steps $st --warmup 3 --no-cpu-baseline || exit 1
        cp "$OUT/prof_$c/run_kernel_stats.csv" "$OUT/${c}_kernel_stats.csv" 2>/dev/null || \
          find "$OUT/prof_$c" -name '*kernel_stats.csv' -exec cp {} "$OUT/${c}_kernel_stats.csv" \;
      done ;;
    pipeline)
      for c in ${PIPE_CONFIGS:-tsp1080 dof4k}; do
        st=200; [ $c = dof4k ] && st=20
        step pipeline1_$c 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
          --master-port 29533 bench.py --gpus 1 --force-dist --pipeline --config $c --steps $st --warmup 5 \
          --no-cpu-baseline || exit 1
        grep '^{' "$OUT/pipeline1_$c.log" > "$OUT/pipeline1_$c.json"
      done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo SESSION_DONE
