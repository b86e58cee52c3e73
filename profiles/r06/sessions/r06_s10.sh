# round 6 session 10: NovelScene1/2 with the split trace and shadow passes specialized on
# the scene's CSG trees (option jit_csg, rtx_trace.h namespace csg) against the precompiled
# passes (RTX_JIT_CSG=0); then the split tests with it, and rocprof kernel statistics.
O=gpurun_out/s10
mkdir -p $O
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  local t0=$(date +%s)
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc $(( $(date +%s) - t0 ))s" >> $O/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc $rc)"; tail -5 $O/$name.err; exit $rc; fi
}
for rep in 1; do
  for v in csg gen; do
    if [ $v = gen ]; then export RTX_JIT_CSG=0; else unset RTX_JIT_CSG; fi
    step ab_ns1_${v}_r$rep 400 python -u bench.py --config ns1 --steps 20 --warmup 3 --no-cpu-baseline
    step ab_ns2_${v}_r$rep 400 python -u bench.py --config ns2 --steps 5 --warmup 2 --no-cpu-baseline
  done
done
unset RTX_JIT_CSG
true \
  --timeout-method thread --durations=12
step rocprof_ns1 300 rocprofv3 --kernel-trace --stats -d $O/prof_ns1 -o run --output-format csv -- python3 bench.py \
  --config ns1 --steps 10 --warmup 3 --no-cpu-baseline
echo done
