# round 6 session 15: the CSG-specialized split passes -- rays in registers (default) with
# occupancy bounds trace A / shadow B waves/SIMD (aXbY, RTX_JIT_FLAGS) against the LDS ray
# stack (lds: a library built with RTX_CSG_RAYREG=0, its own bounds 4 / 1).
O=gpurun_out/s15
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
for rep in 1 2; do
  for v in a4b4 lds a3b4 a3b3 a4b3; do
    unset RTX_LIB_OVERRIDE RTX_JIT_FLAGS
    if [ $v = lds ]; then export RTX_LIB_OVERRIDE=$PWD/_abv/librtx_lds.so
    else a=${v:1:1}; b=${v:3:1}; export RTX_JIT_FLAGS="-URTX_LB_SPLIT_A -DRTX_LB_SPLIT_A=$a -URTX_LB_SPLIT_B -DRTX_LB_SPLIT_B=$b"; fi
    step ab_ns1_${v}_r$rep 300 python -u bench.py --config ns1 --steps 20 --warmup 3 --no-cpu-baseline
    [ $rep = 1 ] && step ab_ns2_${v}_r$rep 300 python -u bench.py --config ns2 --steps 5 --warmup 2 --no-cpu-baseline
  done
done
echo done
