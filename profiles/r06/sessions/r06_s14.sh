# round 6 session 14: occupancy bounds of the CSG-specialized split passes with their rays
# in registers (RTX_JIT_FLAGS: trace RTX_LB_SPLIT_A, shadow RTX_LB_SPLIT_B waves/SIMD).
O=gpurun_out/s14
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
  for v in a4b4 a4b5 a4b6 a5b4 a3b4 a4b3; do
    a=${v:1:1}; b=${v:3:1}
    export RTX_JIT_FLAGS="-URTX_LB_SPLIT_A -DRTX_LB_SPLIT_A=$a -URTX_LB_SPLIT_B -DRTX_LB_SPLIT_B=$b"
    step ab_ns1_${v}_r$rep 300 python -u bench.py --config ns1 --steps 20 --warmup 3 --no-cpu-baseline
    [ $rep = 1 ] && step ab_ns2_${v}_r$rep 300 python -u bench.py --config ns2 --steps 5 --warmup 2 --no-cpu-baseline
  done
done
echo done
