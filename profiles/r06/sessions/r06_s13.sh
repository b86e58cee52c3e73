# round 6 session 13: the CSG-specialized split passes with their rays in registers and no
# LDS stack (default) against the LDS stack (lds: a library built with RTX_CSG_RAYREG=0) and
# with the shadow pass bounded to 4 waves/SIMD (lbb4); the split tests first.
O=gpurun_out/s13
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
step pytest_split 600 python -u -m pytest tests/test_gpu_split.py -m gpu -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread --durations=8
for rep in 1 2; do
  for v in reg lds lbb4; do
    unset RTX_LIB_OVERRIDE RTX_JIT_FLAGS
    [ $v = lds ] && export RTX_LIB_OVERRIDE=$PWD/_abv/librtx_lds.so
    [ $v = lbb4 ] && export RTX_JIT_FLAGS="-URTX_LB_SPLIT_B -DRTX_LB_SPLIT_B=4"
    step ab_ns1_${v}_r$rep 300 python -u bench.py --config ns1 --steps 20 --warmup 3 --no-cpu-baseline
    step ab_ns2_${v}_r$rep 300 python -u bench.py --config ns2 --steps 5 --warmup 2 --no-cpu-baseline
  done
done
echo done
