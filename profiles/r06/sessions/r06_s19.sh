# round 6 session 19: the split shade pass compiled with the scene's counts (option
# csg_shade) -- the split tests with it, then NovelScene1/2 with and without it.
O=gpurun_out/s19
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
step pytest_split 500 python -u -m pytest tests/test_gpu_split.py -m gpu -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread
for rep in 1 2; do
  for v in 1 0; do
    export RTX_CSG_SHADE=$v
    step ab_ns1_shade${v}_r$rep 300 python -u bench.py --config ns1 --steps 20 --warmup 3 --no-cpu-baseline
    [ $rep = 1 ] && step ab_ns2_shade${v}_r$rep 300 python -u bench.py --config ns2 --steps 5 --warmup 2 --no-cpu-baseline
  done
done
echo done
