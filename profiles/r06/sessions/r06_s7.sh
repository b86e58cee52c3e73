# round 6 session 7: heavy-tile chunk size 16 vs 32, three interleaved rounds on the
# 81,920-face mesh and TorusMesh (rocprofv3 kernel statistics of each blob run too).
O=gpurun_out/s7
mkdir -p $O
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc" >> $O/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc $rc)"; exit $rc; fi
}
for rep in 1 2 3; do
  for v in hc16 default; do
    if [ $v = default ]; then unset RTX_LIB_OVERRIDE; else export RTX_LIB_OVERRIDE=$PWD/_abv/librtx_$v.so; fi
    step ab_blob_${v}_r$rep 200 python -u bench.py --config blob1080 --steps 300 --warmup 20 --no-cpu-baseline
    step ab_tm_${v}_r$rep 200 python -u bench.py --config tm1080 --steps 500 --warmup 20 --no-cpu-baseline
  done
done
for v in hc16 default; do
  if [ $v = default ]; then unset RTX_LIB_OVERRIDE; else export RTX_LIB_OVERRIDE=$PWD/_abv/librtx_$v.so; fi
  step rocprof_blob_$v 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 bench.py --config blob1080 --steps 100 --warmup 10 --no-cpu-baseline
done
unset RTX_LIB_OVERRIDE
echo done
