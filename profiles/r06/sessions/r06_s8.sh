# round 6 session 8: heavy-tile chunks of 16 faces for lists longer than 32 (or 24), against
# the default (chunks of 32 for lists longer than 32): the 81,920-face mesh and TorusMesh.
O=gpurun_out/s8
mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc" >> $O/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc $rc)"; exit $rc; fi
}
for rep in 1 2 3; do
  for v in hc16m32 hc16m24 default; do
    if [ $v = default ]; then unset RTX_LIB_OVERRIDE; else export RTX_LIB_OVERRIDE=$PWD/_abv/librtx_$v.so; fi
    step ab_blob_${v}_r$rep 200 python -u bench.py --config blob1080 --steps 300 --warmup 20 --no-cpu-baseline
    step ab_tm_${v}_r$rep 200 python -u bench.py --config tm1080 --steps 500 --warmup 20 --no-cpu-baseline
  done
done
unset RTX_LIB_OVERRIDE
echo done
