# round 6 session 6: the value loop's fixed cost against its length (one-rank RCCL group),
# and the heavy-tile chunk size (16 / 32 / 64 faces) on the 81,920-face mesh.
O=gpurun_out/s6
mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc" >> $O/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc $rc)"; exit $rc; fi
}
step loop_steps 240 python -u tools/loop_steps_probe.py tsp1080
for rep in 1 2; do
  for v in hc16 hc64 default; do
    if [ $v = default ]; then unset RTX_LIB_OVERRIDE; else export RTX_LIB_OVERRIDE=$PWD/_abv/librtx_$v.so; fi
    step ab_${v}_r$rep 200 python -u bench.py --config blob1080 --steps 200 --warmup 20 --no-cpu-baseline
  done
done
unset RTX_LIB_OVERRIDE
echo done
