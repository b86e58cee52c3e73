# round 6 session 16: where the CSG-specialized split passes keep their rays (option
# csg_rays: bit 0 trace, bit 1 shadow in registers, else the LDS stack), and the
# 81,920-face mesh with heavy-tile chunks of 16 for lists > 24 faces (default) against
# chunks of 32 for lists > 32 (hc32) over 300-frame runs.
O=gpurun_out/s16
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
  for v in 3 1 2 0; do
    export RTX_CSG_RAYS=$v
    step ab_ns1_rays${v}_r$rep 300 python -u bench.py --config ns1 --steps 20 --warmup 3 --no-cpu-baseline
    [ $rep = 1 ] && step ab_ns2_rays${v}_r$rep 300 python -u bench.py --config ns2 --steps 5 --warmup 2 --no-cpu-baseline
  done
done
unset RTX_CSG_RAYS
for rep in 1 2 3; do
  for v in hc32 default; do
    if [ $v = default ]; then unset RTX_LIB_OVERRIDE; else export RTX_LIB_OVERRIDE=$PWD/_abv/librtx_$v.so; fi
    step ab_blob_${v}_r$rep 200 python -u bench.py --config blob1080 --steps 300 --warmup 20 --no-cpu-baseline
  done
done
echo done
