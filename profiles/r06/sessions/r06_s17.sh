# round 6 session 17: NovelScene1's CSG-specialized split passes also pinned on the scene's
# counts (RTX_JIT_FLAGS: object / light counts, light kinds, pow bits -- F1 -- and the
# camera's sample counts -- F2), as the flat scenes' specialized kernels are.
O=gpurun_out/s17
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
F1="-DRTX_FIXED_COUNTS -DRTX_FIXED_NP=1 -DRTX_FIXED_NS=0 -DRTX_FIXED_NB=2 -DRTX_FIXED_NM=0 -DRTX_FIXED_NL=2 -DRTX_FIXED_LDIR=3u -DRTX_FIXED_POWBITS=7"
F2="$F1 -DRTX_FIXED_SAMPLES -DRTX_FIXED_NDOF=1 -DRTX_FIXED_NAA=32 -DRTX_FIXED_NTIMES=1 -DRTX_FIXED_STATIC=0 -DRTX_FIXED_DIVPOW2=1 -DRTX_FIXED_JMODE=1"
for rep in 1 2; do
  for v in base f1 f2; do
    case $v in base) export RTX_JIT_FLAGS="" ;; f1) export RTX_JIT_FLAGS="$F1" ;; f2) export RTX_JIT_FLAGS="$F2" ;; esac
    step ab_ns1_${v}_r$rep 300 python -u bench.py --config ns1 --steps 20 --warmup 3 --no-cpu-baseline
  done
done
echo done
