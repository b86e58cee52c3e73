# round 6 session 12: the CSG-specialized split passes of NovelScene1 -- occupancy bounds
# (RTX_JIT_FLAGS) and their counters (instruction mix, waits, instruction cache).
O=gpurun_out/s12
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
  for v in base lbb4 lba3; do
    case $v in
      base) export RTX_JIT_FLAGS="" ;;
      lbb4) export RTX_JIT_FLAGS="-URTX_LB_SPLIT_B -DRTX_LB_SPLIT_B=4" ;;
      lba3) export RTX_JIT_FLAGS="-URTX_LB_SPLIT_A -DRTX_LB_SPLIT_A=3" ;;
    esac
    step ab_ns1_${v}_r$rep 300 python -u bench.py --config ns1 --steps 20 --warmup 3 --no-cpu-baseline
  done
done
unset RTX_JIT_FLAGS
CFG=ns1 TAG=s12/pmc_ns1 PMC_EXTRA="SQC_ICACHE_REQ SQC_ICACHE_MISSES SQC_DCACHE_REQ SQC_DCACHE_MISSES SQ_INSTS_SMEM SQ_WAVES SQ_IFETCH" \
  timeout -k 10 600 bash tools/pmc_session.sh > $O/pmc.log 2>&1
echo "pmc rc=$?" >> $O/steps.txt
echo done
