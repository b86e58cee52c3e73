# round 6 session 9: the CSG ray/point stack in LDS per lane, 9 hlevels - 3 words (default:
# the deepest level holds a ray only) against 9 hlevels (hsold, the round-5 size) and
# 9 (hlevels - 1) with the world ray in registers (hsr0): hierarchy parity with each, then
# NovelScene1/2 frame times (three interleaved rounds) and a scalar-cache counter pass.
O=gpurun_out/s9
mkdir -p $O
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc" >> $O/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc $rc)"; exit $rc; fi
}
HK="Novel or hier or Hier or csg or CSG or split"
step pytest_default 400 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py tests/test_gpu_refvectors.py \
  -k "$HK" -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
RTX_LIB_OVERRIDE=$PWD/_abv/librtx_hsr0.so step pytest_hsr0 400 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py \
  tests/test_gpu_refvectors.py -k "$HK" -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
for rep in 1 2 3; do
  for v in hsold hsr0 default; do
    if [ $v = default ]; then unset RTX_LIB_OVERRIDE; else export RTX_LIB_OVERRIDE=$PWD/_abv/librtx_$v.so; fi
    step ab_ns1_${v}_r$rep 200 python -u bench.py --config ns1 --steps 20 --warmup 3 --no-cpu-baseline
    step ab_ns2_${v}_r$rep 200 python -u bench.py --config ns2 --steps 5 --warmup 2 --no-cpu-baseline
  done
done
unset RTX_LIB_OVERRIDE
mkdir -p $O/sqc
step sqc_ns1 90 rocprofv3 --kernel-trace --pmc SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_ICACHE_REQ SQC_ICACHE_MISSES SQ_INSTS_SMEM SQ_WAVES \
  -d $O/sqc -o pmc --output-format csv -- python3 tools/prof_driver.py --config ns1 --iters 3
echo done
