# round 6 session 18: the CSG-specialized split passes pinned on the scene's
# counts too (jit_fixed_opts, shared with the flat kernels' specs): the whole GPU suite,
# then NovelScene1/2 and the default line.
O=gpurun_out/s18
mkdir -p $O
export TMPDIR=/tmp
TAG=s18 TESTS_TIMEOUT=1000 DURATIONS=10 STEPS="tests" bash tools/session.sh || exit 1
for c in ns1 ns2; do
  st=20; [ $c = ns2 ] && st=5
  timeout -k 10 300 python -u bench.py --config $c --steps $st --warmup 3 --no-cpu-baseline > $O/bench_$c.out 2> $O/bench_$c.err || exit 1
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_default.out 2> $O/bench_default.err || exit 1
echo done
