# round 6 session 11: the hierarchy tests with the split passes specialized on the CSG
# trees (jit_csg, the default now): exactness and how long their compiles take.
O=gpurun_out/s11
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py tests/test_gpu_refvectors.py \
  -k "Novel or hier or Hier or csg or CSG or split or specialized" -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  --durations=25 > $O/pytest_csg.out 2> $O/pytest_csg.err
echo "pytest rc=$?"
tail -40 $O/pytest_csg.out
