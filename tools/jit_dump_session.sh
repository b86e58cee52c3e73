#!/bin/bash
# GPU session: NovelScene1 under library variants (tools/ab_lib.sh), then the default
# configs with RTX_JIT_DUMP=1 (the specialized kernels' hiprtc options and source, for
# offline ISA work with tools/jit_offline.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r03s3}; mkdir -p $O
export TMPDIR=/tmp
if [ -n "${VARIANTS:-}" ]; then
  CONFIGS="${ABCONFIGS:-ns1}" bash tools/ab_lib.sh > $O/ab.log 2>&1; rc=$?; cat $O/ab.log; cp -r gpurun_out/abl $O/; [ $rc = 0 ] || exit 1
fi
for c in ${DUMP:-}; do
  echo "== $c"; RTX_JIT_DUMP=1 timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > $O/$c.log 2>&1 || { echo "rc=$?"; tail -5 $O/$c.log; exit 1; }
  grep '^{' $O/$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config'].get('kernel'))"
done
