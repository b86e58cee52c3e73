#!/bin/bash
# Round-4 session w: split-pass chunk size (RTX_SPLIT_RECORDS: 2^26 default, 2^27, 2^28
# records of 64 B) on NovelScene1/2, interleaved twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04w; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for c in ns1 ns2; do
    st=5; [ $c = ns2 ] && st=2
    for r in 67108864 134217728 268435456; do
      RTX_SPLIT_RECORDS=$r timeout -k 10 200 python bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline \
        > $O/${c}_r$r.$rep.json 2> $O/${c}_r$r.$rep.err || { echo FAIL $c $r; tail -5 $O/${c}_r$r.$rep.err; exit 1; }
      python -c "import json;d=json.load(open('$O/${c}_r$r.$rep.json'));print('$c records=$r.$rep', d['frame_ms'])"
    done
  done
done
echo R04W_DONE
