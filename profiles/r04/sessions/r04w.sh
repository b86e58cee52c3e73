#!/bin/bash
# Round-4 session w: split-pass chunk size (RTX_SPLIT_RECORDS, RS: by default 2^28, 2^29, 2^30
# records of 64 B) on NovelScene1/2, interleaved twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r04w}; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for c in ns1 ns2; do
    st=5; [ $c = ns2 ] && st=2
    for r in ${RS:-268435456 536870912 1073741824}; do
      RTX_SPLIT_RECORDS=$r timeout -k 10 200 python bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline \
        > $O/${c}_r$r.$rep.json 2> $O/${c}_r$r.$rep.err || { echo FAIL $c $r; tail -5 $O/${c}_r$r.$rep.err; exit 1; }
      python -c "import json;d=json.load(open('$O/${c}_r$r.$rep.json'));print('$c records=$r.$rep', d['frame_ms'])"
    done
  done
done
echo R04W_DONE
