#!/bin/bash
# HBM traffic of one frame with the acceleration tables switched off one at a time:
# FETCH_SIZE and WRITE_SIZE passes (rocprofv3 --pmc, one counter each) per variant, each
# summarised by tools/pmc_summary.py -> gpurun_out/$TAG/traffic_<config>_<variant>.json.
#   TAG=name ITEMS="tm1080:base= tm1080:bins=RTX_BINS=0 ..." bash tools/traffic_itemize.sh
# (a variant's value is VAR=VALUE env settings separated by ',', empty for the defaults)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-traffic}
mkdir -p "$OUT"
export TMPDIR=/tmp
for it in ${ITEMS:-tm1080:base=}; do
  cfg=${it%%:*}; rest=${it#*:}; name=${rest%%=*}; envs=${rest#*=}
  d="$OUT/t_${cfg}_$name"
  for c in FETCH_SIZE WRITE_SIZE; do
    ( IFS=','; for e in $envs; do [ -n "$e" ] && export "$e"; done
      timeout -k 10 240 rocprofv3 --kernel-trace --pmc $c -d "$d/p_$c" -o pmc --output-format csv -- \
        python3 tools/prof_driver.py --config $cfg --iters 5 > "$d.$c.log" 2>&1 )
    rc=$?; [ $rc -eq 0 ] || { echo "$cfg $name $c rc=$rc"; tail -20 "$d.$c.log"; exit $rc; }
  done
  python tools/pmc_summary.py "$d" $cfg > "$OUT/traffic_${cfg}_$name.json" || exit 1
  python -c "import json;d=json.load(open('$OUT/traffic_${cfg}_$name.json'));c=d['counters_per_dispatch'];print('$cfg $name', 'fetch_MB %.2f write_MB %.2f hbm_MB %.2f' % (2*c['FETCH_SIZE']*1024/1e6, c['WRITE_SIZE']*1024/1e6, d['hbm_bytes_per_launch']/1e6))"
done
echo TRAFFIC_DONE
