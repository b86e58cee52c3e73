#!/bin/bash
# PMC pass (instruction mix + cycles) for ablation variants: VARIANTS / FLAGS_<name> as in ablate.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-pmcv}
mkdir -p "$OUT" /tmp/rtx_ablate
export TMPDIR=/tmp
for n in ${VARIANTS:-0}; do
  fl_var="FLAGS_$n"; fl="${!fl_var:--DRTX_TOOLS_BUILD -DRTX_ABLATE=$n}"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared $fl \
    -o /tmp/rtx_ablate/librtx_$n.so python-raytracer_amd/csrc/rtx_api.hip python-raytracer_amd/csrc/rtx_kern_ext_m0.hip python-raytracer_amd/csrc/rtx_kern_ext_m1.hip -lhiprtc || exit 1
  RTX_LIB_OVERRIDE=/tmp/rtx_ablate/librtx_$n.so timeout -k 10 240 rocprofv3 --kernel-trace \
    --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM \
    -d "$OUT/$n" -o pmc --output-format csv -- python3 tools/prof_driver.py --config ${CFG:-tsp1080} --iters 5 > "$OUT/$n.log" 2>&1 || exit 1
  mkdir -p "$OUT/$n/p1" && mv "$OUT/$n"/*.csv "$OUT/$n/p1/" 2>/dev/null
  echo "variant $n: $(python3 tools/pmc_summary.py "$OUT/$n" x | python3 -c "
import json,sys; d=json.load(sys.stdin); c=d['counters_per_dispatch']; w=c['SQ_WAVES']
print('valu/w %.0f salu/w %.0f smem/w %.1f wavecyc/w %.0f waitany/w %.0f activevalu/w %.0f' % (c['SQ_INSTS_VALU']/w, c['SQ_INSTS_SALU']/w, c['SQ_INSTS_SMEM']/w, c['SQ_WAVE_CYCLES']/w, c['SQ_WAIT_ANY']/w, c['SQ_ACTIVE_INST_VALU']/w))")"
done
