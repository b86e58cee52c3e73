#!/bin/bash
# Counter collection for the render kernel: one rocprofv3 pass per counter group
# (--pmc passes use --kernel-trace only; never combined with sys/runtime traces).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
CFG=${CFG:-tsp1080}
# PMC_EXTRA="group;group": more passes after the default ones (e.g. the VALU mix)
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/p$i" -o pmc --output-format csv -- python3 tools/prof_driver.py --config $CFG --iters 5 > "$OUT/p$i.log" 2>&1
  rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$OUT/p$i.log"; exit $rc; }
done <<GROUPS
${PMC_GROUPS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE}
$(echo "${PMC_EXTRA:-}" | tr ';' '\n')
GROUPS
echo PMC_DONE
