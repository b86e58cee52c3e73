#!/bin/bash
# Per-kernel VGPR / scratch / occupancy / SGPR-spill summary of a .hip file.
# usage: tools/resource_usage.sh file.hip [extra hipcc flags...]
f=$1; shift
hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -Rpass-analysis=kernel-resource-usage \
  -o /tmp/ru_$$.so "$f" "$@" 2>&1 | python3 -c "
import sys,re
cur=None; rows={}
for l in sys.stdin:
    m=re.search(r'Function Name: (\S+)',l)
    if m: cur=m.group(1); rows[cur]={}; continue
    m=re.search(r'remark:\s+(VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|SGPRs Spill|TotalSGPRs): (\d+)',l)
    if cur and m: rows[cur][m.group(1).split()[0]]=m.group(2)
for k,v in rows.items():
    print('%-60s VGPR %4s scratch %5s occ %s sgpr %4s spill %4s' % (k[:60], v.get('VGPRs'), v.get('ScratchSize'), v.get('Occupancy'), v.get('TotalSGPRs'), v.get('SGPRs')))
"
rm -f /tmp/ru_$$.so
