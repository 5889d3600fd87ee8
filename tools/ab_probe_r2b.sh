#!/bin/bash
# Round-2 probe: where the cross pass's time goes (clamped loads, no barrier, no u_pre store)
set -e
O=gpurun_out/ab_r2b; mkdir -p $O
T="timeout -k 10"
for v in libmgx libmgx_clamp libmgx_nobar libmgx_nostore libmgx; do
  MGX_LIB=hpcclassmultigridproject_amd/$v.so $T 200 python3 tools/ab_levels.py --rounds 3 >> $O/lib_$v.log 2>&1
done
