#!/bin/bash
# Round-2 probe: branch-free cross pass (stores unconditional, exit check per unrolled body)
set -e
O=gpurun_out/ab_r2c; mkdir -p $O
T="timeout -k 10"
for v in libmgx libmgx_free libmgx_freenobar libmgx_clamp libmgx; do
  MGX_LIB=hpcclassmultigridproject_amd/$v.so $T 200 python3 tools/ab_levels.py --rounds 3 >> $O/lib_$v.log 2>&1
done
