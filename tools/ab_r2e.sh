#!/bin/bash
set -e
O=gpurun_out/ab_r2e; mkdir -p $O
T="timeout -k 10"
for v in libmgx_base libmgx libmgx_step libmgx_pairsched libmgx_base libmgx libmgx_step libmgx_pairsched; do
  MGX_LIB=hpcclassmultigridproject_amd/$v.so $T 200 python3 tools/ab_levels.py --rounds 3 >> $O/lib_$v.log 2>&1
done
