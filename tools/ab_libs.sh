#!/bin/bash
# Alternate per-level timings of the default libmgx.so and every
# libmgx_<name>.so variant, ROUNDS times (separate processes, same box):
#   bash tools/ab_libs.sh [ROUNDS] [extra ab_levels args]  -> gpurun_out/ablibs/
set -e
R=${1:-3}; shift || true
O=gpurun_out/ablibs; mkdir -p $O
for r in $(seq 1 $R); do
  for lib in hpcclassmultigridproject_amd/libmgx.so hpcclassmultigridproject_amd/libmgx_*.so; do
    [ -f "$lib" ] || continue
    v=$(basename $lib .so)
    MGX_LIB=$lib timeout -k 10 120 python3 tools/ab_levels.py --rounds 2 "$@" > $O/${v}_$r.log 2>&1
    echo "$v round $r: $(grep -A1 SUMMARY $O/${v}_$r.log | tail -1)"
  done
done
