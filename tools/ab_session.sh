#!/bin/bash
# One GPU session of A/B runs for the work-order / tile / priority / pitch knobs.
set -e
O=gpurun_out/ab; mkdir -p $O
T="timeout -k 10"
$T 300 python3 tools/ab_levels.py march_order=0,1,2,3 tile32_min_n=1073741824,2048,1024 tile_xcd=0,1 --rounds 3 > $O/knobs.log 2>&1
# variant builds (tools/build_variant.sh NAME -D...) are compared the same way:
for lib in hpcclassmultigridproject_amd/libmgx.so hpcclassmultigridproject_amd/libmgx_*.so; do
  [ -f "$lib" ] || continue
  v=$(basename $lib .so)
  MGX_LIB=$lib $T 200 python3 tools/ab_levels.py march_order=0,3 --rounds 5 > $O/lib_$v.log 2>&1
done
for pad in 0 32 48 512; do
  MGX_PITCH_PAD=$pad $T 200 python3 tools/ab_levels.py march_order=0,3 --rounds 4 > $O/pad_$pad.log 2>&1
done
$T 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cross.py tests/test_gpu_ops.py -k "work_order or context_gs or unguarded" > $O/tests.log 2>&1
