#!/bin/bash
# Round-2 probe: speed-of-light variants of the cross pass (divneg, nocoef)
set -e
O=gpurun_out/ab_r2a; mkdir -p $O
T="timeout -k 10"
MGX_LIB=hpcclassmultigridproject_amd/libmgx_divneg.so $T 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_solver.py tests/test_gpu_cross.py tests/test_gpu_ops.py > $O/divneg_tests.log 2>&1
for v in libmgx libmgx_divneg libmgx_nocoef libmgx_nocoefdiv libmgx libmgx_divneg; do
  MGX_LIB=hpcclassmultigridproject_amd/$v.so $T 200 python3 tools/ab_levels.py --rounds 3 >> $O/lib_$v.log 2>&1
done
