#!/bin/bash
# cross pass in step pairs: parity + per-level timing
set -e
O=gpurun_out/ab_r2d; mkdir -p $O
T="timeout -k 10"
$T 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cross.py tests/test_gpu_solver.py tests/test_gpu_dist.py > $O/tests.log 2>&1
$T 200 python3 tools/ab_levels.py --rounds 5 > $O/levels.log 2>&1
