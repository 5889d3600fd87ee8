#!/bin/bash
# Round-4 closing GPU call after the row-block generator: its tests, the
# virtual-rank A/B, the profiles of the final sources, smoke and the bench.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_vgen.py tests/test_gpu_dist.py tests/test_gpu_fake_rccl.py > $O/vg_dist_tests.log 2>&1 || exit 11
tail -2 $O/vg_dist_tests.log
timeout -k 10 300 python -u tools/ab_dist.py --parts 1,8 --overlap 1 --knob vgen=0,1 > $O/vg_dist_ab.log 2>&1 || exit 12
timeout -k 10 700 bash tools/profile_round.sh r4 > $O/prof_r4.log 2>&1 || exit 13
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/r4_smoke.log 2>&1 || exit 14
timeout -k 10 400 python -u bench.py > $O/r4_bench_final.log 2>&1 || exit 15
grep '^{' $O/r4_bench_final.log | tail -1 | cut -c1-200
