set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp MGX_TEST_OUT=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fma.py tests/test_gpu_dist.py -k "whole_launch or recompute or partitioned or overlap or C4 or local" -v --timeout 200 --timeout-method thread > gpurun_out/r4h_tests.log 2>&1
rc=$?
tail -8 gpurun_out/r4h_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/ab_levels.py xwhole=0,1 xre=0,1 --fp fma --rounds 3 > gpurun_out/r4h_ab.log 2>&1 || exit $?
tail -5 gpurun_out/r4h_ab.log
timeout -k 10 300 python -u tools/ab_dist.py --parts 1,2,4,8 --overlap 0,1 --rounds 2 > gpurun_out/r4h_dist.log 2>&1 || exit $?
grep -o '"overlap": [0-9], "G": [0-9], "ms": [0-9.]*, "ms_per_rank": [0-9.]*' gpurun_out/r4h_dist.log
