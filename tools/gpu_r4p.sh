set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp MGX_TEST_OUT=gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_fake_rccl.py tests/test_gpu_fma.py tests/test_gpu_large.py tests/test_gpu_cross.py -k "dist or fake or partitioned or overlap or C4 or C5 or local or rccl or wcycle or block" -v --timeout 300 --timeout-method thread > gpurun_out/r4p_tests.log 2>&1
rc=$?
tail -6 gpurun_out/r4p_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u tools/ab_dist.py --parts 1,2,4,8 --overlap 0,1 --rounds 2 > gpurun_out/r4p_dist.log 2>&1 || exit $?
grep -o '"overlap": [0-9], "G": [0-9], "ms": [0-9.]*, "ms_per_rank": [0-9.]*' gpurun_out/r4p_dist.log
