set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp MGX_TEST_OUT=gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_gpu_fma.py tests/test_gpu_cross.py tests/test_gpu_fake_rccl.py tests/test_gpu_dist.py tests/test_gpu_driver.py -v --timeout 300 --timeout-method thread > gpurun_out/r4f_tests.log 2>&1
rc=$?
tail -8 gpurun_out/r4f_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u tools/rccl_selfcheck1.py > gpurun_out/r4f_rccl1.log 2>&1 || exit $?
tail -c 600 gpurun_out/r4f_rccl1.log
timeout -k 10 300 python -u tools/ab_fp.py --rounds 3 > gpurun_out/r4f_abfp.log 2>&1 || exit $?
tail -4 gpurun_out/r4f_abfp.log
timeout -k 10 200 python -u tools/step_time.py --fp fma --key step_cross --values 0,1 > gpurun_out/r4f_step_fma.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/step_time.py --fp bitwise --key step_cross --values 0,1 > gpurun_out/r4f_step_bit.log 2>&1 || exit $?
tail -2 gpurun_out/r4f_step_fma.log gpurun_out/r4f_step_bit.log
timeout -k 10 300 python -u tools/ab_dist.py --parts 1,2,4,8 --overlap 0,1 --rounds 2 > gpurun_out/r4f_dist.log 2>&1 || exit $?
grep -o '"overlap": [0-9], "G": [0-9], "ms": [0-9.]*, "ms_per_rank": [0-9.]*' gpurun_out/r4f_dist.log
timeout -k 10 500 bash tools/ab_libs.sh 3 --fp fma > gpurun_out/r4f_ablibs.log 2>&1 || exit $?
tail -12 gpurun_out/r4f_ablibs.log
