set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp MGX_TEST_OUT=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fma.py tests/test_gpu_cross.py tests/test_gpu_fake_rccl.py tests/test_gpu_dist.py -v --timeout 300 --timeout-method thread > gpurun_out/r4d_tests.log 2>&1
rc=$?
tail -8 gpurun_out/r4d_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/ab_levels.py cross_cycle=0,1 --shape 2 --fp fma --N 16384 --L 9 --rounds 3 > gpurun_out/r4d_wcycle.log 2>&1 || exit $?
tail -3 gpurun_out/r4d_wcycle.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 2 > gpurun_out/r4d_bench.log 2>&1 || exit $?
tail -c 3000 gpurun_out/r4d_bench.log
