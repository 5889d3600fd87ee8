set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp MGX_TEST_OUT=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -k "overlap or partitioned" -v --timeout 300 --timeout-method thread > gpurun_out/r4l_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4l_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 bash tools/ab_libs.sh 3 --fp fma > gpurun_out/r4l_ablibs.log 2>&1 || exit $?
cat gpurun_out/r4l_ablibs.log
