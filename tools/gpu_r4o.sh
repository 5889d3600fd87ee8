set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp MGX_TEST_OUT=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_cross.py -k "masked_cus" -v --timeout 200 --timeout-method thread > gpurun_out/r4o_tests.log 2>&1
rc=$?
tail -6 gpurun_out/r4o_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u tools/ab_levels.py xcu_edge=0,16,32,48,64 --fp fma --rounds 3 > gpurun_out/r4o_ab.log 2>&1 || exit $?
tail -6 gpurun_out/r4o_ab.log
