set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp MGX_TEST_OUT=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_fma.py -k "16384 or cycles_vs or tiles_equal" -v --timeout 300 --timeout-method thread > gpurun_out/r4n_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r4n_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 700 bash tools/ab_libs.sh 3 --fp fma > gpurun_out/r4n_ablibs.log 2>&1 || exit $?
cat gpurun_out/r4n_ablibs.log
