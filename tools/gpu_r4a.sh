set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_fma.py tests/test_gpu_solver.py tests/test_gpu_cross.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r4a_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r4a_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u tools/ab_fp.py --rounds 3 > gpurun_out/r4a_abfp.log 2>&1
tail -4 gpurun_out/r4a_abfp.log
