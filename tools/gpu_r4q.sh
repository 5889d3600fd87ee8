set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_vgen.py -v --timeout 200 --timeout-method thread > gpurun_out/r4q_tests.log 2>&1
rc=$?
tail -8 gpurun_out/r4q_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/ab_levels.py vgen=0,1 --fp fma --rounds 3 > gpurun_out/r4q_ab.log 2>&1 || exit $?
tail -3 gpurun_out/r4q_ab.log
timeout -k 10 600 bash tools/ab_libs.sh 2 --fp fma > gpurun_out/r4q_ablibs.log 2>&1 || exit $?
cat gpurun_out/r4q_ablibs.log
