set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r4c_tests.log 2>&1
rc=$?
tail -12 gpurun_out/r4c_tests.log
exit $rc
